set -e
mkdir -p gpurun_out/c5gi
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5gi/gi5_$i.json 2> gpurun_out/c5gi/gi5_$i.err
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --tune turn_gi=0 > gpurun_out/c5gi/gi0_$i.json 2> gpurun_out/c5gi/gi0_$i.err
  CSMOM_LIB=ab/libcsmom_gi3.so timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5gi/gi3_$i.json 2> gpurun_out/c5gi/gi3_$i.err
done
