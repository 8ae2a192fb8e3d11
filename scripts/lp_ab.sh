set -e
mkdir -p gpurun_out/lp
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-oracle-mom --match-dates 4 > gpurun_out/lp/c4new_$i.json 2> gpurun_out/lp/c4new_$i.err
  CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-oracle-mom --match-dates 4 > gpurun_out/lp/c4base_$i.json 2> gpurun_out/lp/c4base_$i.err
done
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lp/c5new_$i.json 2> gpurun_out/lp/c5new_$i.err
  CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/lp/c5base_$i.json 2> gpurun_out/lp/c5base_$i.err
done
