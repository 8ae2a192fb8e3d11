set -e
mkdir -p gpurun_out/c5ls
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5ls/first_$i.json 2> gpurun_out/c5ls/first_$i.err
  CSMOM_LIB=ab/libcsmom_mbcnt.so timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5ls/mbcnt_$i.json 2> gpurun_out/c5ls/mbcnt_$i.err
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --tune ls_opt=0 > gpurun_out/c5ls/off_$i.json 2> gpurun_out/c5ls/off_$i.err
done
