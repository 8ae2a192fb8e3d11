# k_signal_tc with 256-thread workgroups (ab/libcsmom_t256.so: two per CU, 4 waves reduce months,
# all 4 fold and scan) at 16-24 chunks vs the shipped 512-thread build at its default 12 (C2).
set -e
mkdir -p gpurun_out/t256
CSMOM_LIB=$PWD/ab/libcsmom_t256.so timeout -k 10 300 python -u -m pytest tests/test_gpu_signal_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t256/tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/t256/base_$rep.json 2>/dev/null
  for C in 24 22 20 16; do
    CSMOM_LIB=$PWD/ab/libcsmom_t256.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 --chunks $C > gpurun_out/t256/c${C}_$rep.json 2>/dev/null
  done
done
