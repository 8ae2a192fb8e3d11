# k_signal_tc variants against the shipped build on C2 (same box, interleaved):
# ab/libcsmom_tc1024.so = 1024 threads per workgroup (16 waves reduce months).
set -e
mkdir -p gpurun_out/tcv
CSMOM_LIB=$PWD/ab/libcsmom_tc1024.so timeout -k 10 300 python -u -m pytest tests/test_gpu_signal_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tcv/tests.log 2>&1
for rep in 1 2; do
for C in 13 12 10; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 --chunks $C > gpurun_out/tcv/base_c${C}_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_tc1024.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 --chunks $C > gpurun_out/tcv/t1024_c${C}_$rep.json 2>/dev/null
done
done
