# k_signal_tc's compile-time-J scan step branch-free (ab/libcsmom_sel.so) vs branchy (in-tree)
set -e
mkdir -p gpurun_out/sel
CSMOM_LIB=$PWD/ab/libcsmom_sel.so timeout -k 10 300 python -u -m pytest tests/test_gpu_signal_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sel/tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/sel/base_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_sel.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/sel/sel_$rep.json 2>/dev/null
done
