# k_signal_tc with the flags polled one lane per flag (in-tree
# build) vs the previous build (ab/libcsmom_base.so) on C2; parity tests; phase stamps.
set -e
mkdir -p gpurun_out/poll
timeout -k 10 300 python -u -m pytest tests/test_gpu_signal_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/poll/tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/poll/new_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/poll/base_$rep.json 2>/dev/null
done
CSMOM_LIB=$PWD/ab/libcsmom_tct.so timeout -k 10 100 python -u scripts/exp_tc_phases.py 12 > gpurun_out/poll/phases_c12.json 2>&1
