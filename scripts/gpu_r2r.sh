#!/bin/bash
# turnover general rows: work list vs full grid (tests, C5 / C3 A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_portfolio.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_tl.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_tl.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune turn_list=$v > gpurun_out/bench_c5_tl.log 2>&1
  rc=$?; echo "[c5 turn_list=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_tl.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --tune turn_list=$v > gpurun_out/bench_c3_tl.log 2>&1
  rc=$?; echo "[c3 turn_list=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_tl.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
