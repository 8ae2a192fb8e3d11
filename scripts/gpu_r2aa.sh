#!/bin/bash
# general turnover rows skip the label loads of ages empty on both legs: tests + C5 / C3 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_aa.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_aa.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_aa.log 2>&1
  rc=$?; echo "[c5 $r]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_aa.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3_aa.log 2>&1
rc=$?; echo "[c3]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_aa.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
