#!/bin/bash
# legs label sort with the whole row in registers: tests + C5 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ab.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_ab.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_ab.log 2>&1
  rc=$?; echo "[c5 $r]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_ab.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
