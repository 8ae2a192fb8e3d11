#!/bin/bash
# one-wave-per-row legs label sort: tests + C5 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_t.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_t.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune sort_wave=$v > gpurun_out/bench_c5_t.log 2>&1
  rc=$?; echo "[sort_wave=$v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_t.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
