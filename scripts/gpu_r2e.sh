#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2e.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_r2e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/exp_dec_merge.py > gpurun_out/exp_dec_merge.log 2>&1
rc=$?; tail -1 gpurun_out/exp_dec_merge.log; [ $rc -eq 0 ] || exit $rc
for v in "" "--tune dec_merge=0"; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 8 $v > gpurun_out/bench_c4_r2e.log 2>&1
  rc=$?; echo "[$v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c4_r2e.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
