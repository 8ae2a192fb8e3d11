#!/bin/bash
# full GPU suite + C4 bench A/B (merged decile pass, 4-wave signal blocks)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r2d.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_r2d.log; [ $rc -eq 0 ] || exit $rc
for v in "" "--tune dec_merge=0" "--tune signal_bwf=1 --tune dec_merge=0" ""; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 8 $v > gpurun_out/bench_c4_r2d.log 2>&1
  rc=$?; echo "[$v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c4_r2d.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
