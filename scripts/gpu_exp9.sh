#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_exp9_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_exp9_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 2 0 16 > gpurun_out/dec_phases9.log 2>&1
rc=$?; tail -1 gpurun_out/dec_phases9.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 8 > gpurun_out/bench_c4_9.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c4_9.log; [ $rc -eq 0 ] || exit $rc
