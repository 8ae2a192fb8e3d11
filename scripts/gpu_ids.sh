#!/bin/bash
# Bucket-id pipeline: its parity tests, the full GPU suite, C4 bench with and without ids.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pipe_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_pipe_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c4_ids.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c4_ids.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ids --match-dates 8 > gpurun_out/bench_c4_noids.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c4_noids.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo ids done
