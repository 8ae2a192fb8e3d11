#!/bin/bash
# turnover general rows via a work list: tests + C5 / C3 benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_fullsize.py tests/test_gpu_features.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_turn.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_turn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_turn.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_turn.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_c3_turn.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c3_turn.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
