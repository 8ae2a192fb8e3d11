#!/bin/bash
# narrow PRE decile kernel: CAP 512, labels-only merged pass at 8 workgroups per CU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_portfolio.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_s.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_s.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_s.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_s.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
