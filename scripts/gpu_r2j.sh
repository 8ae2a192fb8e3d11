#!/bin/bash
# narrow id path (sweeps) tests, full GPU suite, smoke, C4 + C5 benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_pipeline.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_pipeline.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c4.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
