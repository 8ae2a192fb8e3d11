#!/bin/bash
# full GPU suite + smoke + C4 bench on the buffer-load default
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c4.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
