#!/bin/bash
# GPU tests, then the C5 and C3 sweep bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_round.sh tests || exit $?
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q "failed" gpurun_out/gpu_tests.log || exit 1
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5.log
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c3.log
