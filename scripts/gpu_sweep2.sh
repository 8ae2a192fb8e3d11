#!/bin/bash
# GPU tests, then the C5 sweep bench with the per-J scans and with the multi-J scan.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "momentum_multi or multi_J or fixture or decile_cases" > gpurun_out/gpu_tests_mj.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_mj.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_multij.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_multij.log
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --per-j-scan > gpurun_out/bench_c5_perj.log 2>&1 || exit $?
grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_perj.log
