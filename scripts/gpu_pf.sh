#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_features.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pf.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_pf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c3.log | cut -c1-200; grep -o '"stage_ms[^}]*}' gpurun_out/bench_c3.log; grep -o '"cpu_baseline.*' gpurun_out/bench_c3.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c5.log | cut -c1-200; grep -o '"stage_ms[^}]*}' gpurun_out/bench_c5.log; grep -o '"cpu_baseline.*' gpurun_out/bench_c5.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
