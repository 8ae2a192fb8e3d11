#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pf.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_pf.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c3.log | cut -c1-300; grep -o '"stage_ms[^}]*}' gpurun_out/bench_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --panels 200 > gpurun_out/prof_c5.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof_c5.log; exit $rc; }
grep -o '"stage_ms[^}]*}' gpurun_out/prof_c5.log
find gpurun_out/prof_c5 -name "*kernel_stats.csv" -exec head -9 {} \; | cut -c1-200
