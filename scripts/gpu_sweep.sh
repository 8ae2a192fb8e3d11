#!/bin/bash
# GPU session: full -m gpu suite, then the C3 / C5 sweep benches and the default C4 bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/bench_c3.log 2>&1
rc=$?; tail -2 gpurun_out/bench_c3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; tail -2 gpurun_out/bench_c5.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-assets 20000 > gpurun_out/bench_c4.log 2>&1
rc=$?; tail -1 gpurun_out/bench_c4.log; [ $rc -eq 0 ] || exit $rc
echo done
