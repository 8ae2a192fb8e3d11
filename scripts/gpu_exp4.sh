#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_split2.py > gpurun_out/exp_split2.log 2>&1
rc=$?; tail -1 gpurun_out/exp_split2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "signal or fused" > gpurun_out/gpu_sig_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_sig_tests.log; [ $rc -eq 0 ] || exit $rc
