#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread -k day_batch > gpurun_out/gpu_exp6_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_exp6_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 250 python -u scripts/exp_signal2.py 100000 pair_ids,pair_ids_db16,pair_ids_db20,pair_ids_db21 > gpurun_out/exp_signal_db2.log 2>&1
rc=$?; tail -1 gpurun_out/exp_signal_db2.log; [ $rc -eq 0 ] || exit $rc
