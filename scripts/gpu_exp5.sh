#!/bin/bash
# Day-batch signal kernel: parity, A/B; drop-in turnover / ingestion tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_features.py tests/test_gpu_shards_api.py tests/test_panel.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_exp5_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_exp5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 250 python -u scripts/exp_signal2.py 100000 pair_ids,pair_ids_db16,pair_ids_db20,pair_ids_db21,pair_ids_d24 > gpurun_out/exp_signal_db.log 2>&1
rc=$?; tail -1 gpurun_out/exp_signal_db.log; [ $rc -eq 0 ] || exit $rc
echo exp5 done
