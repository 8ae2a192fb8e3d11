#!/bin/bash
# k_signal: barrier-free multi-wave workgroups (adjacent column slices) vs one wave per block
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_signal2.py 100000 pair_ids,pair_ids_bwf4_nbuf3,pair_ids_bwf3_nbuf3,pair_ids_bwf3_nbuf2,pair_ids_bwf2_nbuf2,pair_ids_bwf4_nbuf2,pair_ids_bwf4 > gpurun_out/exp_signal_bwf.log 2>&1
rc=$?; tail -1 gpurun_out/exp_signal_bwf.log; [ $rc -eq 0 ] || exit $rc
