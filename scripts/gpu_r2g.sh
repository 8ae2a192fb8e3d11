#!/bin/bash
# k_signal: register-ring scan (signal_rr) vs LDS ring; no-scan / no-store ablations (C4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_signal2.py 100000 pair_ids_bwf4_nbuf2,pair_ids_bwf4_nbuf2_rr,pair_ids_bwf4_nbuf3_rr,pair_ids_bwf4_nbuf4_rr,pair_ids_bwf1_nbuf2_rr,pair_ids_bwf4_nbuf3,noscan_ids > gpurun_out/exp_signal_rr.log 2>&1
rc=$?; tail -1 gpurun_out/exp_signal_rr.log; [ $rc -eq 0 ] || exit $rc
