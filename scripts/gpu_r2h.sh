#!/bin/bash
# k_signal: raw buffer loads (padding rows out of range) vs clamped re-loads; scan / store ablations (C4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_signal2.py 100000 pair_ids_bwf4_nbuf2,pair_ids_bwf4_nbuf2_nt,pair_ids_bwf4_nbuf2_bl,pair_ids_bwf4_nbuf2_bl_nt,noscanst_ids > gpurun_out/exp_signal_bl.log 2>&1
rc=$?; tail -1 gpurun_out/exp_signal_bl.log; [ $rc -eq 0 ] || exit $rc
