#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_overlap.py 1,4 > gpurun_out/exp_overlap.log 2>&1
rc=$?; tail -1 gpurun_out/exp_overlap.log; [ $rc -eq 0 ] || exit $rc
