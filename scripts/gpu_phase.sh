#!/bin/bash
# Decile-kernel phase timings (wall-clock marks) at C4: default kernel vs the id kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for a in "0 0 0" "2 0 0" "2 0 1" "2 0 0 58"; do
  timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 $a >> gpurun_out/dec_phases.log 2>&1 || exit $?
done
tail -4 gpurun_out/dec_phases.log
