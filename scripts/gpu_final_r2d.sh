#!/bin/bash
# Round-2 closing check D: full GPU suite + smoke on the final code, then the sweep profiles
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile_sweep.sh r02 c5 || exit $?
bash scripts/profile_sweep.sh r02 c3 || exit $?
echo final_d done
