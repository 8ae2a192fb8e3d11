#!/bin/bash
# Round 2 re-entry: smoke, C4 bench on HEAD, rocprofv3 stats + PMC passes into profiles tag r02
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c4.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r02 c4 || exit $?

timeout -k 10 200 python -u scripts/exp_overlap.py 1,4 > gpurun_out/exp_overlap.log 2>&1
rc=$?; tail -1 gpurun_out/exp_overlap.log; [ $rc -eq 0 ] || exit $rc
echo done
timeout -k 10 120 python -u scripts/mb/mb2.py > gpurun_out/mb2.log 2>&1
rc=$?; tail -1 gpurun_out/mb2.log; [ $rc -eq 0 ] || exit $rc
