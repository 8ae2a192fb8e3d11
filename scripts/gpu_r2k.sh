#!/bin/bash
# C5 sweep: decile ids vs streaming; C3; CU-masked overlap experiment (C4)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "" "--no-decile-ids"; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline $v > gpurun_out/bench_c5_ids.log 2>&1
  rc=$?; echo "[$v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_ids.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python -u scripts/exp_cumask.py > gpurun_out/exp_cumask.log 2>&1
rc=$?; tail -1 gpurun_out/exp_cumask.log; [ $rc -eq 0 ] || exit $rc
