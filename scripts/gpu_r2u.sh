#!/bin/bash
# turnover chunking A/B (turn_want): C5 and C3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 4096 65536 131072; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune turn_want=$v > gpurun_out/bench_c5_u.log 2>&1
  rc=$?; echo "[c5 turn_want=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_u.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
for v in 4096 16384; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --tune turn_want=$v > gpurun_out/bench_c3_u.log 2>&1
  rc=$?; echo "[c3 turn_want=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_u.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
