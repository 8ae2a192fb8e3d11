#!/bin/bash
# Round 2 session 3: read-pattern ceilings + split/fused A/B on one box, C2 hipGraph check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/mb/mb2.py > gpurun_out/mb2.log 2>&1
rc=$?; tail -1 gpurun_out/mb2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/exp_split2.py > gpurun_out/split2.log 2>&1
rc=$?; tail -1 gpurun_out/split2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c2_graph.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"hipgraph": [a-z]*\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c2_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u bench.py --config c2 --steps 50 --warmup 5 --no-cpu-baseline --graph off > gpurun_out/bench_c2_nograph.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"hipgraph": [a-z]*' gpurun_out/bench_c2_nograph.log; [ $rc -eq 0 ] || exit $rc
