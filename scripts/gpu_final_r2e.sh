#!/bin/bash
# Round-2 closing benches on the final code: C4 (default), C2, C3, C5 lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c4.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c2 --steps 50 --warmup 5 > gpurun_out/bench_c2.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"hipgraph": [a-z]*' gpurun_out/bench_c2.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/bench_c3.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c3.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c5.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
echo final_e done
