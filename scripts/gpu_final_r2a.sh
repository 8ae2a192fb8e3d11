#!/bin/bash
# Round-2 evidence, part A: full GPU suite, smoke, C4 rocprofv3 stats + PMC, C4 and C2 benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r02 c4 || exit $?
cp gpurun_out/prof_r02_c4/pmc_k_signal.json gpurun_out/prof_r02_c4/pmc_k_deciles.json profiles/ 2>/dev/null
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c4.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config c2 --steps 50 --warmup 5 > gpurun_out/bench_c2.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"hipgraph": [a-z]*' gpurun_out/bench_c2.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
echo final_a done
