#!/bin/bash
# Round-2 evidence, part B: C5 / C3 rocprofv3 stats + PMC (portfolio-stage bytes per step), then
# the C3 and C5 bench lines carrying that traffic
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/profile_sweep.sh r02 c5 || exit $?
bash scripts/profile_sweep.sh r02 c3 || exit $?
cp gpurun_out/prof_r02_c5/pmc_sweep_c5.json gpurun_out/prof_r02_c3/pmc_sweep_c3.json profiles/
timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 > gpurun_out/bench_c3.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c3.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.log 2>&1
rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"traffic": [0-9.e+]*' gpurun_out/bench_c5.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp_shard.py 100000 10000 10 > gpurun_out/exp_shard.log 2>&1
rc=$?; tail -1 gpurun_out/exp_shard.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
echo final_b done
