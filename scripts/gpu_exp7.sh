#!/bin/bash
# Wider fixed map: id-pipeline parity, decile phases, C4 bench, C4 rocprofv3 stats + PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "not c3 and not c5" > gpurun_out/gpu_exp7_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_exp7_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 2 0 0 > gpurun_out/dec_phases7.log 2>&1
rc=$?; tail -1 gpurun_out/dec_phases7.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_c4.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*\|"frac": [0-9.]*' gpurun_out/bench_c4.log; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r02 c4 || exit $?
echo exp7 done
