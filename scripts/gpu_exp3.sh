#!/bin/bash
# Round-2: id-pipeline parity + stress, decile phases, bench, full-size and process-group tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_pipe_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_pipe_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 2 0 0 > gpurun_out/dec_phases3.log 2>&1 && timeout -k 10 200 python -u scripts/exp_signal2.py 100000 pair_ids,pair_ids_sync1,pair_ids_sync2,pair_ids_sync4,nostore >> gpurun_out/dec_phases3.log 2>&1
rc=$?; tail -1 gpurun_out/dec_phases3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 16 > gpurun_out/bench_c4_ids.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' gpurun_out/bench_c4_ids.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_process_group.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_fullsize.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error" gpurun_out/gpu_fullsize.log | tail -20; [ $rc -eq 0 ] || exit $rc
echo exp3 done
