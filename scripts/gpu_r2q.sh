#!/bin/bash
# BM turnover (bit-mask general kernel only), shard pass with bucket ids: tests, C5 bench, shard rehearsal
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_shards_api.py tests/test_gpu_process_group.py tests/test_gpu_portfolio.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_q.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_q.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_q.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_q.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/exp_shard.py 100000 10000 10 > gpurun_out/exp_shard_q.log 2>&1
rc=$?; tail -1 gpurun_out/exp_shard_q.log | cut -c1-500; [ $rc -eq 0 ] || exit $rc
