#!/bin/bash
# paired-asset multi-J scan (mj_reg 2): tests + C5 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "momentum_multi" > gpurun_out/gpu_tests_mj2.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_mj2.log; [ $rc -eq 0 ] || exit $rc
for v in "--tune mj_reg=2" ""; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline $v > gpurun_out/bench_c5_mj2.log 2>&1
  rc=$?; echo "[$v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_mj2.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
