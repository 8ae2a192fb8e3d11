#!/bin/bash
# k_cohort_seg 16-B row staging + k_overlap_rows (C == 1): portfolio tests, C5 / C3 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_w.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests_w.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune seg_stage2=$v > gpurun_out/bench_c5_st$v.log 2>&1
  rc=$?; echo "[c5 seg_stage2=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_st$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
for v in 1 0; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --tune seg_stage2=$v > gpurun_out/bench_c3_st$v.log 2>&1
  rc=$?; echo "[c3 seg_stage2=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_st$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
