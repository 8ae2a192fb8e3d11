#!/bin/bash
# k_overlap_rows: bit-identity tests, then C5 / C3 A/B against k_overlap (overlap_rows 1 / 0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ov.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests_ov.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune overlap_rows=$v > gpurun_out/bench_c5_ov$v.log 2>&1
  rc=$?; echo "[c5 overlap_rows=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_ov$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
for v in 1 0; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --tune overlap_rows=$v > gpurun_out/bench_c3_ov$v.log 2>&1
  rc=$?; echo "[c3 overlap_rows=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_ov$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
