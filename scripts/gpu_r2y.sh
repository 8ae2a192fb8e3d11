#!/bin/bash
# k_turn_prep (steady EW turnover rows without the per-workgroup prologue) + general-row grid A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_y.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_y.log; [ $rc -eq 0 ] || exit $rc
for v in "turn_prep=1" "turn_prep=0" "turn_gen_grid=8192" "turn_gen_grid=512"; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune $v > gpurun_out/bench_c5_y.log 2>&1
  rc=$?; echo "[c5 $v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_y.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
  cp gpurun_out/bench_c5_y.log "gpurun_out/bench_c5_y_$v.log"
done
for v in 1 0; do
  timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --tune turn_prep=$v > gpurun_out/bench_c3_y$v.log 2>&1
  rc=$?; echo "[c3 turn_prep=$v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c3_y$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
