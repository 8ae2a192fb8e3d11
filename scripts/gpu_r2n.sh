#!/bin/bash
# legs-only sweep accounting + paired multi-J scan default: tests, C5 / C3 benches (legs vs full)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_legs.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_legs.log; [ $rc -eq 0 ] || exit $rc
for v in "" "--full-deciles"; do
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline $v > gpurun_out/bench_c5_legs.log 2>&1
  rc=$?; echo "[c5 $v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_legs.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -u bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline $v > gpurun_out/bench_c3_legs.log 2>&1
  rc=$?; echo "[c3 $v]"; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c3_legs.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
