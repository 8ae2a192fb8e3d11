#!/bin/bash
# One guarded GPU session: tests -> smoke -> bench.  Any crash / abort / timeout (exit code
# other than 0 or 1) ends the script immediately; plain test failures (1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STAGE="${1:-all}"
ok_or_fail() { local rc=$1; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "FATAL rc=$rc in $2"; exit "$rc"; fi; }
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; tail -25 gpurun_out/gpu_tests.log; ok_or_fail $rc tests
fi
if [ "$STAGE" = all ] || [ "$STAGE" = smoke ]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -5 gpurun_out/smoke.log; ok_or_fail $rc smoke
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c2.log 2>&1
  rc=$?; tail -3 gpurun_out/bench_c2.log; ok_or_fail $rc bench_c2
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --cpu-assets 20000 > gpurun_out/bench_c4.log 2>&1
  rc=$?; tail -3 gpurun_out/bench_c4.log; ok_or_fail $rc bench_c4
fi
echo "gpu_round done"
