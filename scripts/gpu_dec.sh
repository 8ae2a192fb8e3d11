#!/bin/bash
# Decile-kernel session: GPU tests, then per-phase timings of the wide decile kernel, the
# current build (libcsmom.so) interleaved with a baseline build (libcsmom_base.so, if present),
# plus the register-id variant; then the C4 bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/gpu_round.sh tests || exit $?
grep -q " passed" gpurun_out/gpu_tests.log && ! grep -q "failed" gpurun_out/gpu_tests.log || exit 1
PK=cross-sectional-momentum-strategy-replication-backtesting-framework_amd
: > gpurun_out/ph.log
for rep in 1 2; do
  for lib in libcsmom_base.so libcsmom.so; do
    [ -f $PK/$lib ] || continue
    echo "lib=$lib" >> gpurun_out/ph.log
    CSMOM_LIB=$PK/$lib timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 0 0 >> gpurun_out/ph.log 2>&1 || exit $?
  done
done
echo "lib=libcsmom.so reg=2" >> gpurun_out/ph.log
timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 0 2 >> gpurun_out/ph.log 2>&1 || exit $?
grep 'lib=\|"N"' gpurun_out/ph.log | cut -c1-400
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1 || exit $?
tail -1 gpurun_out/bench_c4.log | cut -c1-200; grep -o '"stage_ms": {[^}]*}' gpurun_out/bench_c4.log
