#!/bin/bash
# general equal-weight turnover launch at 4 (117 VGPRs) / 5 / 8 workgroups per CU (spilling builds)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in default mb5 mb8; do
  if [ $v = default ]; then unset CSMOM_LIB; else export CSMOM_LIB=$PWD/exp_lib/libcsmom_$v.so; fi
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_z_$v.log 2>&1
  rc=$?; echo "[c5 $v]"; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_z_$v.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
done
