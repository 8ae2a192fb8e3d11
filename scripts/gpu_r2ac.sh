#!/bin/bash
# k_turn_prep with its age loop unrolled: tests + C5 line + kernel time
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_portfolio.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_ac.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_tests_ac.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ac -o run -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_ac.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"portfolio[^,]*' gpurun_out/bench_c5_ac.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc
grep -h "k_turn_prep\|k_label_sort_legs" gpurun_out/prof_ac/run_kernel_stats.csv | cut -c1-160
