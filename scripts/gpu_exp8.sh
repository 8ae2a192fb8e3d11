#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/exp_dec_phases.py 100000 2 0 16 > gpurun_out/dec_phases8.log 2>&1
rc=$?; tail -1 gpurun_out/dec_phases8.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "wave_decile" > gpurun_out/gpu_exp8_tests.log 2>&1
rc=$?; tail -1 gpurun_out/gpu_exp8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5_narrow.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_narrow.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --tune dec_wave_max=16384 > gpurun_out/bench_c5_wave.log 2>&1
rc=$?; grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {[^}]*}' gpurun_out/bench_c5_wave.log; [ $rc -eq 0 ] || exit $rc
