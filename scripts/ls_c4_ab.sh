# k_long_short in one round trip: the pipeline / parity tests, a C4 trace and C4 A/B against the
# previous build
set -e
mkdir -p gpurun_out/lsc4
timeout -k 10 900 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lsc4/tests.log 2>&1
bash scripts/gpu_run.sh trace=c4,--steps,5,--warmup,2,--match-dates,4,--no-oracle-mom > gpurun_out/lsc4/trace.txt 2>&1
bash scripts/ab.sh c4 3 --match-dates 4 --no-oracle-mom > gpurun_out/lsc4/ab_c4.txt 2>&1
echo done
