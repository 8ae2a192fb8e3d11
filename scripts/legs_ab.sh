# Legs-only cohort partials in the two-leg layout: the portfolio / sweep / capture tests, the
# C3 / C5 full-size tests, a C5 kernel trace and C5 / C3 A/Bs against the previous build
set -e
mkdir -p gpurun_out/legs
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py tests/test_gpu_capture.py tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/legs/tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "c3 or c5" > gpurun_out/legs/tests_full.log 2>&1
bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/legs/trace.txt 2>&1
bash scripts/ab.sh c5 3 > gpurun_out/legs/ab_c5.txt 2>&1
bash scripts/ab.sh c3 2 > gpurun_out/legs/ab_c3.txt 2>&1
echo done
