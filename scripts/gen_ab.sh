# General turnover rows from per-row age tables: portfolio / sweep / capture tests, the C5 / C3
# full-size tests, a C5 trace and a C5 A/B against the previous build
set -e
mkdir -p gpurun_out/gen
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py tests/test_gpu_capture.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gen/tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "c3 or c5" > gpurun_out/gen/tests_full.log 2>&1
bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/gen/trace.txt 2>&1
bash scripts/ab.sh c5 3 > gpurun_out/gen/ab_c5.txt 2>&1
echo done
