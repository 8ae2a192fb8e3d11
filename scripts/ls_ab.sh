# Long-short / overlap rework: the portfolio and sweep tests, then a C5 / C3 A/B against the
# previous build (ab/libcsmom_base.so)
set -e
mkdir -p gpurun_out/lsab
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py tests/test_gpu_capture.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lsab/tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "c3 or c5" > gpurun_out/lsab/tests_full.log 2>&1
bash scripts/ab.sh c5 2 > gpurun_out/lsab/ab_c5.txt 2>&1
bash scripts/ab.sh c3 2 > gpurun_out/lsab/ab_c3.txt 2>&1
echo done
