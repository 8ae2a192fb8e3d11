# k_turnover_ew_mask with the row's loads issued together: tests, a bit check against the
# previous form (ab/libcsmom_base.so: -DTM_EARLY=0), a C5 trace and A/B
set -e
mkdir -p gpurun_out/tm
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py tests/test_gpu_capture.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tm/tests.log 2>&1
timeout -k 10 200 python -u scripts/gen_tab_bits.py > gpurun_out/tm/bits_new.txt 2>&1
CSMOM_AB_BASE=1 CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 200 python -u scripts/gen_tab_bits.py > gpurun_out/tm/bits_base.txt 2>&1
bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/tm/trace.txt 2>&1
bash scripts/ab.sh c5 3 > gpurun_out/tm/ab_c5.txt 2>&1
echo done
