# k_cohort_seg panel-major XCD order: the portfolio / sweep tests, a C5 trace, C5 / C3 A/Bs
# against the month-major order (ab/libcsmom_base.so: -DSEG_PANEL_MAJOR=0)
set -e
mkdir -p gpurun_out/seg
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/seg/tests.log 2>&1
bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/seg/trace.txt 2>&1
bash scripts/ab.sh c5 3 > gpurun_out/seg/ab_c5.txt 2>&1
echo done
