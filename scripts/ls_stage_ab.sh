# Legs label sort with LDS-staged member-id stores: tests, then C5 A/Bs against the unstaged
# build (ab/libcsmom_base.so) and a trace of the 4-waves-per-EU variant (ab2/libcsmom_wpe4.so)
set -e
mkdir -p gpurun_out/lss
timeout -k 10 900 python -u -m pytest tests/test_gpu_portfolio.py tests/test_gpu_sweep_defer.py tests/test_gpu_boot_scan.py -x -q --timeout 300 --timeout-method thread > gpurun_out/lss/tests.log 2>&1
bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/lss/trace_new.txt 2>&1
CSMOM_AB_BASE=1 CSMOM_LIB=ab2/libcsmom_wpe4.so bash scripts/gpu_run.sh trace=c5,--steps,2,--warmup,1 > gpurun_out/lss/trace_wpe4.txt 2>&1
bash scripts/ab.sh c5 2 > gpurun_out/lss/ab_c5.txt 2>&1
echo done
