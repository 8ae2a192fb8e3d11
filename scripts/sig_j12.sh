# wide k_signal with J = 12's product length fixed at compile time (in-tree build) vs the
# previous build (ab/libcsmom_base.so): parity tests, C4 bench lines interleaved, and the
# 8-way halo rank (its shard kernel takes the same path).
set -e
mkdir -p gpurun_out/j12
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/j12/tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 > gpurun_out/j12/new_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 > gpurun_out/j12/base_$rep.json 2>/dev/null
done
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/j12/halo_new.log 2>&1
CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/j12/halo_base.log 2>&1
