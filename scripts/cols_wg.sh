# halo pass's listed columns one workgroup per column (default) vs one thread per column
# (CSM_TUNE=cols_wg=0): shard parity tests, then the 8-way rank rehearsal interleaved
set -e
mkdir -p gpurun_out/cwg
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_api.py tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/cwg/tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/cwg/new_$rep.log 2>&1
  CSM_TUNE=cols_wg=0 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/cwg/base_$rep.log 2>&1
done
