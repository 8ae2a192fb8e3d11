# k_shard_summary_cols over a strided grid: the shard tests, then the 8-way / 4-way rank rehearsals
set -e
mkdir -p gpurun_out/cg
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_api.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread -k "halo or shard or cols" > gpurun_out/cg/tests.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/cg/g8.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 2500 10 4 > gpurun_out/cg/g4.log 2>&1
echo done
