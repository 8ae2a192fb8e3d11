# The split sweep variants (dec_split_pf auto / prefetch always / never) on the date-shard rank
# rehearsals at G = 8 / 4, plus the split-vs-merged tests
set -e
mkdir -p gpurun_out/pf
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread -k "split or chunk_order" > gpurun_out/pf/tests.log 2>&1
for g in "8 1250" "4 2500"; do
  set -- $g
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 $2 10 $1 > gpurun_out/pf/g$1.log 2>&1
  CSM_TUNE=dec_split_pf=1 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 $2 10 $1 > gpurun_out/pf/g$1_pf1.log 2>&1
  CSM_TUNE=dec_split_pf=0 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 $2 10 $1 > gpurun_out/pf/g$1_pf0.log 2>&1
done
echo done
