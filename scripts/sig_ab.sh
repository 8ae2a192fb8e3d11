set -e
mkdir -p gpurun_out/sig
for i in 1 2; do
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/sig/def_$i.log 2>&1
  CSM_TUNE=signal_bwf=1 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/sig/bwf1_$i.log 2>&1
  CSM_TUNE=signal_vec=1 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/sig/vec1_$i.log 2>&1
done
