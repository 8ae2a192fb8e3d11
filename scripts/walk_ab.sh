set -e
mkdir -p gpurun_out/walk
for i in 1 2; do
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/walk/w8_$i.log 2>&1
  CSMOM_LIB=ab/libcsmom_w16.so timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/walk/w16_$i.log 2>&1
  CSMOM_LIB=ab/libcsmom_w32.so timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/walk/w32_$i.log 2>&1
done
