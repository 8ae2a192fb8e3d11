# Date-shard rank rehearsals: the default halo pass (two launches) at G = 8 / 4 / 2, and the
# split-decile chunk size (dec_split_cells 16384 / 8192 vs the default 32768) at G = 8 / 4
set -e
mkdir -p gpurun_out/sc
for g in "8 1250 10" "4 2500 10" "2 5000 5"; do
  set -- $g
  timeout -k 10 300 python -u scripts/exp_shard_halo.py 100000 $2 $3 $1 > gpurun_out/sc/g$1.log 2>&1
done
for c in 16384 8192; do
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 $c > gpurun_out/sc/g8_c$c.log 2>&1
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 2500 10 4 $c > gpurun_out/sc/g4_c$c.log 2>&1
done
echo done
