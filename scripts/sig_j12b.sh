# second round of the signal_j12 A/B: the 8-way halo rank x3 and C4 x3, interleaved
set -e
mkdir -p gpurun_out/j12b
for rep in 1 2 3; do
  timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/j12b/halo_new_$rep.log 2>&1
  CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/j12b/halo_base_$rep.log 2>&1
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 > gpurun_out/j12b/new_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 > gpurun_out/j12b/base_$rep.json 2>/dev/null
done
