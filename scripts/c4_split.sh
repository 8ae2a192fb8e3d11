# C4: the split decile pass (plan / chunk sweep / finish) forced on the 461-row launch vs the
# merged one-workgroup-per-row pass (default), interleaved
set -e
mkdir -p gpurun_out/c4s
for rep in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 > gpurun_out/c4s/base_$rep.json 2>/dev/null
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --match-dates 4 --tune dec_split=1 > gpurun_out/c4s/split_$rep.json 2>/dev/null
done
