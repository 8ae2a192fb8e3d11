# C2 bench at several month-chunk counts of k_signal_tc (same box, interleaved repetitions).
set -e
mkdir -p gpurun_out/c2ch
for rep in 1 2 3; do
for C in 0 16 14 12 11 10; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 --chunks $C > gpurun_out/c2ch/c${C}_$rep.json 2> gpurun_out/c2ch/c${C}_$rep.err
done
done
