set -e
mkdir -p gpurun_out/c2ch
for rep in 1 2; do
for C in 21 24 25 26 32 16; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --match-dates 4 --chunks $C > gpurun_out/c2ch/c${C}_$rep.json 2> gpurun_out/c2ch/c${C}_$rep.err
done
done
