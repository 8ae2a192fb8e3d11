# Round-6 evidence on the current build: the four profiles (trace + FETCH / WRITE PMC), every
# bench line (reading those profiles back: same library sha), the date-shard rank rehearsals.
# Each step under its own time limit; the first failure ends the script.
set -e
mkdir -p gpurun_out/ev profiles/r06
TAG=r06 HEAD_SHA="$1" bash scripts/gpu_run.sh profile=c4 profile=c2 profile=c3 profile=c5
cp gpurun_out/profiles/r06/*_profile.json profiles/r06/
timeout -k 10 300 python -u bench.py > gpurun_out/ev/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/ev/bench_c2.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/ev/bench_c3.log 2>&1
timeout -k 10 400 python -u bench.py --config c5 > gpurun_out/ev/bench_c5.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/ev/halo_g8.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 2500 10 4 > gpurun_out/ev/halo_g4.log 2>&1
timeout -k 10 300 python -u scripts/exp_shard_halo.py 100000 5000 5 2 > gpurun_out/ev/halo_g2.log 2>&1
echo evidence done
