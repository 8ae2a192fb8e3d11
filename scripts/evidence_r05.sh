# Round-5 bench lines (after the profiles of the same build are committed) and the date-shard
# rank rehearsals; every step under its own time limit, stop at the first failure.
set -e
mkdir -p gpurun_out/ev
timeout -k 10 300 python -u bench.py > gpurun_out/ev/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/ev/bench_c2.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 > gpurun_out/ev/bench_c3.log 2>&1
timeout -k 10 400 python -u bench.py --config c5 > gpurun_out/ev/bench_c5.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/ev/halo_g8.log 2>&1
CSM_DEC_SPLIT=0 timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/ev/halo_g8_split_off.log 2>&1
timeout -k 10 200 python -u scripts/exp_shard_halo.py 100000 2500 10 4 > gpurun_out/ev/halo_g4.log 2>&1
timeout -k 10 300 python -u scripts/exp_shard_halo.py 100000 5000 5 2 > gpurun_out/ev/halo_g2.log 2>&1
