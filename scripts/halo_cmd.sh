set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp_shard_halo.py 100000 1250 10 8 > gpurun_out/halo_g8.log 2>&1 && tail -1 gpurun_out/halo_g8.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_median'], d['halo_back_to_back_ms_median'], d['halo_stages_ms_median'])"
