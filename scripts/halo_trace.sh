set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/halo_tr
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/halo_tr -o run -- python3 scripts/exp_shard_halo.py 100000 1250 3 8 > gpurun_out/halo_tr.log 2>&1 && find gpurun_out/halo_tr -name '*kernel_stats.csv' -exec cp {} gpurun_out/halo_kstats.csv \; && python3 scripts/stats_top.py gpurun_out/halo_kstats.csv 40 | grep -v "at::native\|rocclr" 
