set -u
bash scripts/gpu_round.sh all || exit $?
timeout -k 10 300 python -u scripts/exp_tune.py > gpurun_out/exp_tune.log 2>&1 || { echo "exp_tune failed"; tail -20 gpurun_out/exp_tune.log; exit 1; }
tail -2 gpurun_out/exp_tune.log
timeout -k 10 300 python -u scripts/mb/microbench.py > gpurun_out/mb.log 2>&1 || { echo "mb failed"; tail -20 gpurun_out/mb.log; exit 1; }
tail -2 gpurun_out/mb.log
