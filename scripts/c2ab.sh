set -e
mkdir -p gpurun_out/c2ab
for i in 1 2 3; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --match-dates 8 > gpurun_out/c2ab/tc_$i.json 2> gpurun_out/c2ab/tc_$i.err
  timeout -k 10 120 python -u bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --match-dates 8 --c2-unfused > gpurun_out/c2ab/un_$i.json 2> gpurun_out/c2ab/un_$i.err
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c2ab/prof -o run -- python3 -u bench.py --config c2 --steps 50 --warmup 10 --no-cpu-baseline --match-dates 8 > gpurun_out/c2ab/prof.log 2>&1
