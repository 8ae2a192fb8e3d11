set -e
mkdir -p gpurun_out/c5ab
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5ab/on_$i.json 2> gpurun_out/c5ab/on_$i.err
  timeout -k 10 200 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --tune ls_opt=0 > gpurun_out/c5ab/off_$i.json 2> gpurun_out/c5ab/off_$i.err
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5ab/prof -o run -- python3 -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c5ab/prof.log 2>&1
