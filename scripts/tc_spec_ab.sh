# k_signal_tc with the speculative scan in the idle waves (in-tree build) vs without
# (ab/libcsmom_spec0.so, same barrier-free hand-off) vs the previous build (ab/libcsmom_base.so):
# parity tests first, then C2 bench lines interleaved, then phase stamps (ab/libcsmom_tct.so).
set -e
mkdir -p gpurun_out/spec
timeout -k 10 300 python -u -m pytest tests/test_gpu_signal_chunked.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spec/tests.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/spec/new_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_spec0.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/spec/s0_$rep.json 2>/dev/null
  CSMOM_LIB=$PWD/ab/libcsmom_base.so timeout -k 10 120 python -u bench.py --config c2 --steps 100 --warmup 20 --no-cpu-baseline --match-dates 4 > gpurun_out/spec/base_$rep.json 2>/dev/null
done
CSMOM_LIB=$PWD/ab/libcsmom_tct.so timeout -k 10 100 python -u scripts/exp_tc_phases.py 12 > gpurun_out/spec/phases_c12.json 2>&1
