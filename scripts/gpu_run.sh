#!/bin/bash
# The one GPU-box runner (replaces round 2's single-use launchers).  Steps run in order, each
# under its own time limit, and the run stops at the first failing step (no retries):
#   tests[=<pytest -k expr>]   pytest -m gpu (one process), log gpurun_out/gpu_tests.log
#   smoke                      __graft_entry__.smoke(), log gpurun_out/smoke.log
#   bench=<cfg>[,arg,arg...]   python bench.py --config <cfg> [args], log gpurun_out/bench_<cfg>_<step#>.log
#   trace=<cfg>[,arg...]       rocprofv3 --kernel-trace --stats of bench.py, gpurun_out/trace_<cfg>_<step#>.kernel_stats.csv
#   profile=<cfg>              scripts/profile.sh <tag> <cfg> <head> (tag / head from $TAG / $HEAD_SHA)
#   py=<script>[,arg...]       python <script> [args], log gpurun_out/py_<name>.log
#   bash scripts/gpu_run.sh tests smoke bench=c4,--steps,20,--warmup,5 profile=c4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${TAG:-r03}"
HEAD_SHA="${HEAD_SHA:-unknown}"
idx=0
for step in "$@"; do
  idx=$((idx + 1))
  name="${step%%=*}"
  arg=""
  [ "$step" != "$name" ] && arg="${step#*=}"
  args="${arg//,/ }"
  t0=$(date +%s)
  case "$name" in
    tests)
      if [ -n "$arg" ]; then K=(-k "$arg"); else K=(); fi
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${K[@]}" > gpurun_out/gpu_tests.log 2>&1
      rc=$?; tail -3 gpurun_out/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; tail -2 gpurun_out/smoke.log ;;
    bench)
      cfg="${args%% *}"; rest="${args#"$cfg"}"
      log="gpurun_out/bench_${cfg}_${idx}.log"
      timeout -k 10 600 python -u bench.py --config $cfg $rest > "$log" 2>&1
      rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' "$log" | tr '\n' ' '; echo ;;
    trace)
      cfg="${args%% *}"; rest="${args#"$cfg"}"
      out="gpurun_out/trace_${cfg}_${idx}"
      ( export TMPDIR=/tmp; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 bench.py --config $cfg --no-cpu-baseline $rest > "$out.log" 2>&1 )
      rc=$?; find "$out" -name '*kernel_stats.csv' -exec cp {} "$out.kernel_stats.csv" \; ; rm -rf "$out"
      python3 scripts/stats_top.py "$out.kernel_stats.csv" 25 ;;
    profile)
      timeout -k 10 1000 bash scripts/profile.sh "$TAG" "$arg" "$HEAD_SHA"
      rc=$? ;;
    py)
      scr="${args%% *}"; rest="${args#"$scr"}"
      timeout -k 10 600 python -u $scr $rest > "gpurun_out/py_$(basename "$scr" .py).log" 2>&1
      rc=$?; tail -5 "gpurun_out/py_$(basename "$scr" .py).log" ;;
    *) echo "unknown step $step"; rc=2 ;;
  esac
  echo "[gpu_run] $step rc=$rc $(( $(date +%s) - t0 ))s"
  [ $rc -eq 0 ] || exit $rc
done
echo "[gpu_run] all done"
