#!/bin/bash
# The one GPU-box runner (replaces round 2's single-use launchers).  Steps run in order, each
# under its own time limit, and the run stops at the first failing step (no retries):
#   tests[=<pytest -k expr>]   pytest -m gpu (one process), log gpurun_out/gpu_tests.log
#   smoke                      __graft_entry__.smoke(), log gpurun_out/smoke.log
#   bench=<cfg>[,arg,arg...]   python bench.py --config <cfg> [args], log gpurun_out/bench_<cfg>.log
#   profile=<cfg>              scripts/profile.sh <tag> <cfg> <head> (tag / head from $TAG / $HEAD_SHA)
#   py=<script>[,arg...]       python <script> [args], log gpurun_out/py_<name>.log
#   bash scripts/gpu_run.sh tests smoke bench=c4,--steps,20,--warmup,5 profile=c4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG="${TAG:-r03}"
HEAD_SHA="${HEAD_SHA:-unknown}"
for step in "$@"; do
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
      timeout -k 10 600 python -u bench.py --config $cfg $rest > "gpurun_out/bench_${cfg}.log" 2>&1
      rc=$?; grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.]*\|"frac": [0-9.]*\|"stage_ms": {[^}]*}\|"decile_match_pct": [0-9.]*' "gpurun_out/bench_${cfg}.log" | tr '\n' ' '; echo ;;
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
