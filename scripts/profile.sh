#!/bin/bash
# rocprofv3 evidence for bench.py: kernel trace + stats in one run; HBM counters in separate
# --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a pass); summary via pmc_summary.py.
#   bash scripts/profile.sh <tag> <config> [N T_d]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-r01}"
CFG="${2:-c4}"
NN="${3:-100000}"
TD="${4:-10000}"
OUT="gpurun_out/prof_${TAG}_${CFG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.log" 2>&1
rc=$?; grep -h '"metric"' "$OUT/trace.log" | cut -c1-200; [ $rc -eq 0 ] || { tail -5 "$OUT/trace.log"; echo "FATAL trace rc=$rc"; exit $rc; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_fetch.log"; echo "FATAL fetch rc=$rc"; exit $rc; }
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_write.log"; echo "FATAL write rc=$rc"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" --N "$NN" --T_d "$TD" --workload "bench.py --config $CFG" --source "profiles/$TAG/${CFG}_pmc_summary.json" --emit k_signal k_deciles k_month_end k_cohort_seg k_turnover k_label_sort
echo "profile done"
