#!/bin/bash
# rocprofv3 evidence for the sweep benches (C3 / C5): kernel trace + stats in one run, HBM
# counters in separate --pmc passes, then the portfolio stage's bytes per step.
#   bash scripts/profile_sweep.sh <tag> <c3|c5>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:-r02}"
CFG="${2:-c5}"
OUT="gpurun_out/prof_${TAG}_${CFG}"
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "$CFG" = c5 ]; then RUNS="--steps 1 --warmup 1"; NRUN=2; else RUNS="--steps 3 --warmup 1"; NRUN=4; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --config $CFG $RUNS --no-cpu-baseline > "$OUT/trace.log" 2>&1
rc=$?; grep -h '"metric"' "$OUT/trace.log" | cut -c1-160; [ $rc -eq 0 ] || { tail -5 "$OUT/trace.log"; echo "FATAL trace rc=$rc"; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py --config $CFG $RUNS --no-cpu-baseline > "$OUT/pmc_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_fetch.log"; echo "FATAL fetch rc=$rc"; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py --config $CFG $RUNS --no-cpu-baseline > "$OUT/pmc_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_write.log"; echo "FATAL write rc=$rc"; exit $rc; }
python3 scripts/pmc_summary.py "$OUT" --N 5000 --T_d 6522 --workload "bench.py --config $CFG" \
  --source "profiles/$TAG/${CFG}_pmc_summary.json" --config "$CFG" --step-runs $NRUN \
  --stage "portfolio=k_label_sort,k_label_sort_legs_ew,k_cohort_seg,k_cohort_lds,k_cohort,k_fw_fold,k_turn_prep,k_turnover,k_overlap,k_overlap_rows,k_ls" \
  --stage-label "portfolio(k_cohort+k_turnover+k_overlap+k_ls)"
echo "profile_sweep done"
