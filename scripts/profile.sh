#!/bin/bash
# rocprofv3 evidence for one bench.py configuration, folded into profiles/<tag>/<cfg>_profile.json
# (the file bench.py reads back for roofline.traffic / profile_frac):
#   1. --kernel-trace --stats of the bench command itself (per-kernel average durations);
#   2. two separate --pmc passes, FETCH_SIZE and WRITE_SIZE (they cannot share a pass);
#   3. scripts/profile_summary.py (gfx950 FETCH_SIZE correction, per-instantiation keys).
#   bash scripts/profile.sh <tag> <c4|c2|c3|c5> <git-head> [extra bench args]
# NT / NP: step executions per traced / pmc run -- warmup + timed, + 1 graph replay and an
# untimed eager stage pass of the same length (C2's hipGraph), + the sweeps' untimed stage pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG="${1:?tag}"
CFG="${2:?config}"
HEAD_SHA="${3:-unknown}"
shift 3
EXTRA="$*"
OUT="gpurun_out/prof_${TAG}_${CFG}"
rm -rf "$OUT"
mkdir -p "$OUT"
export TMPDIR=/tmp
case "$CFG" in
  c4) N=100000; TD=10000; RUN="--steps 20 --warmup 5"; NT=25; PMC="--steps 2 --warmup 1"; NP=3; STAGE="" ;;
  c2) N=5000; TD=6522; RUN="--steps 50 --warmup 5"; NT=106; PMC="--steps 2 --warmup 1"; NP=6; STAGE="" ;;
  c3) N=5000; TD=6522; RUN="--steps 10 --warmup 2"; NT=22; PMC="--steps 3 --warmup 1"; NP=7
      STAGE="--stage portfolio(k_cohort+k_turnover+k_overlap+k_ls)=k_label_sort,k_label_sort_legs_ew,k_cohort_seg,k_cohort_lds,k_cohort,k_fw_fold,k_turn_prep,k_turnover,k_overlap,k_overlap_rows,k_ls,k_ls_wide,k_ls_flags,k_ls_rows,k_turnover_vwg,k_turnover_ew_mask" ;;
  c5) N=5000; TD=6522; RUN="--steps 2 --warmup 1"; NT=5; PMC="--steps 1 --warmup 1"; NP=3
      STAGE="--stage portfolio(k_cohort+k_turnover+k_overlap+k_ls)=k_label_sort,k_label_sort_legs_ew,k_cohort_seg,k_cohort_lds,k_cohort,k_fw_fold,k_turn_prep,k_turnover,k_overlap,k_overlap_rows,k_ls,k_ls_wide,k_ls_flags,k_ls_rows,k_turnover_vwg,k_turnover_ew_mask" ;;
  *) echo "unknown config $CFG"; exit 2 ;;
esac
BENCH="bench.py --gpus 1 --config $CFG --no-cpu-baseline $EXTRA"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH $RUN > "$OUT/trace.log" 2>&1
rc=$?; grep -h '"metric"' "$OUT/trace.log" | cut -c1-300; [ $rc -eq 0 ] || { tail -5 "$OUT/trace.log"; echo "FATAL trace rc=$rc"; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 $BENCH $PMC > "$OUT/pmc_fetch.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_fetch.log"; echo "FATAL fetch rc=$rc"; exit $rc; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 $BENCH $PMC > "$OUT/pmc_write.log" 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 "$OUT/pmc_write.log"; echo "FATAL write rc=$rc"; exit $rc; }
python3 scripts/profile_summary.py "$OUT" --config "$CFG" --N $N --T_d $TD \
  --workload "rocprofv3 --kernel-trace --stats -- python3 $BENCH $RUN" --steps-trace $NT \
  --steps-pmc $NP --git-head "$HEAD_SHA" $STAGE --out "gpurun_out/profiles/${TAG}/${CFG}_profile.json"
rc=$?; [ $rc -eq 0 ] || exit $rc
cp "$OUT"/trace/*kernel_stats.csv "gpurun_out/profiles/${TAG}/${CFG}_kernel_stats.csv" 2>/dev/null || \
  find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "gpurun_out/profiles/${TAG}/${CFG}_kernel_stats.csv" \;
echo "profile $CFG done"
