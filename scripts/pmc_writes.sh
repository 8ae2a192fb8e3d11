#!/bin/bash
# k_signal's store traffic by TCC write-request counters (verdict r05 #4): memory-side write
# requests and how many of them are 64-B requests, then L2 write requests from the CUs -- each
# pass its own rocprofv3 run on the C4 bench (2 timed steps), per-kernel sums into one table.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_writes
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-oracle-mom --match-dates 2"
timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$OUT/p1" -o run -- python3 $BENCH > "$OUT/p1.log" 2>&1 || { tail -5 "$OUT/p1.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc TCC_WRITE_sum --output-format csv -d "$OUT/p2" -o run -- python3 $BENCH > "$OUT/p2.log" 2>&1 || { tail -5 "$OUT/p2.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "k_signal" in k or "k_deciles" in k:
        print(k, {c: (len(v), sum(v) / len(v)) for c, v in d.items()})
PY
