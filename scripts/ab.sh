#!/bin/bash
# Same-box A/B of the in-tree libcsmom.so against ab/libcsmom_base.so (scripts/build_variant.py)
# on one bench config, alternating runs so box drift hits both:
#   bash scripts/ab.sh <cfg> <rounds> [bench args...]
# BASE_ARGS="--flag ..." instead: the base runs are the in-tree library with those bench flags.
# Each run under its own time limit; the first failing run ends the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cfg="$1"; rounds="$2"; shift 2
for i in $(seq 1 "$rounds"); do
  for v in new base; do
    log="gpurun_out/ab_${cfg}_${v}_${i}.log"
    if [ "$v" = base ] && [ -n "${BASE_ARGS:-}" ]; then
      timeout -k 10 300 python -u bench.py --config "$cfg" --no-cpu-baseline "$@" $BASE_ARGS > "$log" 2>&1 || { echo "run $v $i failed"; tail -5 "$log"; exit 1; }
    elif [ "$v" = base ]; then
      CSMOM_AB_BASE=1 CSMOM_LIB=ab/libcsmom_base.so timeout -k 10 300 python -u bench.py --config "$cfg" --no-cpu-baseline "$@" > "$log" 2>&1 || { echo "run $v $i failed"; tail -5 "$log"; exit 1; }
    else
      timeout -k 10 300 python -u bench.py --config "$cfg" --no-cpu-baseline "$@" > "$log" 2>&1 || { echo "run $v $i failed"; tail -5 "$log"; exit 1; }
    fi
    python3 - "$log" "$v" <<'EOF'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], round(d["ms_per_step"], 4), {k.split("(")[0]: v for k, v in d["stage_ms"].items()})
EOF
  done
done
