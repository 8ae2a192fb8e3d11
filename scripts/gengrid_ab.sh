# C3: the general-row turnover launch's persistent grid (turn_gen_grid) 1024 / 2048 vs 8192
set -e
mkdir -p gpurun_out/gg
for g in 8192 1024 2048 8192 1024 2048; do
  timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --tune turn_gen_grid=$g > gpurun_out/gg/c3_$g.log 2>&1
  python3 - gpurun_out/gg/c3_$g.log $g <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], round(d["ms_per_step"], 4), {k.split("(")[0]: v for k, v in d["stage_ms"].items()})
PY
done
