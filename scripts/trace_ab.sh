# rocprofv3 kernel stats of one bench config for the in-tree library and ab/libcsmom_base.so
#   bash scripts/trace_ab.sh <cfg> [bench args]
set -u
cfg="$1"; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in new base; do
  out="gpurun_out/trab_${cfg}_${v}"; rm -rf "$out"
  if [ "$v" = base ]; then export CSMOM_LIB=ab/libcsmom_base.so CSMOM_AB_BASE=1; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 bench.py --config "$cfg" --no-cpu-baseline --no-oracle-mom "$@" > "$out.log" 2>&1 || { tail -5 "$out.log"; exit 1; }
  find "$out" -name '*kernel_stats.csv' -exec cp {} "$out.kernel_stats.csv" \;
  echo "== $v"; python3 scripts/stats_top.py "$out.kernel_stats.csv" 14 | grep -v "at::native\|rocclr"
done
