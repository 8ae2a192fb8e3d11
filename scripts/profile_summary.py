"""Fold the rocprofv3 output of scripts/profile.sh into the committed evidence file
profiles/<tag>/<config>_profile.json that bench.py reads back (roofline.traffic, profile_frac):

  kernels: per kernel INSTANTIATION (template arguments kept, so two launches of differently
           specialised kernels are never averaged together): calls and average duration from
           --kernel-trace --stats of the bench command itself; HBM bytes per launch from the
           separate FETCH_SIZE and WRITE_SIZE --pmc passes, corrected per MI355X_MICROARCH.md
           (gfx950 FETCH_SIZE counts half of a wide coalesced read: doubled; WRITE_SIZE as read;
           both in KB);
  stage:   sweeps -- the dominant bench stage's kernels summed per step (device ns and HBM bytes);
  lib_sha256 / git_head: the build and commit profiled (bench.py ignores the file for any other
           build of libcsmom.so).

    python scripts/profile_summary.py <prof_dir> --config c4 --N 100000 --T_d 10000 \
        --steps-trace 25 --steps-pmc 4 --git-head <sha> --out profiles/r03/c4_profile.json
"""
import argparse
import csv
import glob
import hashlib
import json
import os
import re
import socket
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cross-sectional-momentum-strategy-replication-backtesting-framework_amd")


def key(name: str) -> str:
    """'void dec_pre::k_deciles<10, true, true, true>(double const*, ...)' ->
    'k_deciles<10, true, true, true>' (namespace and argument list dropped)."""
    n = name.strip().strip('"')
    n = re.sub(r"^void\s+", "", n)
    depth, out = 0, ""
    for ch in n:   # cut at the argument list's '(' (outside template brackets)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out += ch
    out = out.strip()
    base = out.split("<")[0]
    return base.split("::")[-1] + out[len(base):]


def read_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = key(row["Name"])
                a = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
                a["calls"] += int(row["Calls"])
                a["total_ns"] += float(row["TotalDurationNs"])
    for v in out.values():
        v["avg_ns"] = v["total_ns"] / max(v["calls"], 1)
    return out


def read_counter(d, counter):
    """{kernel: [per-dispatch value]}"""
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name", row.get("Counter-Name")) != counter:
                    continue
                k = key(row.get("Kernel_Name", row.get("Kernel-Name", "")))
                disp = row.get("Dispatch_Id", row.get("Correlation_Id", "0"))
                vals[k][disp] += float(row.get("Counter_Value", row.get("Counter-Value", 0)))
    return {k: list(v.values()) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--config", required=True)
    ap.add_argument("--N", type=int, required=True)
    ap.add_argument("--T_d", type=int, required=True)
    ap.add_argument("--workload", default="")
    ap.add_argument("--steps-trace", type=int, required=True, help="warmup + timed steps traced")
    ap.add_argument("--steps-pmc", type=int, required=True, help="warmup + timed steps per pmc pass")
    ap.add_argument("--git-head", default="")
    ap.add_argument("--stage", default=None, help="LABEL=prefix1,prefix2,... (kernel name prefixes)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    stats = read_stats(os.path.join(a.prof_dir, "trace"))
    fetch = read_counter(os.path.join(a.prof_dir, "pmc_fetch"), "FETCH_SIZE")
    write = read_counter(os.path.join(a.prof_dir, "pmc_write"), "WRITE_SIZE")
    kern = {}
    for k in sorted(set(stats) | set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue   # torch generator / copy kernels of the bench's setup
        e = dict(stats.get(k, {}))
        fv, wv = fetch.get(k, []), write.get(k, [])
        if fv or wv:
            f_kb = sum(fv) / len(fv) if fv else 0.0
            w_kb = sum(wv) / len(wv) if wv else 0.0
            e.update(fetch_bytes=2.0 * f_kb * 1024.0, write_bytes=w_kb * 1024.0,
                     hbm_bytes_per_launch=2.0 * f_kb * 1024.0 + w_kb * 1024.0,
                     pmc_dispatches=max(len(fv), len(wv)))
        kern[k] = e
    lib = os.path.join(PKG, "libcsmom.so")
    out = {"config": a.config, "workload": a.workload, "N": a.N, "T_d": a.T_d,
           "git_head": a.git_head, "host": socket.gethostname(),
           "lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest(),
           "note": "kernel averages: rocprofv3 --kernel-trace --stats of the bench command; HBM "
                   "bytes: separate FETCH_SIZE / WRITE_SIZE --pmc passes, FETCH doubled per "
                   "MI355X_MICROARCH.md (gfx950), both KB",
           "kernels": kern}
    if a.stage:
        label, prefixes = a.stage.split("=")
        ks = [k for k in kern if any(k.startswith(p + "<") or k == p for p in prefixes.split(","))]
        ns = sum(kern[k].get("total_ns", 0.0) for k in ks) / a.steps_trace
        by = sum(kern[k].get("hbm_bytes_per_launch", 0.0) * kern[k].get("pmc_dispatches", 0)
                 for k in ks) / a.steps_pmc
        out["stage"] = {"label": label, "kernels": ks, "ns_per_step": ns, "hbm_bytes_per_step": by}
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps({k: (round(v.get("avg_ns", 0) / 1e3, 2), v.get("hbm_bytes_per_launch"))
                      for k, v in kern.items()}))


if __name__ == "__main__":
    main()
