"""Summarise rocprofv3 output for bench.py runs: per-kernel average duration (kernel stats)
and HBM bytes per launch from separate FETCH_SIZE / WRITE_SIZE passes, corrected per
MI355X_MICROARCH.md (gfx950 FETCH_SIZE counts half of a wide coalesced read: doubled;
WRITE_SIZE as read; both in KB).  Writes <outdir>/summary.json and, per kernel named with
--emit, profiles-ready pmc_<kernel>.json files ({N, T_d, kernel, hbm_bytes_per_launch}).

    python scripts/pmc_summary.py <prof_dir> --N 100000 --T_d 10000 --emit k_signal k_deciles
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short(name: str) -> str:
    """'void k_deciles<10, true>(double const*, ...)' -> 'k_deciles'"""
    n = name.strip().strip('"')
    n = re.sub(r"^void\s+", "", n)
    n = n.split("(")[0]
    n = n.split("<")[0].strip()
    return n.split("::")[-1]   # dec_wide::k_deciles -> k_deciles


def read_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                c, tot = int(row["Calls"]), float(row["TotalDurationNs"])
                a = out.setdefault(k, {"calls": 0, "total_ns": 0.0})
                a["calls"] += c
                a["total_ns"] += tot
    for v in out.values():
        v["avg_ns"] = v["total_ns"] / max(v["calls"], 1)
    return out


def read_counters(d):
    """{kernel: {counter: [per-dispatch values]}}"""
    vals = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", row.get("Kernel-Name", "")))
                disp = row.get("Dispatch_Id", row.get("Correlation_Id", "0"))
                cname = row.get("Counter_Name", row.get("Counter-Name"))
                vals[k][cname][disp] += float(row.get("Counter_Value", row.get("Counter-Value", 0)))
    return {k: {c: list(dv.values()) for c, dv in cs.items()} for k, cs in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prof_dir")
    ap.add_argument("--N", type=int, required=True)
    ap.add_argument("--T_d", type=int, required=True)
    ap.add_argument("--workload", default="")
    ap.add_argument("--emit", nargs="*", default=[])
    ap.add_argument("--emit-dir", default=None)
    ap.add_argument("--source", default="", help="where the committed summary will live")
    ap.add_argument("--stage", default=None,
                    help="sweeps: NAME=k1,k2,... -> pmc_sweep_<config>.json with the stage's HBM "
                         "bytes per step (all dispatches of those kernels / --step-runs)")
    ap.add_argument("--stage-label", default="", help="the bench's stage_ms key of that stage")
    ap.add_argument("--config", default="")
    ap.add_argument("--step-runs", type=int, default=0,
                    help="steps the PMC runs executed (warmup + steps)")
    a = ap.parse_args()
    stats = read_stats(os.path.join(a.prof_dir, "trace"))
    fetch = read_counters(os.path.join(a.prof_dir, "pmc_fetch"))
    write = read_counters(os.path.join(a.prof_dir, "pmc_write"))
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        fv = fetch.get(k, {}).get("FETCH_SIZE", [])
        wv = write.get(k, {}).get("WRITE_SIZE", [])
        if not fv and not wv:
            continue
        f_kb = sum(fv) / len(fv) if fv else 0.0
        w_kb = sum(wv) / len(wv) if wv else 0.0
        kern[k] = {"FETCH_SIZE_KB": f_kb, "WRITE_SIZE_KB": w_kb,
                   "hbm_bytes_corrected": 2.0 * f_kb * 1024.0 + w_kb * 1024.0,
                   "dispatches": max(len(fv), len(wv))}
    summ = {"workload": a.workload, "N": a.N, "T_d": a.T_d,
            "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 reports half of wide "
                    "coalesced reads); WRITE_SIZE as read; separate --pmc passes",
            "kernels": kern, "kernel_stats_ns": stats}
    with open(os.path.join(a.prof_dir, "summary.json"), "w") as fh:
        json.dump(summ, fh, indent=1)
    for k in a.emit:
        if k in kern:
            out = {"N": a.N, "T_d": a.T_d, "kernel": k,
                   "hbm_bytes_per_launch": kern[k]["hbm_bytes_corrected"],
                   "avg_ns": stats.get(k, {}).get("avg_ns"),
                   "source": a.source}
            with open(os.path.join(a.emit_dir or a.prof_dir, f"pmc_{k}.json"), "w") as fh:
                json.dump(out, fh, indent=1)
    if a.stage and a.step_runs > 0:
        name, ks = a.stage.split("=")
        ks = ks.split(",")
        tot = sum(kern[k]["hbm_bytes_corrected"] * kern[k]["dispatches"] for k in ks if k in kern)
        out = {"config": a.config, "N": a.N, "T_d": a.T_d, "stage": name,
               "stage_label": a.stage_label, "kernels": ks, "step_runs": a.step_runs,
               "hbm_bytes_per_step": tot / a.step_runs, "source": a.source}
        with open(os.path.join(a.emit_dir or a.prof_dir, f"pmc_sweep_{a.config}.json"), "w") as fh:
            json.dump(out, fh, indent=1)
        print(json.dumps(out))
    print(json.dumps({k: (v["hbm_bytes_corrected"], stats.get(k, {}).get("avg_ns"))
                      for k, v in kern.items()}))


if __name__ == "__main__":
    main()
