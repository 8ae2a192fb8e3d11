"""Print the last pass of a kernel trace as (start offset us, duration us, kernel) rows."""
import csv
import glob
import sys

rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                         r.get("Queue_Id", "")))
rows.sort()
keep = [r for r in rows if "k_" in r[2]]
last = keep[-int(sys.argv[2]):] if len(sys.argv) > 2 else keep[-20:]
t0 = last[0][0]
for s, e, n, q in last:
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f}  q{q:>3} {n}")
