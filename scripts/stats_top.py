"""Top kernels of a rocprofv3 --stats kernel_stats.csv: calls, total ms, average us, share."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows[:n]:
    print(f"{int(r['Calls']):7d} {float(r['TotalDurationNs']) / 1e6:10.3f} ms "
          f"{float(r['AverageNs']) / 1e3:10.2f} us {float(r['Percentage']):6.2f}%  {r['Name'][:90]}")
