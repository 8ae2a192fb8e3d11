"""Per-kernel totals from a rocprofv3 sqlite output (rocpd schema): python scripts/prof_db.py <dir> [steps]"""
import glob
import sqlite3
import sys

d = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for db in glob.glob(f"{d}/**/*.db", recursive=True):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(duration)/1e6, avg(duration)/1e3 from kernels "
                     "group by name order by 3 desc limit 25").fetchall()
    print(db)
    for name, n, tot, avg in rows:
        print(f"{tot / steps:9.3f} ms/step {n / steps:7.1f} calls/step {avg:9.1f} us  {name[:80]}")
