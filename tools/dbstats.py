"""Per-kernel summary (calls, total, average, share) from a rocprofv3 --kernel-trace database
(the `kernels` view of the .db rocprofv3 writes), optionally exported as the --stats CSV layout.
usage: python tools/dbstats.py results.db [divisor] [top] [--csv out.csv]"""
import csv
import sqlite3
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
out_csv = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
if out_csv in args:
    args.remove(out_csv)
db, div = args[0], float(args[1]) if len(args) > 1 else 1.0
top = int(args[2]) if len(args) > 2 else 30
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
                 f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows)
print(f"total kernel time {tot / 1e6:.2f} ms ({tot / div / 1e6:.2f} ms per unit of {div:g})")
for n, k, s, a, lo, hi in rows[:top]:
    print(f"{n[:90]:90s} {k:6d} {s / div / 1e6:8.2f} ms {100 * s / tot:5.1f}% avg {a / 1e3:8.1f} us")
if out_csv:
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for n, k, s, a, lo, hi in rows:
            w.writerow([n, k, s, a, 100 * s / tot, lo, hi])
