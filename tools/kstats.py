"""Summarise a rocprofv3 --stats kernel CSV: per-step ms and share per kernel."""
import csv, sys
path = sys.argv[1]; steps = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / steps / 1e6:.1f} ms/step")
for r in rows[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{r['Name'][:78]:78s} {int(r['Calls']):6d} {float(r['TotalDurationNs']) / steps / 1e6:8.2f} ms "
          f"{float(r['Percentage']):5.1f}% avg {float(r['AverageNs']) / 1e3:8.1f} us")
