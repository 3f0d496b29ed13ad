"""Summarise rocprofv3 --pmc counter CSVs per kernel (average counter value per dispatch).

usage: python tools/pmc_summary.py <run_counter_collection.csv> [top]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        k = (r["Kernel_Name"][:70], r["Counter_Name"])
        agg[k][0] += 1
        agg[k][1] += float(r["Counter_Value"])
    for (name, ctr), (n, tot) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{name:70s} {ctr:12s} n={n:5d} avg={tot / n:.6g} total={tot:.6g}")


if __name__ == "__main__":
    main()
