"""Run only bench.py's RN50-backbone leg (for rocprofv3 --kernel-trace --stats).

Usage: python tools/rn50_prof.py [--steps 2 --warmup 1]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    a = ap.parse_args()
    print(json.dumps(bench.bench_config3_rn50(32, 16, a.steps, a.warmup, "cuda")))


if __name__ == "__main__":
    main()
