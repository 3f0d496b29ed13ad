#!/bin/bash
# Round evidence on the GPU box, in the order that keeps the bench line's sources current:
#   1. pytest -m gpu (all), smoke
#   2. tools/profile_round.sh TAG: kernel stats + PMC traffic + MFMA busy of the default workload
#   3. its summaries copied into profiles/TAG_* on the box, so that the bench that follows cites
#      PMC passes of this same tree (bench.py reads the newest profiles/r*_v*_pmc_*.json)
#   4. the default bench line
# usage (repo root, on the box): bash tools/evidence.sh r4_v6 [notests]
# Everything lands in gpurun_out/TAG/ (copy the summaries into profiles/ afterwards).
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:?tag}
out=gpurun_out/$tag
mkdir -p "$out"
[ "${2:-}" = notests ] || bash tools/gpu_run.sh "$tag" tests smoke
bash tools/profile_round.sh "$tag"
p=gpurun_out/prof_$tag
cp "$p/kernel_stats.csv" "profiles/${tag}_kernel_stats.csv"
cp "$p/pmc_traffic.json" "profiles/${tag}_pmc_traffic.json"
cp "$p/pmc_mfma_util.json" "profiles/${tag}_pmc_mfma_util.json"
cp "$p/kernel_stats.csv" "$p/pmc_traffic.json" "$p/pmc_mfma_util.json" "$out/"
timeout -k 10 900 python -u bench.py > "$out/bench.log" 2>&1
echo "evidence $tag done" >&2
