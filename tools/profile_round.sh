#!/bin/bash
# Round evidence for the default bench workload (config 3, 32 stories per step), run on the GPU box
# from the repo root:  bash tools/profile_round.sh <tag>
#   1. rocprofv3 --kernel-trace --stats            -> gpurun_out/prof_<tag>/kernel_stats.csv
#   2. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE  -> pmc_traffic.json (tools/pmc_traffic.py)
#   3. rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -> pmc_mfma_util.json
# Each counter pass is a run of its own (counters are not split over passes); every step has its
# own time limit and the first failure ends the script.
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:?tag}
out=gpurun_out/prof_$tag
mkdir -p "$out"
args="--no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer --fwd-steps 0"  # the training step only

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt" -o kt -- \
  python3 bench.py $args --steps 3 --warmup 1 > "$out/kt.log" 2>&1
cp "$(find "$out/kt" -name 'kt_kernel_stats.csv' | head -n1)" "$out/kernel_stats.csv"

timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- \
  python3 bench.py $args --steps 1 --warmup 0 > "$out/fetch.log" 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- \
  python3 bench.py $args --steps 1 --warmup 0 > "$out/write.log" 2>&1
python3 tools/pmc_traffic.py "$(find "$out/fetch" -name '*counter_collection.csv' | head -n1)" \
  "$(find "$out/write" -name '*counter_collection.csv' | head -n1)" "$out/pmc_traffic.json"

timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d "$out/mfma" -o mfma -- python3 bench.py $args --steps 1 --warmup 1 > "$out/mfma.log" 2>&1
python3 tools/pmc_mfma.py "$(find "$out/mfma" -name '*counter_collection.csv' | head -n1)" \
  "$out/pmc_mfma_util.json"
# raw per-dispatch CSVs are large and summarised above
find "$out/kt" -type f ! -name 'kt_kernel_stats.csv' -delete
rm -rf "$out/fetch" "$out/write" "$out/mfma"
echo "profile_round $tag done"
