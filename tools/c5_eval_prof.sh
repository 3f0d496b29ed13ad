#!/bin/bash
# Per-kernel times of the config-5 eval forward, bf16 vs MX-fp8 encoder GEMMs (same box):
#   bash tools/c5_eval_prof.sh <tag>  -> gpurun_out/c5_<tag>/{bf16,mxfp8}_kernel_stats.csv
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/c5_${1:?tag}
mkdir -p "$out"
for mode in bf16 mxfp8; do
  timeout -k 10 300 python3 tools/c5_eval.py $mode 5 > "$out/$mode.log" 2>&1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$mode" -o kt -- \
    python3 tools/c5_eval.py $mode 3 >> "$out/$mode.log" 2>&1
  cp "$(find "$out/$mode" -name 'kt_kernel_stats.csv' | head -n1)" "$out/${mode}_kernel_stats.csv"
  rm -rf "$out/$mode"
done
cat "$out"/*.log | grep mode
