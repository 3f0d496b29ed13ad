#!/bin/bash
# PMC passes over tools/fp8_one.py (MX-fp8 vs bf16 NT GEMM, one shape): bash tools/fp8_pmc.sh <tag> [N K]
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/fp8pmc_${1:?tag}
shift
mkdir -p "$out"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_VMEM --output-format csv -d "$out/p1" -o p1 -- python3 tools/fp8_one.py "$@" > "$out/log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$out/p2" -o p2 -- python3 tools/fp8_one.py "$@" >> "$out/log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/p3" -o p3 -- python3 tools/fp8_one.py "$@" >> "$out/log" 2>&1
for p in p1 p2 p3; do
  python3 tools/pmc_summary.py "$(find "$out/$p" -name '*counter_collection.csv' | head -n1)" 40 > "$out/$p.txt"
done
rm -rf "$out/p1" "$out/p2" "$out/p3"
echo "fp8_pmc done"
