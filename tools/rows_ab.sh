#!/bin/bash
# A/B of the text-rows-only last joint layer (kernels.ROWS, env MMSEQ_ROWS): [full] GPU tests,
# tests/test_rows_gpu.py, then the short config-3 bench alternated off / on twice.
# usage (repo root, on the box): bash tools/rows_ab.sh [notests]
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/rows; mkdir -p $out
if [ "${1:-}" != notests ]; then
  timeout -k 10 600 python -u -m pytest -q -rs --maxfail 20 --timeout 300 --timeout-method thread tests -m gpu > $out/pytest_gpu.log 2>&1
fi
timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_rows_gpu.py -m gpu > $out/rows.log 2>&1
short="--no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer"
for v in 0 1 0 1; do
  MMSEQ_ROWS=$v timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 $short --fwd-steps 0 >> $out/bench_rows$v.log 2>&1
done
echo done >&2
