#!/bin/bash
# Round-3 evidence on the GPU box: default bench line + the round profile (kernel stats, PMC).
# usage: bash tools/r3_evidence.sh <tag> [tests]
set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
tag=${1:?tag}
mkdir -p gpurun_out/$tag
if [ "${2:-}" = tests ]; then
  timeout -k 10 900 python -u -m pytest -q --maxfail 20 --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/$tag/pytest_gpu.log 2>&1
fi
timeout -k 10 400 python -u bench.py > gpurun_out/$tag/bench.log 2>&1
bash tools/profile_round.sh $tag
