set -euo pipefail
export TMPDIR=/tmp PYTHONUNBUFFERED=1
out=gpurun_out/c5rows; mkdir -p $out
for v in 0 1; do for mode in bf16 fp8dg; do
  MMSEQ_ROWS=$v timeout -k 10 300 python3 tools/c5_train.py $mode 3 >> $out/c5_rows$v.log 2>&1
done; done
for v in 0 1; do for mode in bf16 fp8dg; do
  MMSEQ_ROWS=$v timeout -k 10 300 python3 tools/c5_train.py $mode 3 >> $out/c5_rows$v.log 2>&1
done; done
