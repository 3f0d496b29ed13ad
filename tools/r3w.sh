# attention forward with the full-tile body specialised (nkb = 4 at compile time) vs HEAD
mkdir -p gpurun_out/r3w
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropout_gpu.py tests/test_fp8_gpu.py -m gpu -k "attention or attn" > gpurun_out/r3w/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3w/tests.log
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3w/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r3w/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r3w/$n -name 'kt_kernel_stats.csv' | head -n1); cat $f >> gpurun_out/r3w/${n}_stats.csv; rm -rf gpurun_out/r3w/$n
done
