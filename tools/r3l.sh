# isolate the bf16 decisive-margin regression of 1c3d01d; per-kernel attention times (rocprof) A/B
mkdir -p gpurun_out/r3l
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in ab/libmmseq_1c_oldattn.so ab/libmmseq_1c_oldgemm.so; do
  export MMSEQ_BENCH_LIB=$lib
  echo "== $lib" >> gpurun_out/r3l/bisect.log
  timeout -k 10 200 python -u -m pytest -q -s --timeout 150 --timeout-method thread tests/test_order_gpu.py -m gpu -k "bf16 and config3" >> gpurun_out/r3l/bisect.log 2>&1
  rc=$?; echo "rc $rc" >> gpurun_out/r3l/bisect.log; [ $rc -le 1 ] || exit 1
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_nofold.so; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=$(basename $lib .so); fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3l/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r3l/$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r3l/$n -name 'kt_kernel_stats.csv' | head -n1); cp $f gpurun_out/r3l/${n}_stats.csv
  find gpurun_out/r3l/$n -type f ! -name 'kt_kernel_stats.csv' -delete
done
