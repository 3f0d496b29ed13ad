# bisect the bf16 decisive-margin regression across builds; attention dQ tail-fold A/B; full GPU suite
mkdir -p gpurun_out/r3k
export PYTHONUNBUFFERED=1
for lib in ab/libmmseq_c451d3e.so ab/libmmseq_1c3d01d.so ab/libmmseq_f64a72b.so ab/libmmseq_head.so; do
  export MMSEQ_BENCH_LIB=$lib
  echo "== $lib" >> gpurun_out/r3k/bisect.log
  timeout -k 10 200 python -u -m pytest -q -s --timeout 150 --timeout-method thread tests/test_order_gpu.py -m gpu -k bf16 >> gpurun_out/r3k/bisect.log 2>&1
  rc=$?; echo "rc $rc" >> gpurun_out/r3k/bisect.log; [ $rc -le 1 ] || exit 1
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_nofold.so ab/libmmseq_head.so tree ab/libmmseq_nofold.so; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3k/attn.log
  timeout -k 10 120 python -u tools/attn_bench.py 1 >> gpurun_out/r3k/attn.log 2>&1 || exit 1
done
unset MMSEQ_BENCH_LIB
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --maxfail 30 > gpurun_out/r3k/pytest_gpu.log 2>&1
echo "suite rc $?"
