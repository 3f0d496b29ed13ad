# MX-fp8 GEMM: F8 LDS re-layout + Q8 scale stores through a descriptor (no spills) vs HEAD
mkdir -p gpurun_out/r3y
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_fp8_gpu.py tests/test_kernels_gpu.py tests/test_realshape_gpu.py -m gpu > gpurun_out/r3y/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3y/tests.log
for lib in ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 200 python3 tools/fp8_bench.py > gpurun_out/r3y/fp8_$n.json 2>&1 || exit 1
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  for mode in bf16 mxfp8; do
    timeout -k 10 300 python3 tools/c5_eval.py $mode 5 >> gpurun_out/r3y/c5_$n.log 2>&1 || exit 1
  done
done
