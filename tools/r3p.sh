# fp8 8-phase kernel: correctness (fp8 tests), GEMM A/B vs the old fp8 kernels and bf16, config-5 eval
mkdir -p gpurun_out/r3p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fp8_gpu.py -m gpu > gpurun_out/r3p/tests.log 2>&1 || exit 1
for lib in ab/libmmseq_f8old.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3p/gemm.log
  timeout -k 10 200 python -u tools/fp8_bench.py >> gpurun_out/r3p/gemm.log 2>&1 || exit 1
done
unset MMSEQ_BENCH_LIB
for mode in bf16 mxfp8; do timeout -k 10 300 python3 tools/c5_eval.py $mode 5 >> gpurun_out/r3p/c5.log 2>&1 || exit 1; done
