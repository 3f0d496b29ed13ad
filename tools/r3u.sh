# GELU / QuickGELU gate table in the NT forward epilogues vs the fitted logistic (A/B: ab/libmmseq_gfit.so)
mkdir -p gpurun_out/r3u
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp8_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/r3u/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3u/tests.log
for lib in ab/libmmseq_gfit.so tree ab/libmmseq_gfit.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3u/epi.log
  timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 >> gpurun_out/r3u/epi.log 2>&1 || exit 1
done
for lib in ab/libmmseq_gfit.so tree ab/libmmseq_gfit.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3u/bench.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer >> gpurun_out/r3u/bench.log 2>&1 || exit 1
done
