# forward attention (permlane max, MFMA row sums) + sigmoid-form GELU epilogue: tests, then A/B
mkdir -p gpurun_out/r3d
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropout_gpu.py -m gpu > gpurun_out/r3d/tests.log 2>&1 || exit 1
for r in 1 2; do
  MMSEQ_BENCH_LIB=ab/libmmseq_base.so timeout -k 10 120 python -u tools/attn_bench.py 1 > gpurun_out/r3d/attn_base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/attn_bench.py 1 > gpurun_out/r3d/attn_new_$r.log 2>&1 || exit 1
  MMSEQ_BENCH_LIB=ab/libmmseq_base.so timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3d/epi_base_$r.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3d/epi_new_$r.log 2>&1 || exit 1
done
