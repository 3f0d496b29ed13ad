# attention changes: kernel tests, then A/B timing against ab/libmmseq_base.so on the same box
mkdir -p gpurun_out/r3c
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropout_gpu.py -k "attention" -m gpu > gpurun_out/r3c/attn_tests.log 2>&1 || exit 1
for r in 1 2; do
  MMSEQ_BENCH_LIB=ab/libmmseq_base.so timeout -k 10 120 python -u tools/attn_bench.py 1 > gpurun_out/r3c/attn_base_$r.log 2>&1 || exit 1
  timeout -k 10 120 python -u tools/attn_bench.py 1 > gpurun_out/r3c/attn_new_$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/gemm_epi_bench.py 4 5 > gpurun_out/r3c/epi.log 2>&1
