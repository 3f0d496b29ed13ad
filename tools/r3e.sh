# GELU' epilogue + forward attention: kernel tests, epilogue A/B, full bench
mkdir -p gpurun_out/r3e
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/r3e/tests.log 2>&1 || exit 1
MMSEQ_BENCH_LIB=ab/libmmseq_base.so timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3e/epi_base.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3e/epi_new.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3e/bench.log 2>&1
