mkdir -p gpurun_out/r3g
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/r3g/tests.log 2>&1 || exit 1
MMSEQ_BENCH_LIB=ab/libmmseq_base.so timeout -k 10 300 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3g/epi_base.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3g/epi_new.log 2>&1
