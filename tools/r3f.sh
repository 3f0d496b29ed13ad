mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u tools/gemm_census.py > gpurun_out/r3f/census.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/gemm_epi_bench.py 4 > gpurun_out/r3f/epi.log 2>&1
