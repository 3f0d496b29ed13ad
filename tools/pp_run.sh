set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5_v4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "pingpong or gemm256_persistent" > gpurun_out/r5_v4/pytest_pp.log 2>&1
timeout -k 10 200 python3 tools/gemm_epi_bench.py 6 4 > gpurun_out/r5_v4/epi.log 2>&1
