mkdir -p gpurun_out/r3j
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_fp8_gpu.py -m gpu > gpurun_out/r3j/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3j/bench.log 2>&1
