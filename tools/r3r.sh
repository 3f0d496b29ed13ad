# fp8 eval path with fused LayerNorm -> MX-fp8: config-5 + fp8 tests, eval A/B, kernel stats
mkdir -p gpurun_out/r3r
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_realshape_gpu.py tests/test_fp8_gpu.py -m gpu -k "config5 or fp8 or mxfp8" > gpurun_out/r3r/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3r/tests.log
for mode in bf16 mxfp8 bf16 mxfp8; do timeout -k 10 300 python3 tools/c5_eval.py $mode 5 >> gpurun_out/r3r/c5.log 2>&1 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r/kt -o kt -- python3 tools/c5_eval.py mxfp8 3 > gpurun_out/r3r/kt.log 2>&1 || exit 1
cp "$(find gpurun_out/r3r/kt -name 'kt_kernel_stats.csv' | head -n1)" gpurun_out/r3r/mxfp8_kernel_stats.csv; rm -rf gpurun_out/r3r/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3r/kt -o kt -- python3 tools/c5_eval.py bf16 3 > gpurun_out/r3r/kt.log 2>&1 || exit 1
cp "$(find gpurun_out/r3r/kt -name 'kt_kernel_stats.csv' | head -n1)" gpurun_out/r3r/bf16_kernel_stats.csv; rm -rf gpurun_out/r3r/kt
