# fp8 eval path with all four encoder GEMMs on the fp8 MFMA: config-5 tests, fp8 tests, eval A/B
mkdir -p gpurun_out/r3q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -s --timeout 200 --timeout-method thread tests/test_realshape_gpu.py tests/test_fp8_gpu.py -m gpu -k "config5 or fp8 or mxfp8" > gpurun_out/r3q/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3q/tests.log
for mode in bf16 mxfp8 bf16 mxfp8; do timeout -k 10 300 python3 tools/c5_eval.py $mode 5 >> gpurun_out/r3q/c5.log 2>&1 || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3q/kt -o kt -- python3 tools/c5_eval.py mxfp8 3 > gpurun_out/r3q/kt.log 2>&1 || exit 1
cp "$(find gpurun_out/r3q/kt -name 'kt_kernel_stats.csv' | head -n1)" gpurun_out/r3q/mxfp8_kernel_stats.csv; rm -rf gpurun_out/r3q/kt
