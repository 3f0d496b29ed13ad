# attention prologues: branch-free buffer loads issued before the first use (one round trip) vs HEAD
mkdir -p gpurun_out/r3z
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropout_gpu.py tests/test_fp8_gpu.py tests/test_realshape_gpu.py tests/test_parity_gpu.py -m gpu > gpurun_out/r3z/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3z/tests.log
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3z/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r3z/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r3z/$n -name 'kt_kernel_stats.csv' | head -n1); cat $f >> gpurun_out/r3z/${n}_stats.csv; rm -rf gpurun_out/r3z/$n
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer >> gpurun_out/r3z/bench_$n.log 2>&1 || exit 1
done
