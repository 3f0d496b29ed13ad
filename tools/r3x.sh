# attention forward: cross-lane row max only inside the (rare) rescale branch vs HEAD
mkdir -p gpurun_out/r3x
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropout_gpu.py tests/test_fp8_gpu.py -m gpu -k "attention or attn" > gpurun_out/r3x/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r3x/tests.log
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3x/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r3x/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r3x/$n -name 'kt_kernel_stats.csv' | head -n1); cat $f >> gpurun_out/r3x/${n}_stats.csv; rm -rf gpurun_out/r3x/$n
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer >> gpurun_out/r3x/bench_$n.log 2>&1 || exit 1
done
