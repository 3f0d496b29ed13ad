# full GPU suite; attention A/B (HEAD build vs tree); default bench
mkdir -p gpurun_out/r3n
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu --maxfail 20 > gpurun_out/r3n/pytest_gpu.log 2>&1
echo "suite rc $?" >> gpurun_out/r3n/pytest_gpu.log
for lib in ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r3n/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r3n/$n -name 'kt_kernel_stats.csv' | head -n1); cp $f gpurun_out/r3n/${n}_stats.csv; rm -rf gpurun_out/r3n/$n
done
unset MMSEQ_BENCH_LIB
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r3n/bench.log 2>&1
