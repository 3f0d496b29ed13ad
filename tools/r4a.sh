# NT GEMM bias through LDS-DMA before the K-loop (no epilogue-start vmcnt(0)) vs HEAD
mkdir -p gpurun_out/r4a
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4a/tests.log 2>&1
echo "tests rc $?" >> gpurun_out/r4a/tests.log
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 200 python3 tools/gemm_epi_bench.py 4 >> gpurun_out/r4a/epi_$n.log 2>&1 || exit 1
done
for lib in ab/libmmseq_head.so tree ab/libmmseq_head.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=head; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer >> gpurun_out/r4a/bench_$n.log 2>&1 || exit 1
done
