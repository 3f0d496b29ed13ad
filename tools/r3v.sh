# GELU / QuickGELU non-temporal epilogue stores (A/B: ab/libmmseq_ntst.so)
mkdir -p gpurun_out/r3v
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in ab/libmmseq_ntst.so tree ab/libmmseq_ntst.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3v/epi.log
  timeout -k 10 200 python -u tools/gemm_epi_bench.py 4 >> gpurun_out/r3v/epi.log 2>&1 || exit 1
done
for lib in ab/libmmseq_ntst.so tree ab/libmmseq_ntst.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
  echo "== $lib" >> gpurun_out/r3v/bench.log
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer >> gpurun_out/r3v/bench.log 2>&1 || exit 1
done
