# -fno-slp-vectorize (no compiler-packed v_pk_* f32 ops beside the MFMAs) vs HEAD: attention + GEMM + bench
mkdir -p gpurun_out/r4c
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in ab/libmmseq_noslp.so tree ab/libmmseq_noslp.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=noslp; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4c/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r4c/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r4c/$n -name 'kt_kernel_stats.csv' | head -n1); cat $f >> gpurun_out/r4c/${n}_stats.csv; rm -rf gpurun_out/r4c/$n
  timeout -k 10 200 python3 tools/gemm_epi_bench.py 4 >> gpurun_out/r4c/epi_$n.log 2>&1 || exit 1
done
for lib in ab/libmmseq_noslp.so tree ab/libmmseq_noslp.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=noslp; fi
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-config2 --no-config5 --no-rn50 --no-gemm-timer --fwd-steps 0 >> gpurun_out/r4c/bench_$n.log 2>&1 || exit 1
done
