# forward attention at 2 vs 3 workgroups per CU (LDS-padded build): is the tail fold's occupancy cost affordable?
mkdir -p gpurun_out/r3o
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for lib in ab/libmmseq_fwd3.so ab/libmmseq_fwd2.so ab/libmmseq_fwd3.so ab/libmmseq_fwd2.so; do
  export MMSEQ_BENCH_LIB=$lib
  echo "== $lib" >> gpurun_out/r3o/attn.log
  timeout -k 10 120 python -u tools/attn_bench.py 1 >> gpurun_out/r3o/attn.log 2>&1 || exit 1
done
