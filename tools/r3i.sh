# tile order: head (row-major, per-stage divisions), gm1 (row-major, hoisted), tree (grouped 8, hoisted)
mkdir -p gpurun_out/r3i
export TMPDIR=/tmp
for r in 1 2; do
  for sh in "3072 768" "768 768" "2304 768" "768 3072"; do
    for lib in ab/libmmseq_head.so ab/libmmseq_gm1.so tree; do
      if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; else export MMSEQ_BENCH_LIB=$lib; fi
      timeout -k 10 60 python -u tools/gemm_one.py $sh plain >> gpurun_out/r3i/time.log 2>&1 || exit 1
    done
  done
done
unset MMSEQ_BENCH_LIB
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3i/f_tree -o f -- python3 tools/gemm_one.py 3072 768 plain 3 > gpurun_out/r3i/f_tree.log 2>&1
