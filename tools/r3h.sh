# grouped tile order (tree) vs row-major (ab/libmmseq_head.so): timing and FETCH_SIZE per launch
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
for r in 1 2; do
  for sh in "3072 768" "768 768" "2304 768" "768 3072"; do
    MMSEQ_BENCH_LIB=ab/libmmseq_head.so timeout -k 10 60 python -u tools/gemm_one.py $sh plain >> gpurun_out/r3h/time.log 2>&1 || exit 1
    timeout -k 10 60 python -u tools/gemm_one.py $sh plain >> gpurun_out/r3h/time.log 2>&1 || exit 1
  done
done
for lib in head tree; do
  if [ $lib = head ]; then export MMSEQ_BENCH_LIB=ab/libmmseq_head.so; else unset MMSEQ_BENCH_LIB; fi
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3h/f_$lib -o f -- python3 tools/gemm_one.py 3072 768 plain 3 > gpurun_out/r3h/f_$lib.log 2>&1 || exit 1
done
