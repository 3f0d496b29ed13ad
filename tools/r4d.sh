# GPU tests + smoke on the -fno-slp-vectorize build; attention under -amdgpu-sched-strategy=iterative-ilp vs the tree
mkdir -p gpurun_out/r4d
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --maxfail 20 --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4d/pytest_gpu.log 2>&1
echo "tests rc $?" >> gpurun_out/r4d/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d/smoke.log 2>&1
echo "smoke rc $?" >> gpurun_out/r4d/smoke.log
for lib in ab/libmmseq_itilp.so tree ab/libmmseq_itilp.so tree; do
  if [ $lib = tree ]; then unset MMSEQ_BENCH_LIB; n=tree; else export MMSEQ_BENCH_LIB=$lib; n=itilp; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4d/$n -o kt -- python3 tools/attn_bench.py 1 > gpurun_out/r4d/attn_$n.log 2>&1 || exit 1
  f=$(find gpurun_out/r4d/$n -name 'kt_kernel_stats.csv' | head -n1); cat $f >> gpurun_out/r4d/${n}_stats.csv; rm -rf gpurun_out/r4d/$n
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r4d/sq -o sq -- python3 tools/attn_bench.py 1 > gpurun_out/r4d/sq.log 2>&1
python3 tools/pmc_attn_sq.py "$(find gpurun_out/r4d/sq -name '*counter_collection.csv' | head -n1)" gpurun_out/r4d/attn_sq_pmc.json >> gpurun_out/r4d/sq.log 2>&1
rm -rf gpurun_out/r4d/sq
