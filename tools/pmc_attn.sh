set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for v in 1 2; do
  export ATTN_VARIANT=$v
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc_att$v -o p1 -- python3 tools/attn_one.py 512 > gpurun_out/pmc_att$v.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d gpurun_out/pmc_att$v -o p2 -- python3 tools/attn_one.py 512 >> gpurun_out/pmc_att$v.log 2>&1
done
