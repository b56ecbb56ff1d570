#!/bin/bash
# PMC passes over the pipelined Winograd conv (tools/prof_traffic.py: 10 conv + 10 upfirdn2d
# launches): HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes) and SQ stall counters.
# One counter group per pass, each pass under its own time limit.
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
    "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d gpurun_out/pmc/p$i -o pmc --output-format csv -- python tools/prof_traffic.py > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
