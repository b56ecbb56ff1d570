#!/bin/bash
# Round-3 PMC passes: one counter group per rocprofv3 run, each under its own limit.
mkdir -p gpurun_out/pmc3; export TMPDIR=/tmp
i=0
run() {  # mode counters...
  i=$((i+1)); local mode=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pmc3/p${i}_$mode -o pmc --output-format csv -- python tools/prof_r02.py $mode > gpurun_out/pmc3/p${i}_$mode.log 2>&1 || { echo "pass $i ($mode $*) failed"; tail -5 gpurun_out/pmc3/p${i}_$mode.log; exit 1; }
  echo "pass $i $mode ok"
}
run wino_one SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
run wino_one SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
run mix FETCH_SIZE
run mix WRITE_SIZE
run ns FETCH_SIZE
run ns WRITE_SIZE
run ns SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run upfirdn FETCH_SIZE
run upfirdn WRITE_SIZE
