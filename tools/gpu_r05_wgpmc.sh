#!/bin/bash
# Round 5: SQ counters of the Winograd weight gradient (one 128->128 @128^2 launch, B=16)
mkdir -p gpurun_out/pmc_wg; export TMPDIR=/tmp; rm -rf gpurun_out/pmc_wg/sq1 gpurun_out/pmc_wg/sq2
D=gpurun_out/pmc_wg
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $D/sq1 -o pmc --output-format csv -- python3 tools/prof_r02.py wgrad_one > $D/sq1.log 2>&1 || { tail -5 $D/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $D/sq2 -o pmc --output-format csv -- python3 tools/prof_r02.py wgrad_one > $D/sq2.log 2>&1 || { tail -5 $D/sq2.log; exit 1; }
echo done
