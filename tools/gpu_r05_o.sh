#!/bin/bash
# Round 5: where the PINN step's implicit-GEMM time goes -- per-node aten attribution of one
# eager step, kernel times and SQ counters of the heaviest igemm shapes.
mkdir -p gpurun_out/r05o; export TMPDIR=/tmp
O=gpurun_out/r05o
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o ig --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o pmc --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/sq2 -o pmc --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
timeout -k 10 300 python tools/pinn_op_sources.py > $O/pinn_ops.log 2>&1 || { tail -5 $O/pinn_ops.log; exit 1; }
echo done
