#!/bin/bash
# Round 4: SQ counters of the implicit-GEMM forward on the CIFAR-10 8^2 level shape
# (B = 128, 256 -> 256, 3x3): issue mix and busy cycles, two passes.
mkdir -p gpurun_out/igpmc; export TMPDIR=/tmp
A="fwd 128 256 8 8 256 3 1 1 20"
timeout -k 10 120 python tools/igemm_one.py $A || exit 1
timeout -k 10 120 python tools/igemm_one.py dgrad 128 256 8 8 256 3 1 1 20 || exit 1
timeout -k 10 120 python tools/igemm_one.py wgrad 128 256 8 8 256 3 1 1 20 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/igpmc/p1 -o pmc --output-format csv -- python tools/igemm_one.py $A > gpurun_out/igpmc/p1.log 2>&1 || { tail gpurun_out/igpmc/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/igpmc/p2 -o pmc --output-format csv -- python tools/igemm_one.py $A > gpurun_out/igpmc/p2.log 2>&1 || { tail gpurun_out/igpmc/p2.log; exit 1; }
echo PMC_OK
