#!/bin/bash
# r03 session 2: FIR pad(2,2) rolling kernel with the strip's output rows kept in registers
# and stored after its last row (BPK_UPFIRDN_FIR_RB=1): parity tests with it on, then the
# four-shape A/B twice
mkdir -p gpurun_out; export TMPDIR=/tmp
TESTENV="BPK_UPFIRDN_FIR_RB=1" bash tools/gpu_upfirdn_roll.sh BPK_UPFIRDN_FIR_RB=1 || exit 1
bash tools/gpu_upfirdn_ab.sh BPK_UPFIRDN_FIR_RB=1 || exit 1
