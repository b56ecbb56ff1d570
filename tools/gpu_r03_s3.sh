#!/bin/bash
# r03 session 2: upfirdn2d rolling kernel with 1-3 rows of loads in flight (BPK_UPFIRDN_PF) and
# taller strips: parity tests under each PF, then the four-shape A/B twice (interleaved).
mkdir -p gpurun_out; export TMPDIR=/tmp
V="BPK_UPFIRDN_PF=2 BPK_UPFIRDN_PF=3 BPK_UPFIRDN_PF=2,BPK_UPFIRDN_ROLL=8 BPK_UPFIRDN_PF=3,BPK_UPFIRDN_ROLL=8 BPK_UPFIRDN_PF=3,BPK_UPFIRDN_ROLL=16"
TESTENV="BPK_UPFIRDN_PF=2 BPK_UPFIRDN_PF=3" bash tools/gpu_upfirdn_roll.sh $V || exit 1
bash tools/gpu_upfirdn_ab.sh $V || exit 1
