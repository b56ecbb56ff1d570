#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
for rt in 8 4 2; do
BPK_UPFIRDN_RT=$rt timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -q -k "upfirdn" -p no:cacheprovider 2>&1 | tail -1 || exit 1
done
for rt in 8 4 2 8 4 2; do
BPK_UPFIRDN_RT=$rt timeout -k 10 300 python -c "
import sys, json, torch; sys.argv=['bench']
import bench
r = bench.upfirdn_rooflines(torch.device('cuda:0'), 64)[3]; print('RT=$rt', r['ms_per_launch'], r['frac'])
" || exit 1
done
