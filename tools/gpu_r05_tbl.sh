#!/bin/bash
# Round 5: why the CIFAR phase of a full bench run measures 13.2 or 14.5 steps/s -- the conv
# choices (BPK_CONV_TABLE records them) of full runs vs a sampler + train + CIFAR run.
mkdir -p gpurun_out/r05tbl; export TMPDIR=/tmp
O=gpurun_out/r05tbl
rm -f $O/*.json
BPK_CONV_TABLE=$O/tbl_full2.json timeout -k 10 900 python bench.py --no-cpu-baseline --ns-steps 0 > $O/full2.log 2> $O/full2.err || { tail -20 $O/full2.err; exit 1; }
python tools/show_line.py $O/full2.log | head -1
BPK_CONV_TABLE=$O/tbl_tc.json timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-pinn --no-dps --steps 1 --warmup 1 > $O/tc.log 2> $O/tc.err || { tail -20 $O/tc.err; exit 1; }
python tools/show_line.py $O/tc.log | head -1
