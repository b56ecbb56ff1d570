#!/bin/bash
# Round 4: rocprofv3 kernel trace of the DSM train step (NCSN++ 128^2, B = 64; 5 steps) on the
# current tree.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04_train -o train --output-format csv -- python tools/prof_train.py > gpurun_out/prof_r04_train.log 2>&1 || { tail gpurun_out/prof_r04_train.log; exit 1; }
echo PROF_TRAIN_OK
