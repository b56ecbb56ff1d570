#!/bin/bash
# Round 5: wgrad V-record stride 20 -> 24 floats -- wgrad / GN-conv tests, SQ bank-conflict pass,
# wgrad kernel time (128->128 @128^2, B=16), DSM train + CIFAR bench phases.
mkdir -p gpurun_out/r05n; export TMPDIR=/tmp
O=gpurun_out/r05n
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "weight_gradient or gn_silu or wgrad" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o pmc --output-format csv -- python3 tools/prof_r02.py wgrad_one > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o wg --output-format csv -- python3 tools/prof_r02.py wgrad_one > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-pinn --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
