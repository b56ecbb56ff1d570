#!/bin/bash
# Round 5: igemm weight gradient with the 32-bit offsets, wave-uniform k, unconditional TAP loads --
# igemm tests, kernel times + SQ counters of the igemm shape set, PINN bench + kernel count.
mkdir -p gpurun_out/r05s; export TMPDIR=/tmp
O=gpurun_out/r05s
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread -k "igemm or conv2d or small_cout or wgrad" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o ig --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d $O/sq1 -o pmc --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/sq1.log 2>&1 || { tail -5 $O/sq1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/sq2 -o pmc --output-format csv -- python3 tools/prof_r02.py igemm_set > $O/sq2.log 2>&1 || { tail -5 $O/sq2.log; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-dps --no-train --cifar-steps 0 --steps 1 --warmup 1 > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/pinn64 -o pinn --output-format csv -- python3 tools/prof_pinn.py > $O/pinn64.log 2>&1 || { tail -5 $O/pinn64.log; exit 1; }
python tools/trace_steps.py $O/pinn64/pinn_kernel_trace.csv 7 30
