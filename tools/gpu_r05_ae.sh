#!/bin/bash
# Round 5: 1x1 MFMA GEMM with four K-chunks in flight -- GEMM / 1x1 / model tests, sampler
# kernel trace (1x1 launch times), bench phases (sampler, CIFAR, DPS, PINN) and the per-rank B=8.
mkdir -p gpurun_out/r05ae; export TMPDIR=/tmp
O=gpurun_out/r05ae
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -x -q --timeout 300 --timeout-method thread -k "gemm or conv1x1 or nin or attention or ncsnpp or ddpm" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/b64 -o b64 --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-train --no-pinn --no-dps --cifar-steps 0 --ns-steps 0 --ncddpmpp-steps 0 --no-roofline > $O/b64.log 2>&1 || { tail -5 $O/b64.log; exit 1; }
timeout -k 10 900 python bench.py --no-cpu-baseline --ns-steps 0 --no-train > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python tools/show_line.py $O/bench.log | head -2
timeout -k 10 600 python bench.py --no-cpu-baseline --ns-steps 0 --ncddpmpp-steps 0 --no-pinn --no-dps --cifar-steps 0 --per-rank-of 8 > $O/bench8.log 2> $O/bench8.err || { tail -20 $O/bench8.err; exit 1; }
python tools/show_line.py $O/bench8.log | head -2
