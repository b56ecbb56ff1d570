#!/bin/bash
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py -m gpu -q -k "rccl or sampler" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dist.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dist.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_roofline_mix_prof.sh
