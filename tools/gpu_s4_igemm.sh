#!/bin/bash
# igemm conv milestone: its parity tests + the model-level GPU tests that run through it,
# then the bench (no CPU baseline) and steady-state kernel breakdowns of the PINN and CIFAR
# train steps.  Each GPU step has its own limit; stop at the first failure.
mkdir -p gpurun_out; export TMPDIR=/tmp
export MIOPEN_CUSTOM_CACHE_DIR=$PWD/b-pinn-kalman-filter_amd/miopen_cache/kernels MIOPEN_USER_DB_PATH=$PWD/b-pinn-kalman-filter_amd/miopen_cache/db
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_pinn.py tests/test_gpu_configs.py tests/test_gpu_models.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_s4.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_s4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_s4.log 2> gpurun_out/bench_s4.err || { tail -20 gpurun_out/bench_s4.err; exit 1; }
cat gpurun_out/bench_s4.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pinn -o pinn --output-format csv -- python tools/prof_pinn.py > gpurun_out/prof_pinn.log 2>&1 || { tail gpurun_out/prof_pinn.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_pinn/pinn_kernel_trace.csv gs_grad2 0 2 3 45 > gpurun_out/pinn_steady.txt
rm -f gpurun_out/prof_pinn/pinn_kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cifar -o cifar --output-format csv -- python tools/prof_cifar.py > gpurun_out/prof_cifar.log 2>&1 || { tail gpurun_out/prof_cifar.log; exit 1; }
python tools/slice_trace.py gpurun_out/prof_cifar/cifar_kernel_trace.csv multi_tensor_apply 0 2 3 45 > gpurun_out/cifar_steady.txt
rm -f gpurun_out/prof_cifar/cifar_kernel_trace.csv
head -30 gpurun_out/pinn_steady.txt gpurun_out/cifar_steady.txt
