#!/bin/bash
# r03 first box: the new GPU tests (EMA/eval interleave, bench --gpus 2 vs 1), then the default bench line.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_models.py::test_eval_step_between_train_steps_leaves_training_unchanged \
  tests/test_gpu_dist.py::test_bench_gpus_2_matches_world_1_samples > gpurun_out/pytest_a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_a.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_a.log 2> gpurun_out/bench_a.err || { tail -20 gpurun_out/bench_a.err; exit 1; }
cat gpurun_out/bench_a.log
