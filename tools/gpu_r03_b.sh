#!/bin/bash
# r03: new GPU tests, a check that the EMA test catches the r02 behaviour, the full bench
# line, then the PINN graph-replay diagnostic (current vs r02 losses.py).
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_models.py::test_eval_step_between_train_steps_leaves_training_unchanged \
  tests/test_gpu_dist.py::test_bench_gpus_2_matches_world_1_samples > gpurun_out/pytest_b.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_b.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python - > gpurun_out/ema_old.log 2>&1 <<'PY'
import sys; sys.path[:0] = ["tests", "b-pinn-kalman-filter_amd", "."]
import torch
from models.ema import ExponentialMovingAverage as E
def copy_to(self, ps):
    for s, p in zip(self.shadow_params, [p for p in ps if p.requires_grad]): p.data.copy_(s.data)
def restore(self, ps):
    for c, p in zip(self.collected_params, ps): p.data.copy_(c.data)
E.copy_to, E.restore = copy_to, restore
import test_gpu_models as t
try:
    t.test_eval_step_between_train_steps_leaves_training_unchanged(torch.device("cuda:0"))
    print("OLD_EMA_NOT_CAUGHT")
except AssertionError as e:
    print("OLD_EMA_CAUGHT", e)
PY
rc=$?; tail -2 gpurun_out/ema_old.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > gpurun_out/bench_b.log 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 1; }
cat gpurun_out/bench_b.log
timeout -k 10 600 python -u tools/diag_pinn_graph4.py > gpurun_out/diag_pinn_graph4.log 2>&1; rc=$?
tail -14 gpurun_out/diag_pinn_graph4.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in default prio8 sched1 sched2v1 sched3v2; do
  if [ $v = default ]; then L=b-pinn-kalman-filter_amd/lib/libbpk.so; else L=b-pinn-kalman-filter_amd/lib/variants/libbpk_$v.so; fi
  BPK_LIB=$L timeout -k 10 120 python tools/bench_wino_mix.py > gpurun_out/mix_$v.txt 2>&1 || { tail -5 gpurun_out/mix_$v.txt; exit 1; }
  echo "$v $(tail -1 gpurun_out/mix_$v.txt)"
done; done
