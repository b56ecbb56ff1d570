#!/bin/bash
# r03: the 16-cin chunk 8-wave Winograd kernel (BPK_WINO_K16): conv parity with it forced on
# every supported launch, then the weighted PRE-conv mix A/B vs the 8-cin form.
mkdir -p gpurun_out; export TMPDIR=/tmp
BPK_WINO_K16=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "conv3x3_winograd" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/k16_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/k16_pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do for v in 0 1; do
  BPK_WINO_K16=$v timeout -k 10 120 python tools/bench_wino_mix.py > gpurun_out/mix_k16_$v.txt 2>&1 || { tail -5 gpurun_out/mix_k16_$v.txt; exit 1; }
  echo "K16=$v $(tail -1 gpurun_out/mix_k16_$v.txt)"
done; done
cat gpurun_out/mix_k16_1.txt
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_models.py::test_eval_step_between_train_steps_leaves_training_unchanged \
  tests/test_gpu_pinn.py::test_pinn_step_graph_replay_matches_eager > gpurun_out/pytest_c.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_c.log; [ $rc -eq 0 ] || exit $rc
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
rc=$?; tail -1 gpurun_out/ema_old.log; [ $rc -eq 0 ] || exit $rc
B=64 timeout -k 10 600 python -u tools/diag_pinn_graph4.py > gpurun_out/diag_pinn_graph4_b64.log 2>&1; rc=$?
grep -v Warning gpurun_out/diag_pinn_graph4_b64.log | tail -12; [ $rc -eq 0 ] || exit $rc
