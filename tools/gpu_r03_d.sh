#!/bin/bash
# r03: EMA + PINN-graph tests, the r02-EMA detection check, PINN graph diag at B=64, K16 on
# every supported launch (residual-tail and plain forms) vs K16 for the PRE+stats form only,
# and the per-workgroup timeline of the K16 kernel.
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_models.py::test_eval_step_between_train_steps_leaves_training_unchanged \
  tests/test_gpu_pinn.py::test_pinn_step_graph_replay_matches_eager > gpurun_out/pytest_d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_d.log; [ $rc -eq 0 ] || exit $rc
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
for v in 1 2; do
  BPK_WINO_K16=$v timeout -k 10 120 python tools/bench_wino_mix.py > gpurun_out/mix_k16_$v.txt 2>&1 || { tail -5 gpurun_out/mix_k16_$v.txt; exit 1; }
  echo "K16=$v"; cat gpurun_out/mix_k16_$v.txt
done
for v in 0 1; do
  echo "### timeline K16=$v"
  BPK_WINO_K16=$v WINO_TIMING_LIB=b-pinn-kalman-filter_amd/lib/libbpk_wino_timing_k16.so timeout -k 10 120 python tools/wino_timing.py 128 128 128 256 256 64 512 256 64 > gpurun_out/tl_k16_$v.txt 2>&1 || { tail -5 gpurun_out/tl_k16_$v.txt; exit 1; }
  grep "==\|  loop\|  prologue \|  epilogue" gpurun_out/tl_k16_$v.txt
done
B=64 timeout -k 10 600 python -u tools/diag_pinn_graph4.py > gpurun_out/diag_pinn_graph4_b64.log 2>&1; rc=$?
grep -v Warning gpurun_out/diag_pinn_graph4_b64.log | tail -12; [ $rc -eq 0 ] || exit $rc
