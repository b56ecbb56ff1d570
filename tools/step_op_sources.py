"""Which autograd nodes issue a bench step's aten launches: the step bench.py counts FLOPs on
(bench.counted, one eager step after the warm-up) runs under a TorchDispatchMode; every aten op
is keyed by (op, the autograd node running it or "<forward>"), ops outside any node also by
their innermost repo call site.  python tools/step_op_sources.py cifar|pinn|dps (configs[1]
train step / configs[3] PINN step / one configs[5] DPS function evaluation; the DSM 128^2 step runs the NCSN++ family inside bench.main)"""
import collections
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
from op import _hipenv  # noqa: E402,F401
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402
import dist  # noqa: E402

SKIP = {"empty", "empty_strided", "view", "_unsafe_view", "detach", "t", "as_strided",
        "expand", "reshape", "permute", "transpose", "unsqueeze", "squeeze", "slice", "select",
        "alias", "_reshape_alias", "lift_fresh", "split", "unbind", "is_same_size"}
cnt, sites = collections.Counter(), collections.Counter()


def _site():
    for fr in reversed(traceback.extract_stack()[:-3]):
        if (REPO in fr.filename and "step_op_sources" not in fr.filename
                and not fr.filename.endswith("op/flops.py")):
            return f"{os.path.relpath(fr.filename, REPO)}:{fr.lineno} {fr.line}"
    return "?"


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in SKIP:
            node = torch._C._current_autograd_node()
            key = node.name() if node is not None else "<forward>"
            cnt[(name, key)] += 1
            sites[(name, key if node is not None else _site())] += 1
        return func(*args, **(kwargs or {}))


_counted = bench.counted


def counted(fn, dev):
    with Mode():
        return _counted(fn, dev)


bench.counted = counted
which = sys.argv[1]
extra = sys.argv[2:]  # e.g. --per-rank-of 8
sys.argv = ["bench.py", "--cifar-steps", "1", "--pinn-steps", "1", "--pinn-warmup", "1",
            "--dps-steps", "1"] + extra
args = bench.parse()
ctx = dist.init_from_env()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
{"cifar": bench.bench_cifar_train, "pinn": bench.bench_pinn, "dps": bench.bench_dps}[which](
    args, ctx, dev)
tot = sum(cnt.values())
print(f"{which}: {tot} aten ops in one step (views skipped)")
by_op = collections.Counter()
for (op, _), v in cnt.items():
    by_op[op] += v
print("by op:", by_op.most_common(25))
for (op, node), v in cnt.most_common(40):
    print(f"{v:6d}  {op:28s} {node}")
print("every (op, node) of the launch-heavy ops:")
for (op, node), v in sorted(cnt.items(), key=lambda kv: (kv[0][0], -kv[1])):
    if op in ("clone", "copy_", "add", "zeros_like", "zeros", "mul", "div", "neg", "sum", "cat",
              "linalg_vector_norm", "_to_copy", "fill_"):
        print(f"{v:6d}  {op:12s} {node}")
print("ops outside any autograd node, by call site:")
for (op, site), v in sites.most_common(60):
    if not site.startswith(("_", "torch::")) and "Backward" not in site:
        print(f"{v:6d}  {op:12s} {site}")
