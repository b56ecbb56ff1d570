"""Which autograd nodes issue the PINN step's aten launches (configs[3], B=64, one eager step):
every aten op under a TorchDispatchMode, keyed by (op, the autograd node running it or
"<forward>"), sorted by count.  The engine's own gradient accumulation shows up under the
node whose output it accumulates."""
import collections
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402
from dist import DistContext  # noqa: E402

SKIP = {"empty", "empty_strided", "view", "_unsafe_view", "detach", "t", "as_strided",
        "expand", "reshape", "permute", "transpose", "unsqueeze", "squeeze", "slice", "select",
        "alias", "_reshape_alias", "lift_fresh", "split", "unbind", "is_same_size"}
cnt = collections.Counter()
sites = collections.Counter()  # (op, innermost repo frame) of the ops issued outside any node
TRACE = {"clone", "zeros_like", "zeros", "add", "mul", "_to_copy", "div", "copy_", "sum",
         "empty_like"}


def _site():
    import traceback
    for fr in reversed(traceback.extract_stack()[:-3]):
        if REPO in fr.filename and "pinn_op_sources" not in fr.filename:
            return f"{os.path.relpath(fr.filename, REPO)}:{fr.lineno} {fr.line}"
    return "?"


class Mode(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.overloadpacket.__name__
        if name not in SKIP:
            node = torch._C._current_autograd_node()
            cnt[(name, node.name() if node is not None else "<forward>")] += 1
            if node is None and name in TRACE:
                sites[(name, _site())] += 1
        return func(*args, **(kwargs or {}))


class A:
    pass


args = A()
args.batch = None
args.weak = False
args.per_rank_of = int(sys.argv[1]) if len(sys.argv) > 1 else None  # 8: the B = 8 rank
args.pinn_warmup, args.pinn_steps, args.pinn_eager = 1, 1, True
dev = torch.device("cuda:0")
bench.bench_pinn(args, DistContext(), dev)  # warm (conv choices, filter caches)
args.pinn_warmup = 0
with Mode():
    bench.bench_pinn(args, DistContext(), dev)
tot = sum(cnt.values())
print(f"{tot} aten ops (views skipped)")
by_op = collections.Counter()
for (op, _), v in cnt.items():
    by_op[op] += v
print("by op:", by_op.most_common(25))
for (op, node), v in cnt.most_common(60):
    print(f"{v:6d}  {op:28s} {node}")
print("ops outside any autograd node, by call site:")
for (op, site), v in sites.most_common(40):
    print(f"{v:6d}  {op:12s} {site}")
