"""HIP runtime settings the hipGraph paths depend on (imported before anything touches the
device: op/__init__, bench.py, __graft_entry__.py and tests/conftest.py import it first).

The HIP runtime reads these when it initializes -- the first HIP call of the process -- so
they are set in the environment here, before torch initializes the device.

DEBUG_CLR_GRAPH_PACKET_CAPTURE=0.  By default this runtime ("graph packet capture")
pre-builds the AQL packets of a graph's kernel nodes with their kernel arguments placed in the
device kernel-argument pool, the same ring buffer every eagerly launched kernel writes its
arguments into.  Once eager launches after the capture have written about the pool's size of
arguments, the ring wraps over the graph's, and later replays run the graph's kernels with
other launches' arguments: silently wrong results, no fault.  Measured (tools/audit_pinn_graph.py,
profiles/r05_pinn_graph_iso.txt): the PINN step graph replayed with fixed inputs stays
bit-identical with 2000 small-argument fills, hipMemsetAsync or D2H reads between replays, and
goes wrong after 8-19 replays with eager kernels carrying large argument blocks between them
(reductions, non-contiguous elementwise ops: 800 KB-1 MB of arguments).  The same failing run
is bit-stable with this variable at 0 (the packets are rebuilt per replay,
the PINN replay time unchanged: 84.4 vs 84.0 ms) or with a 64 MB pool (HSA_KERNARG_POOL_SIZE:
only delays the wrap).  The audit of every pointer the captured step reads found no aliasing:
all of them lie in the graph's private pool or in live tensors (profiles/r05_pinn_graph_audit.json).
The PC sampler's step graph (B = 8, 24 steps, the same large-argument launches between steps)
stayed bit-identical to the run without them with the setting at 1 and at 0 (round 5) -- not
shown vulnerable, covered by the setting all the same.
"""
from __future__ import annotations

import os
import sys

GRAPH_PACKET_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"
_PRESET = os.environ.get(GRAPH_PACKET_CAPTURE)
os.environ.setdefault(GRAPH_PACKET_CAPTURE, "0")
# HIP was already initialized when this module was first imported (too late for the setting to
# take effect) -- only knowable through torch, if it is loaded
_torch = sys.modules.get("torch")
_LATE = _PRESET is None and _torch is not None and _torch.cuda.is_initialized()


def graph_replays_safe() -> bool:
    """True when this process's hipGraph replays do not read kernel arguments from the eager
    launch ring (the setting above is in effect)."""
    return os.environ.get(GRAPH_PACKET_CAPTURE) == "0" and not _LATE


_WARNED = [False]


def warn_if_unsafe(what: str) -> None:
    if graph_replays_safe() or _WARNED[0]:
        return
    _WARNED[0] = True
    import warnings
    warnings.warn(f"{what}: this process's HIP runtime captures graph kernel packets with their "
                  f"arguments in the eager launch ring ({GRAPH_PACKET_CAPTURE} is not 0 when the "
                  "runtime initialized); replays may read other launches' arguments once eager "
                  "work has filled the ring.  Import `op` (or set "
                  f"{GRAPH_PACKET_CAPTURE}=0) before the first device call.", RuntimeWarning,
                  stacklevel=3)
