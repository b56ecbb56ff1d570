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

GRAPH_PACKET_CAPTURE = "DEBUG_CLR_GRAPH_PACKET_CAPTURE"


def _runtime_started() -> bool:
    """True when the ROCm runtime of this process has already initialized, i.e. holds the KFD
    device node open.  The HIP runtime reads its DEBUG_CLR_* settings in its init, which opens
    /dev/kfd (hipInit -> ROCr hsa_init) -- so an environment setting made while no descriptor
    of this process points at /dev/kfd is in effect.  torch.cuda.is_initialized() is not
    enough: torch.cuda.is_available() / device_count() start the HIP runtime without
    initializing torch's CUDA state.  Unknowable (no /proc): assume started."""
    try:
        fds = os.listdir("/proc/self/fd")
    except OSError:
        return True
    for fd in fds:
        try:
            if os.readlink(f"/proc/self/fd/{fd}") == "/dev/kfd":
                return True
        except OSError:
            continue
    return False


_PRESET = os.environ.get(GRAPH_PACKET_CAPTURE)
_STARTED = _runtime_started()
os.environ.setdefault(GRAPH_PACKET_CAPTURE, "0")
# the setting is proven in effect only if it was in the environment before the runtime started:
# preset by the caller, or set here while the runtime was not yet up
_PROVEN = _PRESET == "0" or (_PRESET is None and not _STARTED)


def graph_replays_safe() -> bool:
    """True when this process's hipGraph replays provably do not read kernel arguments from the
    eager launch ring (the setting above was in the environment before the runtime started)."""
    return _PROVEN and os.environ.get(GRAPH_PACKET_CAPTURE) == "0"


_WARNED = set()


def graphs_allowed(what: str) -> bool:
    """The hipGraph paths (PCEngine(use_graph=True), get_pinn_step_fn(graph=True)) ask this
    before capturing: False -- with one RuntimeWarning per caller -- when replays are not proven
    safe, and the caller then runs its eager step instead.  Never capture-and-hope: the failure
    the setting prevents is silently wrong results."""
    if graph_replays_safe():
        return True
    if what not in _WARNED:
        _WARNED.add(what)
        import warnings
        why = (f"{GRAPH_PACKET_CAPTURE}={os.environ.get(GRAPH_PACKET_CAPTURE)!r} was preset"
               if _PRESET not in (None, "0") else
               "the HIP runtime had started before `op` was imported")
        warnings.warn(f"{what}: running the eager step instead of hipGraph replays ({why}; "
                      "with graph packet capture on, replays can read other launches' kernel "
                      "arguments from the eager launch ring).  Import `op` (or set "
                      f"{GRAPH_PACKET_CAPTURE}=0) before the first device call -- "
                      "INTEGRATION.md section 1.", RuntimeWarning, stacklevel=3)
    return False
