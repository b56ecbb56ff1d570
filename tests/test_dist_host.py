"""CPU (gloo, world size 2) tests of the host-side multi-rank logic: the backward-overlapped
gradient buckets of the PINN step (losses.GradBucketer) equal the coalesced average, incl.
parameters that receive no gradient, and a NaN on one rank reaches every rank."""
import os
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _worker(rank, world, port, inject_nan, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                          WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
        sys.path[:0] = [HERE, os.path.join(HERE, "..", "b-pinn-kalman-filter_amd"),
                        os.path.join(HERE, "..")]
        import dist
        import losses
        ctx = dist.init_from_env(backend="gloo")
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.Tanh(),
                                  torch.nn.Linear(256, 256), torch.nn.Tanh(),
                                  torch.nn.Linear(256, 8))
        unused = torch.nn.Linear(3, 3)  # never receives a gradient
        params = list(net.parameters()) + list(unused.parameters())
        buck = losses.GradBucketer(params, ctx, bucket_mb=0.1)
        g = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(16, 64, generator=g)
        if inject_nan and rank == 1:
            x[3, 5] = float("nan")
        out = []
        for _ in range(2):  # twice: the buckets reset between steps
            for p in params:
                p.grad = None
            net(x).pow(2).mean().backward()
            mine = [p.grad.numpy().copy() for p in net.parameters()]
            buck.finish()
            out.append(([p.grad.numpy().copy() for p in net.parameters()], mine,
                        [p.grad for p in unused.parameters()]))
        q.put((rank, out, len(buck.buckets), None))
        torch.distributed.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put((rank, None, 0, traceback.format_exc()))


def _run(inject_nan):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31000 + (os.getpid() * 3 + int(inject_nan)) % 2000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, inject_nan, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted((q.get(timeout=300) for _ in ps), key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, r[3]
    return res


def test_grad_buckets_equal_the_coalesced_average():
    (r0, out0, nb, _), (r1, out1, _, _) = _run(False)
    assert nb >= 2  # several buckets, launched from the hooks
    for (avg0, mine0, un0), (avg1, mine1, un1) in zip(out0, out1):
        for a0, a1, m0, m1 in zip(avg0, avg1, mine0, mine1):
            np.testing.assert_array_equal(a0, a1)
            np.testing.assert_allclose(a0, (m0 + m1) / 2, rtol=1e-6, atol=1e-7)
        assert all(g is None for g in un0 + un1)


def test_nan_on_one_rank_reaches_every_rank():
    (_, out0, _, _), (_, out1, _, _) = _run(True)
    for (avg0, mine0, _), (avg1, _, _) in zip(out0, out1):
        assert not any(np.isnan(m).any() for m in mine0)  # rank 0's own grads are finite
        last0, last1 = avg0[-2], avg1[-2]  # the output layer's weight (the PINN check's analogue)
        assert np.isnan(last0).any() and np.isnan(last1).any()
