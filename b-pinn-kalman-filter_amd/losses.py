"""Training losses and the one-step train/eval function (reference: losses.py:29-224).

Same factories and state contract: `get_optimizer(config, params)`,
`optimization_manager(config)` (linear warm-up, grad-norm clipping),
`get_sde_loss_fn` (denoising score matching), `get_smld_loss_fn`,
`get_ddpm_loss_fn`, and `get_step_fn(sde, train, optimize_fn, reduce_mean,
continuous, likelihood_weighting)` -> `step_fn(state, batch)` with
state = {'optimizer', 'model', 'ema', 'step'}.

MI355X notes: the model runs on the fused HIP block ops; Adam uses the
fused multi-tensor implementation on the GPU (BPK_ADAM_FUSED=0: foreach); for batch-sharded data parallelism wrap
the model in torch DistributedDataParallel (RCCL all-reduce of the gradient
buckets, overlapped with backward) -- each rank's loss is the mean over its
shard, so the averaged gradient equals the single-process full-batch gradient.
The PINN step functions live in pinn_kalman/.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.optim as optim

from models import utils as mutils
from sde_lib import VESDE, VPSDE


_ADAM_FUSED = True


def get_optimizer(config, params, lr_mul=1.0, is_bpinn=False):
    lr = config.optim.bpinn_lr if is_bpinn else config.optim.lr
    decay = config.optim.bpinn_weight_decay if is_bpinn else config.optim.weight_decay
    if config.optim.optimizer != "Adam":
        raise NotImplementedError(f"Optimizer {config.optim.optimizer} not supported yet!")
    params = list(params)
    # on the GPU: the fused (single multi-tensor kernel per step) Adam, which also keeps the
    # per-parameter step counts and bias corrections on the device -- the foreach form
    # spends ~ms of host time per step on them for the ~700 NCSN++ tensors
    fused = _ADAM_FUSED and len(params) > 0 and all(
        (p["params"][0] if isinstance(p, dict) else p).is_cuda for p in params)
    kind = dict(fused=True) if fused else dict(foreach=True)
    return optim.Adam(params, lr=lr * lr_mul, betas=(config.optim.beta1, 0.999),
                      eps=config.optim.eps, weight_decay=decay, **kind)


def optimization_manager(config, is_bpinn=False):
    base_lr = config.optim.bpinn_lr if is_bpinn else config.optim.lr

    def optimize_fn(optimizer, params, step, lr=base_lr, warmup=config.optim.warmup,
                    grad_clip=config.optim.grad_clip):
        if warmup > 0:
            for g in optimizer.param_groups:
                g["lr"] = lr * np.minimum(step / warmup, 1.0)
        if grad_clip >= 0:
            torch.nn.utils.clip_grad_norm_(params, max_norm=grad_clip, foreach=True)
        optimizer.step()

    return optimize_fn


def _reducer(reduce_mean):
    if reduce_mean:
        return torch.mean
    return lambda *a, **k: 0.5 * torch.sum(*a, **k)


def get_sde_loss_fn(sde, train, reduce_mean=True, continuous=True, likelihood_weighting=True,
                    eps=1e-5):
    """Denoising score matching over t ~ U(eps, T) (reference losses.py:69-115)."""
    reduce_op = _reducer(reduce_mean)

    def loss_fn(model, batch):
        score_fn = mutils.get_score_fn(sde, model, train=train, continuous=continuous)
        t = torch.rand(batch.shape[0], device=batch.device) * (sde.T - eps) + eps
        z = torch.randn_like(batch)
        mean, std = sde.marginal_prob(batch, t)
        perturbed = mean + std[:, None, None, None] * z
        score = score_fn(perturbed, t)
        if not likelihood_weighting:
            losses = torch.square(score * std[:, None, None, None] + z)
            losses = reduce_op(losses.reshape(losses.shape[0], -1), dim=-1)
        else:
            g2 = sde.sde(torch.zeros_like(batch), t)[1] ** 2
            losses = torch.square(score + z / std[:, None, None, None])
            losses = reduce_op(losses.reshape(losses.shape[0], -1), dim=-1) * g2
        return torch.mean(losses)

    return loss_fn


def get_smld_loss_fn(vesde, train, reduce_mean=False):
    """Legacy NCSN loss (reference losses.py:118-139)."""
    assert isinstance(vesde, VESDE), "SMLD training only works for VESDEs."
    sigmas_desc = torch.flip(vesde.discrete_sigmas, dims=(0,))
    reduce_op = _reducer(reduce_mean)

    def loss_fn(model, batch):
        model_fn = mutils.get_model_fn(model, train=train)
        labels = torch.randint(0, vesde.N, (batch.shape[0],), device=batch.device)
        sig = sigmas_desc.to(batch.device)[labels]
        noise = torch.randn_like(batch) * sig[:, None, None, None]
        score = model_fn(noise + batch, labels)
        target = -noise / (sig ** 2)[:, None, None, None]
        losses = torch.square(score - target)
        losses = reduce_op(losses.reshape(losses.shape[0], -1), dim=-1) * sig ** 2
        return torch.mean(losses)

    return loss_fn


def get_ddpm_loss_fn(vpsde, train, reduce_mean=True):
    """Legacy DDPM loss (reference losses.py:142-162)."""
    assert isinstance(vpsde, VPSDE), "DDPM training only works for VPSDEs."
    reduce_op = _reducer(reduce_mean)

    def loss_fn(model, batch):
        model_fn = mutils.get_model_fn(model, train=train)
        labels = torch.randint(0, vpsde.N, (batch.shape[0],), device=batch.device)
        sa = vpsde.sqrt_alphas_cumprod.to(batch.device)
        s1 = vpsde.sqrt_1m_alphas_cumprod.to(batch.device)
        noise = torch.randn_like(batch)
        perturbed = sa[labels, None, None, None] * batch + s1[labels, None, None, None] * noise
        out = model_fn(perturbed, labels)
        losses = torch.square(out - noise)
        losses = reduce_op(losses.reshape(losses.shape[0], -1), dim=-1)
        return torch.mean(losses)

    return loss_fn


def get_step_fn(sde, train, optimize_fn=None, reduce_mean=False, continuous=True,
                likelihood_weighting=False):
    """One optimisation / evaluation step (reference losses.py:165-224)."""
    if continuous:
        loss_fn = get_sde_loss_fn(sde, train, reduce_mean=reduce_mean, continuous=True,
                                  likelihood_weighting=likelihood_weighting)
    else:
        assert not likelihood_weighting, \
            "Likelihood weighting is not supported for original SMLD/DDPM training."
        if isinstance(sde, VESDE):
            loss_fn = get_smld_loss_fn(sde, train, reduce_mean=reduce_mean)
        elif isinstance(sde, VPSDE):
            loss_fn = get_ddpm_loss_fn(sde, train, reduce_mean=reduce_mean)
        else:
            raise ValueError(f"Discrete training for {sde.__class__.__name__} is not recommended.")

    def step_fn(state, batch):
        model = state["model"]
        if train:
            from op import conv as conv_op
            optimizer = state["optimizer"]
            optimizer.zero_grad(set_to_none=True)
            # every Winograd filter of the step transformed in one launch (the weights change
            # after each optimizer step)
            with conv_op.batched_filters(model, enabled=batch.is_cuda):
                loss = loss_fn(model, batch)
                loss.backward()
            optimize_fn(optimizer, model.parameters(), step=state["step"])
            state["step"] += 1
            state["ema"].update(model.parameters())
        else:
            with torch.no_grad():
                ema = state["ema"]
                ema.store(model.parameters())
                ema.copy_to(model.parameters())
                loss = loss_fn(model, batch)
                ema.restore(model.parameters())
        return loss

    return step_fn


# ---------------------------------------------------------------- PINN steps

def check_for_nans(model):
    """True (and the offending name printed) if any parameter holds a NaN (losses.py:225-230)."""
    for name, param in model.named_parameters():
        if torch.isnan(param).any():
            print(f"NaN detected in parameter: {name}")
            return True
    return False


def _sync_grads(params, ctx):
    """Batch-sharded PINN training: average the gradients over ranks with one coalesced
    all-reduce per flat bucket (RCCL over xGMI).  Each rank's loss is a mean over its
    shard, so the average equals the full-batch gradient."""
    if ctx is None or not ctx.enabled:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch._utils._flatten_dense_tensors(grads)
    ctx.all_reduce_sum_(flat)
    flat.div_(ctx.world_size)
    for g, s in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
        g.copy_(s)


class GradBucketer:
    """Gradient averaging overlapped with backward, for models whose backward DDP cannot
    hook (the PINN step differentiates the networks twice, then calls backward()).

    Parameters are grouped, in reverse registration order (roughly the order backward
    produces their gradients), into buckets of ~bucket_mb; a post-accumulate-grad hook
    counts the bucket's arrivals and, when the last one lands, flattens the bucket and
    starts an asynchronous all-reduce (RCCL on its own stream over xGMI) while backward
    keeps running.  finish() waits for the in-flight buckets, syncs the ones that never
    completed (parameters without a gradient this step) with one coalesced call, and
    divides by the world size -- the same values as _sync_grads.  A NaN on any rank
    reaches every rank's averaged gradient, so the NaN-skip of the step functions
    (reference losses.py:361-366) is taken by all ranks together."""

    def __init__(self, params, ctx, bucket_mb=16.0):
        self.ctx = ctx
        self.params = [p for p in params if p.requires_grad]
        self.buckets, cur, size = [], [], 0
        for p in reversed(self.params):
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_mb * 2 ** 20:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self.where = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self.handles = [p.register_post_accumulate_grad_hook(self._arrived) for p in self.params]
        self.reset()

    def reset(self):
        self.count = [0] * len(self.buckets)
        self.works = {}

    def _arrived(self, p):
        i = self.where[id(p)]
        self.count[i] += 1
        if self.count[i] == len(self.buckets[i]):
            grads = [q.grad for q in self.buckets[i]]
            flat = torch._utils._flatten_dense_tensors(grads)
            work = torch.distributed.all_reduce(flat, group=self.ctx.group, async_op=True)
            self.works[i] = (work, flat, grads)

    def finish(self):
        n = self.ctx.world_size
        for i, (work, flat, grads) in sorted(self.works.items()):
            work.wait()
            flat.div_(n)
            for g, s in zip(grads, torch._utils._unflatten_dense_tensors(flat, grads)):
                g.copy_(s)
        rest = [p for i, b in enumerate(self.buckets) if i not in self.works for p in b]
        _sync_grads(rest, self.ctx)
        self.reset()

    def remove(self):
        for h in self.handles:
            h.remove()


def _observe(config, operator, f, noise=None):
    """inpainting measurement + Gaussian noise of variance config.inverse.variance (`noise`:
    the standard-normal draw, else torch.randn_like(f))."""
    z = torch.randn_like(f) if noise is None else noise
    return operator(f, keep_shape=True) + z * config.inverse.variance ** 0.5


def get_prelim_step_fn(config, train, optimize_fn, is_bpinn=False, ctx=None):
    """Schedule 1 of PINN training: data losses of FlowNet and PressureNet, each with its
    own Adam (reference losses.py:233-329).  Returns step_fn(state, operator, batch) ->
    (loss, v_loss, p_loss) with batch = (f1, f2, x, y, t, target)."""
    if is_bpinn:
        raise NotImplementedError("B-PINN needs bayesian_torch (not on the MI355X hot path)")
    error_fn = torch.nn.MSELoss()

    def flow_loss_fn(model, operator, batch):
        f1, f2, x, y, t, target = batch
        f1 = _observe(config, operator, f1)
        f2 = _observe(config, operator, f2)
        return model.multiscale_data_mse(model(f1, f2, x, y, t), target, error_fn=error_fn)

    def pres_loss_fn(model, batch):
        f1, f2, x, y, t, target = batch
        pyramid = [target[:, 0:2]]
        for _ in range(len(config.model.feature_nums)):
            flow = pyramid[-1]
            pyramid.append(torch.nn.functional.interpolate(
                flow, size=(flow.shape[2] // 2, flow.shape[3] // 2), mode="bilinear",
                align_corners=False))
        return model.data_mse(model(pyramid[::-1], x, y, t), target, error_fn=error_fn)

    def step_fn(state, operator, batch):
        model = state["model"]
        flownet, pressurenet = model.flownet, model.pressurenet
        operator.next()
        if train:
            opt_flow, opt_pres = state["optimizer"]
            flownet.train()
            opt_flow.zero_grad()
            v_loss = flow_loss_fn(flownet, operator, batch)
            v_loss.backward()
            _sync_grads(list(flownet.parameters()), ctx)
            optimize_fn(opt_flow, flownet.parameters(), step=state["step"])
            pressurenet.train()
            opt_pres.zero_grad()
            p_loss = pres_loss_fn(pressurenet, batch)
            p_loss.backward()
            _sync_grads(list(pressurenet.parameters()), ctx)
            optimize_fn(opt_pres, pressurenet.parameters(), step=state["step"])
            state["step"] += 1
            state["ema"].update(model.parameters())
        else:
            model.eval()
            ema = state["ema"]
            ema.store(model.parameters())
            ema.copy_to(model.parameters())
            v_loss = flow_loss_fn(flownet, operator, batch)
            p_loss = pres_loss_fn(pressurenet, batch)
            ema.restore(model.parameters())
        return v_loss + p_loss, v_loss, p_loss

    return step_fn


# Copies of the batch the PINN residual's derivative passes run on (PINN.forward_residual_copies):
# "auto" picks by the per-GPU batch, or a fixed 1 / 2 / 4 (1: the reference's seven passes).
# Measured on configs[3]'s graph step (profiles/r06_pinn_copies.txt): B = 8 (a rank of the 8-GPU
# point) 26.3 / 32.1 / 33.9 steps/s with 1 / 2 / 4 copies; B = 32 20.7 / 21.4 with 2 / 4;
# B = 64 14.3 / 15.5 / 13.8 with 1 / 2 / 4 (profiles/r06_pinn_copies.txt).  Re-measured on the
# final tree (deferred weight gradients, fan-outs; interleaved x3, one box,
# profiles/r06_pinn_copies_s2/): B = 8 40.7-41.3 with 4 vs 39.1-39.8 with 2; B = 16 32.1-33.3 vs
# 33.2-34.0; B = 32 23.6-23.8 vs 24.6-25.3 -- two copies from B = 16 on; B = 64 15.4 / 17.2 /
# 15.0 with 1 / 2 / 4 (b64.txt).
_COPIES = os.environ.get("BPK_PINN_COPIES", "auto")
# the PINN backward's weight gradients deferred and run two sources per launch
# (op.conv.deferred_weight_grads); BPK_DEFER_WGRAD=0: autograd's per-node weight gradients
_DEFER_WGRAD = os.environ.get("BPK_DEFER_WGRAD", "1") == "1"
_COPIES_AUTO = ((8, 4), (64, 2))  # (largest per-GPU batch, copies); larger batches: 1


def residual_copies(batch, on_gpu=True):
    if _COPIES != "auto":
        return int(_COPIES)
    if not on_gpu:
        return 1
    return next((k for b, k in _COPIES_AUTO if batch <= b), 1)


def get_pinn_step_fn(config, train, optimize_fn, ctx=None, graph=False):
    """Schedule 2: data losses + pinn_loss_weight * Navier-Stokes residual (Re = 1e7), both
    nets trained together; a NaN gradient on PressureNet's last 1x1 conv skips the update
    (reference losses.py:332-386).  Returns step_fn(state, operator, batch) ->
    (loss, pinn_loss, data_loss).  config.training.pinn_residual = 'stencil' switches the
    residual to `PINN.equation_mse_fd` (spatial derivatives on the ns_step stencil kernel);
    the default 'autograd' is the reference's.

    The reference probes that gradient with an extra autograd.grad pass before
    backward(); here it is read from .grad after the one backward -- the same value, and
    an identical skip (no optimizer step, no EMA update, step not advanced; the next
    step starts with zero_grad).  Under batch sharding the averaged gradient carries any
    rank's NaN, so every rank takes the same decision."""

    from pinn_kalman import pinn as _pinn

    def loss_fn(model, operator, batch, noise=(None, None)):
        _pinn._mark("forward")
        f1, f2, x, y, t, target = batch
        f1 = _observe(config, operator, f1, noise[0])
        f2 = _observe(config, operator, f2, noise[1])
        stencil = getattr(config.training, "pinn_residual", "autograd") == "stencil"
        copies = 1 if stencil else residual_copies(x.shape[0], f1.is_cuda)
        if copies > 1:
            # forward + residual with the derivative passes batched over input copies (same
            # values and gradients, ~half the launches: PINN.forward_residual_copies)
            flow_pred, pres_pred, res = model.forward_residual_copies(
                f1, f2, x, y, t, 10000000.0, copies)
        else:
            flow_pred, pres_pred = model(f1, f2, x, y, t)
            residual = model.equation_mse_fd if stencil else model.equation_mse
        data_loss = (model.flownet.multiscale_data_mse(flow_pred, target)
                     + model.pressurenet.data_mse(pres_pred, target))
        if copies == 1:
            res = residual(x, y, t, flow_pred[-1], pres_pred, 10000000.0)
        pinn_loss = res * config.training.pinn_loss_weight
        _pinn._mark("backward")
        return pinn_loss + data_loss, pinn_loss, data_loss

    if graph and train:
        from op import _hipenv
        # replays are only trusted with the runtime setting of op/_hipenv.py proven in effect;
        # otherwise (warned once) the eager step below runs instead
        if _hipenv.graphs_allowed("get_pinn_step_fn(graph=True)"):
            return _PinnGraphStep(loss_fn, optimize_fn, ctx, config.optim.grad_clip)

    bucketer = [None]  # eager + sharded: gradient buckets all-reduced during backward

    def step_fn(state, operator, batch):
        model = state["model"]
        operator.next()
        if train:
            opt_flow, opt_pres = state["optimizer"]
            model.train()
            if ctx is not None and ctx.enabled and bucketer[0] is None:
                bucketer[0] = GradBucketer(model.parameters(), ctx)
            opt_flow.zero_grad()
            opt_pres.zero_grad()
            from op import conv as conv_op
            with conv_op.batched_filters(model, enabled=batch[0].is_cuda):
                loss, pinn_loss, data_loss = loss_fn(model, operator, batch)
                # weight gradients two sources per launch (op.conv.deferred_weight_grads);
                # not under the bucketer, whose all-reduces ride the accumulation hooks
                with conv_op.deferred_weight_grads(_DEFER_WGRAD and bucketer[0] is None
                                                   and batch[0].is_cuda):
                    loss.backward()
            # the values only: a returned loss that still carries the spent autograd graph
            # keeps the parameters' AccumulateGrad nodes alive, and a hipGraph captured later
            # on another stream (get_pinn_step_fn(graph=True)) then accumulates through them
            # (stream mismatch: corrupted gradients, or a crash inside the capture)
            loss, pinn_loss, data_loss = loss.detach(), pinn_loss.detach(), data_loss.detach()
            if bucketer[0] is not None:
                bucketer[0].finish()  # buckets all-reduced while backward ran
            else:
                _sync_grads(list(model.parameters()), ctx)
            w = model.pressurenet.end[-1].weight
            if w.grad is not None and torch.isnan(w.grad).any():
                print(">>> Nan Grad Detected <<<")
                return loss, pinn_loss, data_loss
            optimize_fn(opt_flow, model.flownet.parameters(), step=state["step"])
            optimize_fn(opt_pres, model.pressurenet.parameters(), step=state["step"])
            state["step"] += 1
            state["ema"].update(model.parameters())
        else:
            model.eval()
            ema = state["ema"]
            ema.store(model.parameters())
            ema.copy_to(model.parameters())
            loss, pinn_loss, data_loss = loss_fn(model, operator, batch)
            ema.restore(model.parameters())
        return loss, pinn_loss, data_loss

    return step_fn


class _MaskOperator:
    """The inpainting operator on a static device mask (keep_shape form, the one the PINN
    observation uses): what a captured step reads, refilled before every replay."""

    def __init__(self, mask):
        self.mask = mask

    def __call__(self, x, keep_shape=True, invert=False):
        assert keep_shape
        return (1 - self.mask) * x if invert else self.mask * x


class _PinnGraphStep:
    """get_pinn_step_fn(graph=True): the forward (both nets, the residual's first and second
    derivatives) and the backward of one PINN train step as ONE hipGraph, replayed per step;
    the NaN-gradient skip, both Adam steps and the EMA update run eagerly after it (a handful
    of fused launches).  The eager step is ~9.4 k launches, host-bound at every batch size.

    What the capture needs, and round 3's withdrawn attempt lacked:
      * static inputs: the batch tensors and the observation mask are copied into buffers the
        graph owns before each replay.  The eager operator moves its CPU mask to the device
        inside the call (a host-to-device copy from a pageable tensor that the next
        operator.next() frees), so a captured step read a dead host buffer;
      * gradients: .grad is None when the graph is captured, so autograd allocates it from
        the graph's pool and every replay rewrites it in place (no zero_grad while replaying:
        setting .grad to None would detach the parameters from the graph's buffers);
      * native kernels only inside the graph (op.conv.native_only: no MIOpen convs, no
        library workspace state), the conv choices made eagerly during the warm-up.
    The observation noise is drawn eagerly into static buffers before each replay (the same
    draws, in the same order, as the eager step's two randn_like calls).
    Sharded (ctx): gradients are averaged with one all-reduce per step after the replay.
    Replays are safe against any eager work between steps (an eval step, metrics, reductions,
    RCCL calls) with the HIP runtime setting of op/_hipenv.py in effect: round 4's "eager
    reductions corrupt later replays" was the runtime's graph packet capture reading kernel
    arguments from the eager launch ring (root cause and measurements in op/_hipenv.py).
    Reference losses.py:332-386."""

    def __init__(self, loss_fn, optimize_fn, ctx, grad_clip=-1.0):
        self.loss_fn, self.optimize_fn, self.ctx = loss_fn, optimize_fn, ctx
        self.grad_clip = float(grad_clip)
        self.graph = None
        self.key = None

    def _capture(self, model, operator, batch):
        from op import conv as conv_op
        dev = batch[0].device
        self.static = [b.detach().clone() for b in batch]
        for i, b in enumerate(batch):
            if b.requires_grad:
                self.static[i].requires_grad_(True)
        self.mask = operator.mask.to(dev).clone()
        self.noise = (torch.zeros_like(self.static[0]), torch.zeros_like(self.static[1]))
        sop = _MaskOperator(self.mask)
        params = list(model.parameters())
        with conv_op.native_only():
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):  # kernel choices, allocator, lazy state: off the capture
                    for p in params:
                        p.grad = None
                    with conv_op.batched_filters(model):
                        loss, _pl, _dl = self.loss_fn(model, sop, self.static, self.noise)
                        with conv_op.deferred_weight_grads(_DEFER_WGRAD):
                            loss.backward(inputs=params)
            # nothing of the warm-up may be freed while the capture runs: a block released
            # mid-capture went back to the general pool and could be handed to the graph, which
            # then shared it with eager allocations after the capture (replays read garbage a
            # few steps later)
            del loss, _pl, _dl
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            for p in params:
                p.grad = None
            for b in self.static:
                b.grad = None
            # the host side reads eager-owned copies the graph writes (gradients, losses); the
            # NaN probe and the clipping norms run in a second captured graph (fewer launches)
            gbufs = [torch.zeros_like(p) for p in params]
            obuf = torch.zeros(4, device=dev, dtype=torch.float32)
            g = torch.cuda.CUDAGraph()
            # captured on the warm-up stream: the parameters' AccumulateGrad nodes (created
            # in the warm-up) record that stream.  backward(inputs=params): the coordinate
            # inputs' .grad (unused; the eager step accumulates them as the reference does)
            # is neither computed nor accumulated by the replays
            with torch.cuda.graph(g, stream=s):
                # one recorded launch transforms every Winograd filter of the step (the job
                # table and the transform buffers were built by the warm-up)
                with conv_op.batched_filters(model):
                    loss, pl, dl = self.loss_fn(model, sop, self.static, self.noise)
                    with conv_op.deferred_weight_grads(_DEFER_WGRAD):
                        loss.backward(inputs=params)
                live = [(gb, p.grad) for gb, p in zip(gbufs, params) if p.grad is not None]
                torch._foreach_copy_([a for a, _ in live], [b for _, b in live])
                obuf[:3].copy_(torch.stack([loss.detach(), pl.detach(), dl.detach()]))
            # the graph's own gradient tensors stay referenced (their memory is the graph's);
            # the parameters' .grad become the eager-owned copies from here on
            self.graph_grads = [p.grad for p in params]
            for p, gb in zip(params, gbufs):
                p.grad = gb if p.grad is not None else None
            # graph B, replayed after the (sharded: all-reduced) gradients are final: the
            # reference's NaN probe on the pressure net's last weight, then clip_grad_norm_ of
            # each optimizer's parameters (optimization_manager; torch's formula)
            w = model.pressurenet.end[-1].weight
            groups = [[p.grad for p in m.parameters() if p.grad is not None]
                      for m in (model.flownet, model.pressurenet)]
            gb_ = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gb_, stream=s):
                obuf[3:].copy_(torch.isnan(w.grad).any().float().reshape(1))
                if self.grad_clip >= 0:
                    for grads in groups:
                        norms = torch._foreach_norm(grads, 2.0)
                        total = torch.linalg.vector_norm(torch.stack(norms), 2.0)
                        coef = torch.clamp(self.grad_clip / (total + 1e-6), max=1.0)
                        torch._foreach_mul_(grads, coef)
        self.out = (obuf[0], obuf[1], obuf[2])
        self.obuf = obuf
        self.gbufs = [p.grad for p in params]
        self.graph = g
        self.graph_b = gb_
        self.params = params
        # the graph recorded raw pointers: the parameters' storage and the FilterBatch's job
        # table / transform buffers (kept alive here; a replaced weight changes the key below
        # and forces a recapture instead of replaying into freed memory -- ADVICE r05)
        self.filter_batch = conv_op.filter_batch_for(model)
        self.key = self._key(model, batch)

    @staticmethod
    def _key(model, batch):
        return (id(model), tuple((b.shape, b.dtype) for b in batch),
                tuple(p.data_ptr() for p in model.parameters()))

    def __call__(self, state, operator, batch):
        model = state["model"]
        operator.next()
        opt_flow, opt_pres = state["optimizer"]
        model.train()
        if self.graph is None or self._key(model, batch) != self.key:
            self._capture(model, operator, batch)
        # the optimizers read p.grad: point it back at the buffers the graphs write, in case a
        # caller's zero_grad(set_to_none=True) or an eager step replaced it since the last call
        #  -- else Adam would apply stale gradients, or skip every parameter
        for p, gb in zip(self.params, self.gbufs):
            if p.grad is not gb:
                p.grad = gb
        with torch.no_grad():
            for d, b in zip(self.static, batch):
                d.copy_(b)
            m = operator.mask
            self.mask.copy_(m if m.device == self.mask.device else m.to(self.mask.device))
            for z in self.noise:
                z.normal_()
        self.graph.replay()
        _sync_grads(self.params, self.ctx)
        self.graph_b.replay()
        loss, pinn_loss, data_loss = (t.detach().clone() for t in self.out)
        if bool(self.obuf[3].item()):
            print(">>> Nan Grad Detected <<<")
            return loss, pinn_loss, data_loss
        # clipped inside graph B already
        self.optimize_fn(opt_flow, model.flownet.parameters(), step=state["step"], grad_clip=-1.0)
        self.optimize_fn(opt_pres, model.pressurenet.parameters(), step=state["step"],
                         grad_clip=-1.0)
        state["step"] += 1
        state["ema"].update(model.parameters())
        return loss, pinn_loss, data_loss

