"""torch.autograd.Function over the C-ABI: one fused RK4 solve (+ its VJP).

Forward : pack weights -> ude_rk4_forward (latent, stage checkpoints, side stats)
Backward: ude_rk4_backward (dy0, every weight/bias gradient) -> split into the
          parameters' shapes.
PyTorch only provides device memory and the current HIP stream here.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import torch

from . import _native
from .schedule import Schedule


@dataclass
class Plan:
    lib: "_native.NativeLib"
    desc: "_native.UdeModelDesc"
    prob: "_native.UdeProblem"
    sizes: "_native.UdeSizes"
    sched_dev: torch.Tensor
    n_times: int
    n_eval: int
    param_shapes: List[torch.Size]


def make_plan(cfg, schedule: Schedule, n_traj: int, fa_w: float, device: torch.device,
              param_shapes: List[torch.Size]) -> Plan:
    lib = _native.library_for(cfg)
    desc = _native.make_desc(cfg)
    prob = _native.UdeProblem()
    prob.n_traj = int(n_traj)
    prob.n_steps = schedule.n_steps
    prob.n_out = schedule.n_out
    prob.fa_w = float(fa_w)
    dev_index = device.index if device.index is not None else torch.cuda.current_device()
    sizes = lib.query(desc, prob, dev_index)
    sched = torch.from_numpy(schedule.to_bytes()).to(device, non_blocking=False)
    n_eval = 4 * schedule.n_steps * n_traj * cfg[1]
    return Plan(lib, desc, prob, sizes, sched, schedule.n_times, n_eval, param_shapes)


# Optional HIP-event instrumentation (bench.py): when a list, every forward /
# backward C-ABI call appends (kind, start_event, end_event) recorded on the
# stream the kernels are launched on.
EVENTS = None


def _ev(dev):
    return torch.cuda.Event(enable_timing=True)


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class SirSink:
    """Compact S, I, R cotangents of a fused solve's latent, deposited by consumers that read
    only latent[..., :3] (the fused loss head, ude_amd/loss_head.py) in place of a full-size
    (T, N, R, L) gradient that would be 5/8 zeros at L = 8.  A consumer that
    deposits returns ZERO_GRAD-like stride-0 zeros for the latent itself, so the solve's backward
    still runs; it adds the deposit to whatever full gradient other consumers produced."""

    def __init__(self):
        self.dl3 = None

    def add(self, dl3: torch.Tensor) -> None:
        self.dl3 = dl3 if self.dl3 is None else self.dl3 + dl3


_ZEROS = {}


def zero_grad_like(t: torch.Tensor) -> torch.Tensor:
    """A stride-0 zero tensor of t's shape (no memory): the placeholder gradient of a latent
    whose real cotangent went to its SirSink."""
    key = (str(t.device), t.dtype)
    z = _ZEROS.get(key)
    if z is None:
        z = _ZEROS[key] = torch.zeros((), dtype=t.dtype, device=t.device)
    return z.expand(t.shape)


def _is_placeholder(g: torch.Tensor) -> bool:
    z = _ZEROS.get((str(g.device), g.dtype))
    return z is not None and g.data_ptr() == z.data_ptr() and all(st == 0 for st in g.stride())


class FusedRK4(torch.autograd.Function):
    """Returns (latent, stats, ckpt); ckpt (the stage inputs of every step) is only a real
    output when keep_ckpt is set (materialised tracking), else an empty tensor.  latent carries
    a SirSink (``latent._ude_sir_sink``) for compact S, I, R cotangents."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, keep_ckpt: bool, *params: torch.Tensor):
        dev = y0.device
        stream = _stream(dev)
        sz = plan.sizes
        ws = [p.contiguous() for p in params[0::2]]
        bs = [p.contiguous() for p in params[1::2]]
        pack = torch.empty(sz.pack_bytes // 4, dtype=torch.float32, device=dev)
        plan.lib.pack(plan.desc, [w.data_ptr() for w in ws], [b.data_ptr() for b in bs], pack.data_ptr(), stream)
        latent = torch.empty((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        need_grad = any(ctx.needs_input_grad[1:])
        ckpt = torch.empty(max(sz.ckpt_bytes // 4, 1), dtype=torch.float32, device=dev) \
            if (need_grad or keep_ckpt) else None
        stats_slab = torch.empty(max(sz.stats_slab_bytes // 8, 1), dtype=torch.float64, device=dev)
        stats = torch.zeros(5, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.forward(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                         latent.data_ptr(), _ptr(ckpt), stats_slab.data_ptr(), stats.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("fwd", e0, e1))
        ctx.plan = plan
        ctx.sink = SirSink()
        ctx.set_materialize_grads(False)
        if need_grad:
            ctx.save_for_backward(y0, pack, ckpt, stats)
        out_ck = ckpt if keep_ckpt else torch.empty(0, dtype=torch.float32, device=dev)
        ctx.mark_non_differentiable(out_ck)
        latent._ude_sir_sink = ctx.sink
        return latent, stats, out_ck

    @staticmethod
    def backward(ctx, dlatent, dstats, _dckpt=None):
        plan: Plan = ctx.plan
        y0, pack, ckpt, stats = ctx.saved_tensors
        dev = y0.device
        stream = _stream(dev)
        dl3, ctx.sink.dl3 = ctx.sink.dl3, None
        if dlatent is not None and _is_placeholder(dlatent):
            dlatent = None                          # every consumer deposited compactly
        if dlatent is None and dl3 is None:
            dlatent = torch.zeros((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        if dlatent is not None:
            dlatent = dlatent.contiguous().to(torch.float32)
            if dl3 is not None:                     # other consumers too: one full cotangent
                dlatent = dlatent.clone()
                dlatent[..., :3] += dl3
                dl3 = None
        dstats = torch.zeros(5, dtype=torch.float32, device=dev) if dstats is None else dstats.contiguous().float()
        dy0 = torch.empty_like(y0)
        slab = torch.empty(max(plan.sizes.grad_slab_bytes // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty(plan.sizes.n_params, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.backward_sir(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                              ckpt.data_ptr(), _ptr(dlatent), _ptr(dl3), stats.data_ptr(), dstats.data_ptr(),
                              dy0.data_ptr(), slab.data_ptr(), dparams.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("bwd", e0, e1))
        return (None, dy0, None) + tuple(_split(dparams, plan.param_shapes))


def _split(flat: torch.Tensor, shapes) -> List[torch.Tensor]:
    out, off = [], 0
    for shp in shapes:
        n = 1
        for s in shp:
            n *= s
        out.append(flat[off:off + n].view(shp))
        off += n
    return out


class FusedBayesRK4(torch.autograd.Function):
    """Bayesian RHS (lib/in_development/models_bayes.py): every RHS evaluation of the
    solve uses its own weight sample w_e = mean + eps_e * |std| (Dense_Variational
    .forward, :43-48), eps = the (4 n_steps, n_params) draw stream.

    Inputs: plan, y0, eps, then the means (w, b per layer, torch order) and the raw
    stds in the same order.  The kernel returns d/d mean and d/d |std|; the sign of
    std (torch's abs backward) is applied here."""

    @staticmethod
    def forward(ctx, plan: Plan, y0: torch.Tensor, eps: torch.Tensor, *params: torch.Tensor):
        dev = y0.device
        stream = _stream(dev)
        sz = plan.sizes
        k = len(params) // 2
        mus = [p.contiguous() for p in params[:k]]
        sds = [p.contiguous() for p in params[k:]]
        eps = eps.contiguous()
        pack = torch.empty(max(sz.pack_bytes // 4, 1), dtype=torch.float32, device=dev)
        plan.lib.pack_bayes(plan.desc, plan.prob, [w.data_ptr() for w in mus[0::2]], [b.data_ptr() for b in mus[1::2]],
                            [w.data_ptr() for w in sds[0::2]], [b.data_ptr() for b in sds[1::2]], eps.data_ptr(),
                            pack.data_ptr(), stream)
        latent = torch.empty((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        need_grad = any(ctx.needs_input_grad[1:])
        ckpt = torch.empty(max(sz.ckpt_bytes // 4, 1), dtype=torch.float32, device=dev) if need_grad else None
        stats_slab = torch.empty(max(sz.stats_slab_bytes // 8, 1), dtype=torch.float64, device=dev)
        stats = torch.zeros(5, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.forward(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                         latent.data_ptr(), _ptr(ckpt), stats_slab.data_ptr(), stats.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("fwd", e0, e1))
        ctx.plan = plan
        if need_grad:
            ctx.save_for_backward(y0, pack, ckpt, stats, *sds)
        return latent, stats

    @staticmethod
    def backward(ctx, dlatent, dstats):
        plan: Plan = ctx.plan
        y0, pack, ckpt, stats, *sds = ctx.saved_tensors
        dev = y0.device
        stream = _stream(dev)
        if dlatent is None:
            dlatent = torch.zeros((plan.n_times,) + tuple(y0.shape), dtype=torch.float32, device=dev)
        dlatent = dlatent.contiguous().to(torch.float32)
        dstats = torch.zeros(5, dtype=torch.float32, device=dev) if dstats is None else dstats.contiguous().float()
        dy0 = torch.empty_like(y0)
        slab = torch.empty(max(plan.sizes.grad_slab_bytes // 4, 1), dtype=torch.float32, device=dev)
        dparams = torch.empty(plan.sizes.n_params, dtype=torch.float32, device=dev)
        if EVENTS is not None:
            e0 = _ev(dev); e0.record()
        plan.lib.backward(plan.desc, plan.prob, pack.data_ptr(), plan.sched_dev.data_ptr(), y0.data_ptr(),
                          _ptr(ckpt), dlatent.data_ptr(), stats.data_ptr(), dstats.data_ptr(),
                          dy0.data_ptr(), slab.data_ptr(), dparams.data_ptr(), stream)
        if EVENTS is not None:
            e1 = _ev(dev); e1.record(); EVENTS.append(("bwd", e0, e1))
        n = plan.sizes.n_params // 2
        d_mu = _split(dparams[:n], plan.param_shapes)
        d_abs = _split(dparams[n:], plan.param_shapes)
        d_sd = [g * torch.sign(s) for g, s in zip(d_abs, sds)]
        return (None, dy0, None) + tuple(d_mu) + tuple(d_sd)
