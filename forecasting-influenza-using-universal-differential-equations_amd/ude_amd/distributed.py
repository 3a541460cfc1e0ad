"""Data-parallel pieces of the hot path (one process per GPU, RCCL over xGMI).

Trajectories are independent, so the batch shards along windows (SURVEY
section 8e; keep all MC samples of a window on one rank so the per-window
sample statistics of ``nll_loss`` stay local).  Two exchanges are real:

1. forward: the posterior over *all* recorded rates and the Fa norm are
   global (lib/models.py:152-156, lib/VAE.py:180).  Each rank's fused solve
   leaves its fp64 totals (n, sum b, sum g, sum b^2, sum g^2, sum Fa^2) in the
   stats slab; ``sync_side_stats`` all-reduces those 6 doubles and forms the
   global (mean, std, |Fa|) as the kernel's finaliser does.  The all-reduce is
   differentiable (its backward all-reduces the cotangent; ``fused.stat_sums``
   maps it onto the kernel's (d mean, d std, d |Fa|) input), so every rank's
   kernel receives d loss_total / d stats in its backward.  Entries without
   fp64 totals (eager evaluations) go through sufficient statistics rebuilt
   from (n, mean, std, |Fa|).
2. backward: bucketed all-reduces of the flat parameter gradients, each issued
   from autograd hooks as soon as its bucket is complete (``GradReducer``) and
   overlapped with the rest of the backward; ``all_reduce_grads`` is the
   one-shot form after ``backward``.  The 6-double statistics exchange's
   backward (the cotangent all-reduce) is the first node autograd reaches
   below the loss, so it runs ahead of the solve's backward kernels.
"""
from __future__ import annotations

from typing import Iterable, List

import torch
import torch.distributed as dist


def _active(group=None) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


def world_size(group=None) -> int:
    return dist.get_world_size(group) if (dist.is_available() and dist.is_initialized()) else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if (dist.is_available() and dist.is_initialized()) else 0


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        y = x.clone()
        dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.clone()
        dist.all_reduce(g, op=dist.ReduceOp.SUM, group=ctx.group)
        return g, None


def all_reduce_sum(x: torch.Tensor, group=None) -> torch.Tensor:
    """Differentiable SUM all-reduce (identity when not distributed)."""
    if not _active(group):
        return x
    return _AllReduceSum.apply(x, group)


def all_reduce_values(x: torch.Tensor, group=None) -> torch.Tensor:
    """SUM all-reduce of a detached vector (reported loss terms)."""
    if not _active(group):
        return x
    y = x.clone()
    dist.all_reduce(y, op=dist.ReduceOp.SUM, group=group)
    return y


def broadcast_parameters(params: Iterable[torch.nn.Parameter], src: int = 0, group=None) -> None:
    """Rank src's parameter values on every rank (one flat bucket)."""
    if not _active(group):
        return
    ps = list(params)
    if not ps:
        return
    with torch.no_grad():
        flat = torch.cat([p.detach().reshape(-1) for p in ps])
        dist.broadcast(flat, src=src, group=group)
        off = 0
        for p in ps:
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p))
            off += n


def broadcast_rng_state(device, src: int = 0, group=None) -> None:
    """Rank src's RNG state (the host generator and, for a HIP device, that device's) on every
    rank, so replicated random draws (the VAE's full-batch eps) agree without per-step traffic.

    This synchronises the process-wide generators: from the call on, every torch draw (the VAE's
    eps, but also dropout or any other sampling of the caller) is identical on every rank.  The
    data-parallel VAE step relies on exactly that (each rank slices the same full-batch eps);
    code that needs per-rank randomness after it must use its own ``torch.Generator``."""
    if not _active(group):
        return
    dev = torch.device(device)
    comm = dev if (dev.type == "cuda" and dist.get_backend(group) == "nccl") else torch.device("cpu")
    def bcast(state):
        buf = state.to(comm)
        dist.broadcast(buf, src=src, group=group)
        return buf.cpu()
    torch.set_rng_state(bcast(torch.get_rng_state()))
    if dev.type == "cuda":
        torch.cuda.set_rng_state(bcast(torch.cuda.get_rng_state(dev)), dev)


def combine_stats(n_local: float, mean: torch.Tensor, std: torch.Tensor, norm: torch.Tensor, group=None):
    """Global (n, mean, std, norm) from per-rank values (Chan's pooled variance, fp64)."""
    n = torch.tensor([n_local], dtype=torch.float64, device=mean.device)
    m = mean.double()
    s = std.double()
    suff = torch.cat([n, n * m, (n - 1.0) * s * s + n * m * m, norm.double().reshape(1) ** 2])
    tot = all_reduce_sum(suff, group)
    n_tot = tot[0]
    gmean = tot[1:3] / n_tot
    gvar = (tot[3:5] - n_tot * gmean * gmean) / (n_tot - 1.0)
    gstd = torch.sqrt(torch.clamp(gvar, min=0.0))
    gnorm = torch.sqrt(tot[5:6])
    return n_tot, gmean.to(mean.dtype), gstd.to(std.dtype), gnorm.to(norm.dtype)


def combine_sums(n_local: float, sums: torch.Tensor, group=None):
    """Global (n, mean, std, norm) from per-rank fp64 totals (sum b, sum g, sum b^2, sum g^2,
    sum Fa^2): one differentiable 6-double all-reduce, then the kernel's own finalisation
    (ude_stats_finalize_kernel) in fp64."""
    n = torch.tensor([n_local], dtype=torch.float64, device=sums.device)
    tot = all_reduce_sum(torch.cat([n, sums.double()]), group)
    n_tot = tot[0]
    gmean = tot[1:3] / n_tot
    gvar = (tot[3:5] - n_tot * gmean * gmean) / (n_tot - 1.0)
    gstd = torch.sqrt(torch.clamp(gvar, min=0.0))
    gnorm = torch.sqrt(tot[5:6])
    return n_tot, gmean, gstd, gnorm


def _sync_from_sums(module, group) -> bool:
    """The exchange on the fused solves' fp64 totals; False when some recorded entry
    has none (eager evaluations, materialised lists, the dopri5 forward), for the fallback."""
    from .fused import stat_sums
    from .rhs import eager_params
    sums = module._fused_sums
    has_p = module.ode_type in ("Fp", "FaFp")
    has_a = module.ode_type in ("Fa", "FaFp")
    if not sums or eager_params(module.params):
        return False
    if has_p and len(module._fused_rates) != len(sums):
        return False
    if has_a and len(module.tracker) != len(sums):
        return False
    n = sum(e[0] for e in sums)
    local = stat_sums(sums[0][1], sums[0][2], sums[0][0])
    for e in sums[1:]:
        local = local + stat_sums(e[1], e[2], e[0])
    n_tot, gm, gs, gn = combine_sums(n, local, group)
    dt = module._fused_rates[0][1].dtype if has_p else None
    module.params = []                      # drops the local statistics (and their sums)
    if has_p:
        module._fused_rates = [(n_tot.detach(), gm.to(dt), gs.to(dt))]
    if has_a:
        module.tracker = [gn.to(module.tracker[0].dtype)]
    return True


def sync_side_stats(module, group=None) -> None:
    """Replace the module's recorded fused-solve statistics by their global values: an
    all-reduce of the kernel's fp64 totals when every entry has them, else of the sufficient
    statistics rebuilt from (n, mean, std, |Fa|)."""
    if not _active(group):
        return
    if _sync_from_sums(module, group):
        return
    # eager evaluations (params / tracker lists of per-evaluation tensors) are folded into
    # the same sufficient statistics as the fused solves' entries
    from .rhs import eager_params
    groups = list(module._fused_rates)
    eager = eager_params(module.params)     # materialised fused entries are already in _fused_rates
    if eager:
        p = torch.stack(eager).reshape(-1, 2)
        groups.append((float(p.shape[0]), p.mean(0), p.std(0)))
    tracker = list(module.tracker)
    if not groups and not tracker:
        return
    if groups:
        n = sum(g[0] for g in groups)
        m = sum(g[0] * g[1] for g in groups) / n
        s = torch.sqrt(sum((g[0] - 1.0) * g[2] ** 2 + g[0] * (g[1] - m) ** 2 for g in groups) / (n - 1.0)) \
            if len(groups) > 1 else groups[0][2]
    else:
        dev = tracker[-1].device
        n, m, s = 1.0, torch.zeros(2, device=dev), torch.ones(2, device=dev)
    # == torch.norm(torch.stack(tracker)) of lib/VAE.py:180 (the norm of every entry together)
    if tracker:
        norm = torch.norm(torch.cat([x.reshape(-1) for x in tracker])).reshape(1)
    else:
        norm = torch.zeros(1, device=m.device)
    n_tot, gm, gs, gn = combine_stats(n, m, s, norm, group)
    module.params = []
    if groups:
        module._fused_rates = [(n_tot.detach(), gm, gs)]
    if tracker:
        module.tracker = [gn]


class GradReducer:
    """The data-parallel gradient all-reduce, overlapped with the rest of the backward (VERDICT r4
    item 6).  Parameters are split into buckets in reverse registration order (the order autograd
    produces their gradients: the decoder's, then the ODE's, then the encoder's in the VAE,
    lib/VAE.py:200-223); ``groups`` (a list of parameter lists in registration order, e.g. one per
    submodule) keeps every bucket inside one group, so a small model still gets one bucket per stage
    instead of a single bucket completed only by the last hook.  A post-accumulate-grad hook marks
    each parameter, and buckets are issued strictly in bucket-index order, as DDP does: bucket b goes
    out the moment it and every bucket before it are complete, asynchronously -- on a side stream
    for a HIP device (RCCL then runs while the backward's remaining kernels, e.g. the encoder's, run
    on the compute stream), on gloo's worker thread on the CPU.  The issue order is therefore the
    same on every rank whatever order the hooks fire in (a rank whose autograd reaches the buckets in
    another order, or a parameter that got no gradient on one rank's shard, only delays the issue;
    the collectives still pair up).  A bucket's flat buffer always covers every parameter of the
    bucket (zeros for a parameter without a gradient on this rank), so its size is the same on every
    rank; a parameter without a gradient gets the reduced slice unless that slice is all zero.

    ``arm()`` before the step's ``backward`` (the hooks do nothing otherwise, so other backward
    passes -- pre-training, evaluation -- are untouched), ``finish()`` after it issues every bucket
    not yet issued (in index order), waits for the all-reduces, and writes the summed (``average``:
    / world) gradients back.  One backward per ``arm()``: a parameter whose hook fires twice in one
    armed pass (gradient accumulation, a second loss, retain_graph) raises, since its bucket may
    already be reduced.  ``log`` (when a list) receives ("grad", bucket) per hook, ("issue", bucket)
    and ("wait", bucket) in order: the CPU rehearsal's record of the overlap."""

    def __init__(self, params: Iterable[torch.nn.Parameter] = (), average: bool = True, group=None,
                 bucket_bytes: int = 4 << 20, log=None, groups=None):
        self.group, self.average, self.log = group, average, log
        segs = [list(g) for g in groups] if groups is not None else [list(params)]
        segs = [[p for p in g if p.requires_grad] for g in segs]
        ps = [p for g in segs for p in g]
        self.buckets: List[List[torch.nn.Parameter]] = []
        for seg in reversed(segs):
            cur, size = [], 0
            for p in reversed(seg):
                cur.append(p)
                size += p.numel() * p.element_size()
                if size >= bucket_bytes:
                    self.buckets.append(cur)
                    cur, size = [], 0
            if cur:
                self.buckets.append(cur)
        self._where = {}
        for b, bucket in enumerate(self.buckets):
            for p in bucket:
                if id(p) in self._where:
                    raise ValueError("GradReducer: a parameter appears twice")
                self._where[id(p)] = b
        self._hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in ps] if _active(group) else []
        self._stream = None
        self._reset()

    def _reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._seen = set()
        self._next = 0                      # the next bucket to issue (index order)
        self._inflight = {}                 # bucket -> (work, flat, params)
        self._armed = False

    def arm(self) -> "GradReducer":
        self._reset()
        self._armed = True
        return self

    def _ready(self, p):
        if not self._armed:
            return
        if id(p) in self._seen:
            raise RuntimeError("GradReducer: a parameter received a second gradient in one armed backward "
                               "(one backward per arm(): accumulate with arm()/finish() around each backward, "
                               "or reduce once after the last with all_reduce_grads)")
        self._seen.add(id(p))
        b = self._where[id(p)]
        self._pending[b] -= 1
        if self.log is not None:
            self.log.append(("grad", b))
        while self._next < len(self.buckets) and self._pending[self._next] == 0:
            self._issue(self._next)
            self._next += 1

    def _issue(self, b):
        ps = self.buckets[b]
        have = [p for p in ps if p.grad is not None]
        if have:
            dev, dt = have[0].grad.device, have[0].grad.dtype
        else:
            dev, dt = ps[0].device, ps[0].dtype

        def flatten():
            return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p, dtype=dt)).reshape(-1)
                              for p in ps])
        if dev.type == "cuda":
            if self._stream is None:
                self._stream = torch.cuda.Stream(dev)
            self._stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(self._stream):
                flat = flatten()
                work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        else:
            flat = flatten()
            work = dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._inflight[b] = (work, flat, ps)
        if self.log is not None:
            self.log.append(("issue", b))

    def finish(self) -> None:
        if not _active(self.group):
            return
        assert self._armed, "GradReducer.finish() without arm() before the backward"
        while self._next < len(self.buckets):
            self._issue(self._next)
            self._next += 1
        ws = dist.get_world_size(self.group)
        for b in range(len(self.buckets)):
            work, flat, ps = self._inflight[b]
            work.wait()
            if self.log is not None:
                self.log.append(("wait", b))
            dev = flat.device
            if dev.type == "cuda":
                torch.cuda.current_stream(dev).wait_stream(self._stream)
                flat.record_stream(torch.cuda.current_stream(dev))
            if self.average:
                flat /= ws
            off = 0
            for p in ps:
                n = p.numel()
                sl = flat[off:off + n].view_as(p)
                off += n
                if p.grad is not None:
                    p.grad.copy_(sl)
                elif bool(sl.ne(0).any()):
                    p.grad = sl.clone()
        self._reset()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


def all_reduce_grads(params: Iterable[torch.nn.Parameter], average: bool = True, group=None) -> None:
    """One flat bucket (the ODE has <= ~0.3 MB of gradients, the whole VAE <= ~1 MB: a single
    ring all-reduce).  Parameters without a gradient are skipped (the bucket layout is the same
    on every rank: the same model, the same loss terms)."""
    if not _active(group):
        return
    ps: List[torch.nn.Parameter] = [p for p in params if p.grad is not None]
    if not ps:
        return
    flat = torch.cat([p.grad.reshape(-1) for p in ps])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if average:
        flat /= dist.get_world_size(group)
    off = 0
    for p in ps:
        n = p.grad.numel()
        p.grad.copy_(flat[off:off + n].view_as(p.grad))
        off += n
