"""Data-parallel exchange steps on a gloo/CPU group (world_size 2).

The posterior statistics and |Fa| are global over every rank's trajectories
(lib/models.py:152-156, lib/VAE.py:180); ude_amd.distributed.combine_stats
all-reduces their sufficient statistics differentiably.  Checked against the
single-process values and gradients of the same data.
"""
import os
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO, import_pkg

WORLD = 2


MODE = ["stats"]


def _worker(rank, port, q, mode="stats"):
    MODE[0] = mode
    try:
        sys.path.insert(0, REPO)
        import_pkg()
        from ude_amd import distributed as udist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        gen = torch.Generator().manual_seed(11)
        p_all = torch.rand(300, 2, generator=gen, dtype=torch.float64) + 0.1
        fa_all = torch.randn(300, 3, generator=gen, dtype=torch.float64)
        lo, hi = (0, 180) if rank == 0 else (180, 300)      # uneven shards
        p = p_all[lo:hi].clone().requires_grad_(True)
        fa = fa_all[lo:hi].clone().requires_grad_(True)
        if MODE[0] == "sums":
            # the fused solves' path: fp64 totals made differentiable through (mean, std, |Fa|)
            from ude_amd.fused import stat_sums
            stats = torch.cat([p.mean(0), p.std(0), torch.norm(fa).reshape(1)])
            raw = torch.cat([p.sum(0), (p * p).sum(0), (fa * fa).sum().reshape(1)]).detach()
            n_tot, m, s, nrm = udist.combine_sums(float(hi - lo), stat_sums(stats, raw, float(hi - lo)))
        else:
            n_tot, m, s, nrm = udist.combine_stats(float(hi - lo), p.mean(0), p.std(0), torch.norm(fa))
        # every rank computes the same global loss term; grads of the SUM over ranks
        loss = (m * torch.tensor([0.3, -0.2], dtype=torch.float64)).sum() \
            + (s * torch.tensor([0.5, 0.1], dtype=torch.float64)).sum() + 0.1 * nrm.sum()
        loss.backward()
        gp = p.grad.clone()
        gf = fa.grad.clone()
        # gradient averaging across ranks as in all_reduce_grads: grads here are per-rank
        # contributions d(sum_r loss_r)/d p_local, which must equal WORLD x the single-process grad
        q.put((rank, float(n_tot), m.detach().numpy(), s.detach().numpy(), nrm.detach().numpy(), gp.numpy(), gf.numpy(), lo, hi))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))


@pytest.mark.parametrize("mode", ["stats", "sums"])
def test_combine_stats_matches_single_process(mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + (11 if mode == "sums" else 0)
    procs = [ctx.Process(target=_worker, args=(r, port, q, mode)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), res
    gen = torch.Generator().manual_seed(11)
    p_all = (torch.rand(300, 2, generator=gen, dtype=torch.float64) + 0.1).requires_grad_(True)
    fa_all = torch.randn(300, 3, generator=gen, dtype=torch.float64).requires_grad_(True)
    m, s, nrm = p_all.mean(0), p_all.std(0), torch.norm(fa_all)
    loss = (m * torch.tensor([0.3, -0.2], dtype=torch.float64)).sum() \
        + (s * torch.tensor([0.5, 0.1], dtype=torch.float64)).sum() + 0.1 * nrm
    loss.backward()
    for rank, n_tot, rm, rs, rn, gp, gf, lo, hi in res:
        rm, rs, rn, gp, gf = (torch.from_numpy(x) for x in (rm, rs, rn, gp, gf))
        assert n_tot == 300
        assert torch.allclose(rm, m.detach()) and torch.allclose(rs, s.detach())
        assert torch.allclose(rn, nrm.detach().reshape(1))
        assert torch.allclose(gp, WORLD * p_all.grad[lo:hi])
        assert torch.allclose(gf, WORLD * fa_all.grad[lo:hi])


def test_stat_sums_cotangent_maps_onto_the_kernel_inputs(pkg):
    """fused.stat_sums: the cotangent of the fp64 totals, handed to the kernel as (d mean, d std,
    d |Fa|) and applied per entry as the kernel backward does, equals d/dp of the totals."""
    from ude_amd.fused import stat_sums
    gen = torch.Generator().manual_seed(3)
    p = (torch.rand(50, 2, generator=gen, dtype=torch.float64) + 0.2).requires_grad_(True)
    fa = torch.randn(50, 3, generator=gen, dtype=torch.float64).requires_grad_(True)
    g = torch.randn(5, generator=gen, dtype=torch.float64)
    stats = torch.cat([p.mean(0), p.std(0), torch.norm(fa).reshape(1)])
    raw = torch.cat([p.sum(0), (p * p).sum(0), (fa * fa).sum().reshape(1)]).detach()
    (stat_sums(stats, raw, 50.0) * g).sum().backward()
    gp, gf = p.grad.clone(), fa.grad.clone()
    p.grad = None
    fa.grad = None
    (torch.cat([p.sum(0), (p * p).sum(0), (fa * fa).sum().reshape(1)]) * g).sum().backward()
    assert torch.allclose(gp, p.grad) and torch.allclose(gf, fa.grad)


def test_stat_sums_from_separate_outputs(pkg):
    """The fused solves return (mean, std, |Fa|) as three outputs: stat_sums over them gives the same
    totals and the same per-entry gradients as over the legacy 5-vector."""
    from ude_amd.fused import stat_sums
    gen = torch.Generator().manual_seed(4)
    p = (torch.rand(40, 2, generator=gen, dtype=torch.float64) + 0.2).requires_grad_(True)
    fa = torch.randn(40, 3, generator=gen, dtype=torch.float64).requires_grad_(True)
    g = torch.randn(5, generator=gen, dtype=torch.float64)
    raw = torch.cat([p.sum(0), (p * p).sum(0), (fa * fa).sum().reshape(1)]).detach()
    (stat_sums((p.mean(0), p.std(0), torch.norm(fa).reshape(1)), raw, 40.0) * g).sum().backward()
    g3 = (p.grad.clone(), fa.grad.clone())
    p.grad = None
    fa.grad = None
    (stat_sums(torch.cat([p.mean(0), p.std(0), torch.norm(fa).reshape(1)]), raw, 40.0) * g).sum().backward()
    assert torch.allclose(g3[0], p.grad) and torch.allclose(g3[1], fa.grad)


def test_tracker_entry_norm_is_a_view(pkg):
    """torch.norm(torch.stack(ode.tracker)) (lib/VAE.py:180) over the one |Fa|
    entry a fused solve records is that entry (no device operator; its cotangent passes unchanged);
    over several entries, or for other norms, the stock operators run."""
    from ude_amd.rhs import FaNormEntry
    src = torch.tensor([2.5], requires_grad=True)
    e = (src * 1.0).as_subclass(FaNormEntry)
    n = torch.norm(torch.stack([e]))
    assert type(n) is torch.Tensor and n.shape == () and float(n.detach()) == 2.5
    assert n.grad_fn is not None and "NormOfOne" in type(n.grad_fn).__name__
    (3.0 * n).backward()
    assert float(src.grad) == 3.0
    # two entries: the norm of both, gradient x / |x|
    src.grad = None
    e = (src * 1.0).as_subclass(FaNormEntry)
    e2 = (src * 2.0).as_subclass(FaNormEntry)
    n2 = torch.norm(torch.stack([e, e2]))
    assert abs(float(n2) - (2.5 ** 2 + 5.0 ** 2) ** 0.5) < 1e-6 and type(n2) is torch.Tensor
    n2.backward()
    assert abs(float(src.grad) - (2.5 * 1 + 5.0 * 2) / float(n2)) < 1e-6
    # other operators: plain tensors out
    assert type(e + 1) is torch.Tensor and float(torch.norm(torch.stack([e]), p=1)) == 2.5


def _reducer_worker(rank, port, q):
    """A two-stage model (an 'encoder' Linear feeding an 'ODE' Linear, like lib/VAE.py's encoder ->
    solve): the overlapped GradReducer against the one-shot all_reduce_grads, with the order in which
    the all-reduces were issued relative to the encoder's backward."""
    try:
        sys.path.insert(0, REPO)
        import_pkg()
        from ude_amd import distributed as udist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        torch.manual_seed(0)
        enc, ode = torch.nn.Linear(6, 5), torch.nn.Linear(5, 4)
        params = list(enc.parameters()) + list(ode.parameters())
        log = []

        class Tag(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x):
                return x.view_as(x)

            @staticmethod
            def backward(ctx, g):
                log.append(("encoder backward",))
                return g

        gen = torch.Generator().manual_seed(100 + rank)
        x = torch.randn(7 + 3 * rank, 6, generator=gen)

        def loss_fn():
            return (ode(Tag.apply(torch.tanh(enc(x)))) ** 2).sum()

        red = udist.GradReducer(params, average=True, bucket_bytes=1, log=log)   # one bucket per tensor
        outs = []
        for _ in range(2):                                   # two steps: the hooks re-arm
            for p in params:
                p.grad = None
            red.arm()
            loss_fn().backward()
            red.finish()
            outs.append([p.grad.clone() for p in params])
        steps_log = list(log)
        for p in params:
            p.grad = None
        loss_fn().backward()
        udist.all_reduce_grads(params, average=True)
        ref = [p.grad.clone() for p in params]
        # a backward without arm() issues nothing
        n_log = len(log)
        loss_fn().backward()
        q.put((rank, [[g.numpy() for g in o] for o in outs], [g.numpy() for g in ref], steps_log, len(log) - n_log,
               [len(b) for b in red.buckets]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put(("err", repr(e)))


def test_grad_reducer_overlaps_and_matches_all_reduce_grads():
    """VERDICT r4 item 6 (CPU rehearsal, gloo world 2): GradReducer's bucket all-reduces are issued
    from the gradient hooks -- the ODE stage's buckets before the encoder's backward has run, the
    encoder's after it -- and waited on only in finish(); the gradients equal all_reduce_grads' on
    every rank, step after step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + 23
    procs = [ctx.Process(target=_reducer_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), res
    for rank, outs, ref, log, extra, sizes in res:
        assert sizes == [1, 1, 1, 1]
        for o in outs:
            for a, b in zip(o, ref):
                assert torch.allclose(torch.from_numpy(a), torch.from_numpy(b), rtol=1e-6, atol=1e-7)
        log = [e for e in log if e[0] != "grad"]
        step = log[:len(log) // 2]
        assert step == log[len(log) // 2:]                  # the same order every step
        enc_at = step.index(("encoder backward",))
        # buckets 0, 1 = ode bias / weight (reverse registration order), 2, 3 = encoder
        assert {("issue", 0), ("issue", 1)} == set(step[:enc_at]), step
        assert {("issue", 2), ("issue", 3)} <= set(step[enc_at:]), step
        first_wait = min(i for i, e in enumerate(step) if e[0] == "wait")
        assert first_wait > max(i for i, e in enumerate(step) if e[0] == "issue"), step
        assert extra == 1                                   # unarmed backward: the Tag only
    # the ranks hold identical (summed) gradients
    for a, b in zip(res[0][1][0], res[1][1][0]):
        assert (a == b).all()


WORLD4 = 4


def _skew_worker(rank, port, q):
    """Four ranks whose autograd reaches the same parameters in rank-dependent orders (each rank
    applies the three stages of the model in its own rotation, so the post-accumulate-grad hooks fire
    in a different order on every rank), one parameter that gets no gradient on rank 1, and a second
    backward inside one armed pass."""
    try:
        sys.path.insert(0, REPO)
        import_pkg()
        from ude_amd import distributed as udist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WORLD4)
        torch.manual_seed(0)
        stages = [torch.nn.Linear(4, 4) for _ in range(3)]
        extra = torch.nn.Parameter(torch.randn(4))
        groups = [list(m.parameters()) for m in stages] + [[extra]]
        params = [p for g in groups for p in g]
        gen = torch.Generator().manual_seed(200 + rank)
        xs = [torch.randn(5 + rank, 4, generator=gen) for _ in range(3)]
        order = [(i + rank) % 3 for i in range(3)]

        def loss_fn():
            tot = 0.0
            for i in order:                     # the last stage applied is the first to get gradients
                tot = tot + torch.tanh(stages[i](xs[i])).pow(2).sum()
            if rank != 1:                       # rank 1's shard leaves `extra` without a gradient
                tot = tot + (extra * xs[0][0]).sum()
            return tot

        log = []
        red = udist.GradReducer(groups=groups, average=True, bucket_bytes=1, log=log)
        for p in params:
            p.grad = None
        red.arm()
        loss_fn().backward()
        red.finish()
        got = [None if p.grad is None else p.grad.clone() for p in params]
        grad_order = [e[1] for e in log if e[0] == "grad"]
        issue_order = [e[1] for e in log if e[0] == "issue"]
        # reference: the one-shot reduction with the missing gradient as zeros
        for p in params:
            p.grad = None
        loss_fn().backward()
        if extra.grad is None:
            extra.grad = torch.zeros_like(extra)
        udist.all_reduce_grads(params, average=True)
        ref = [p.grad.clone() for p in params]
        # one backward per arm(): a second backward in the same armed pass raises
        for p in params:
            p.grad = None
        red.arm()
        loss_fn().backward()
        try:
            loss_fn().backward()
            second = "no error"
        except RuntimeError as e:
            second = "raised" if "one backward per arm" in str(e) else repr(e)
        red.finish()                            # every rank still runs the same 7 collectives
        q.put((rank, [None if g is None else g.numpy() for g in got], [g.numpy() for g in ref], grad_order,
               issue_order, second, [len(b) for b in red.buckets]))
        red.remove()
        dist.barrier()
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_grad_reducer_in_order_under_skewed_hooks_world4():
    """VERDICT r5 item 7 / ADVICE r5 (gloo world 4): with hooks completing in a different order on every
    rank (7 buckets, one per tensor; bucket groups kept apart), GradReducer issues the buckets strictly
    in bucket-index order on every rank, as DDP does, so the collectives pair up; a parameter without a
    gradient on one rank's shard only delays its bucket (zeros in the flat, same size on every rank);
    the gradients equal all_reduce_grads' on every rank; a second backward in one armed pass raises."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000 + 47
    procs = [ctx.Process(target=_skew_worker, args=(r, port, q)) for r in range(WORLD4)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(WORLD4)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), [r[1] for r in res if r[0] == "err"]
    grad_orders = set()
    for rank, got, ref, grad_order, issue_order, second, sizes in res:
        assert sizes == [1] * 7, sizes
        assert issue_order == list(range(7)), (rank, issue_order)
        grad_orders.add(tuple(grad_order))
        for a, b in zip(got, ref):
            assert a is not None
            assert torch.allclose(torch.from_numpy(a), torch.from_numpy(b), rtol=1e-6, atol=1e-7)
        assert second == "raised", second
    assert len(grad_orders) >= 3, grad_orders          # the hooks really fired in different orders
    for a, b in zip(res[0][1], res[1][1]):
        assert (a == b).all()
