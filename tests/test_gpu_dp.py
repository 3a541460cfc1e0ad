"""Data-parallel hot path on the GPU: 2 ranks (gloo process group, both on
cuda:0 -- the 1-GPU test box) each solve half of the trajectories with the fused
kernel; the side statistics are combined with ude_amd.distributed and the
parameter gradients summed.  Must equal the single-process solve of the whole
batch (same loss: data term + global posterior / |Fa| terms once).  The gradients are summed by
GradReducer (bucket all-reduces issued during the backward on a side stream) in the "stats" case and
by the one-shot all_reduce_grads in the "materialized" one."""
import os
import sys

import pytest
import torch
import torch.multiprocessing as mp

from conftest import REPO, import_pkg

pytestmark = pytest.mark.gpu
WORLD = 2
N = 96


def _setup(pkg, dev, materialize=False):
    torch.manual_seed(0)
    mod = pkg.FaFp(10, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(dev)
    # materialised per-evaluation lists must not be counted twice by sync_side_stats
    mod.materialize_tracking = materialize
    gen = torch.Generator().manual_seed(9)
    S = torch.rand(N, 10, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, 10, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, 10, 5, generator=gen)], -1)
    t = torch.arange(5, dtype=torch.float32)
    dl = torch.randn((5, N, 10, 8), generator=gen)
    return mod, (y0 + 1e-5).to(dev), t, dl.to(dev)


def _loss(pkg, mod, y0, t, dl, world):
    from ude_amd import distributed as udist
    mod.clear_tracking()
    lat = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=t[1] - t[0]))
    udist.sync_side_stats(mod)
    post = mod.posterior()
    nrm = torch.norm(torch.stack(mod.tracker))
    dev = y0.device
    stats_term = (post.loc * torch.tensor([0.3, -0.2], device=dev)).sum() \
        + (post.scale * torch.tensor([0.5, 0.1], device=dev)).sum() + 0.1 * nrm
    return (lat * dl).sum() + stats_term / world, post.loc.detach(), post.scale.detach(), nrm.detach()


def _worker(rank, port, q, materialize):
    try:
        sys.path.insert(0, REPO)
        pkg = import_pkg()
        import torch.distributed as dist
        from ude_amd import distributed as udist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        dev = torch.device("cuda", 0)
        mod, y0, t, dl = _setup(pkg, dev, materialize)
        lo, hi = (0, 40) if rank == 0 else (40, N)          # uneven shards
        red = None if materialize else udist.GradReducer(mod.parameters(), average=False, bucket_bytes=64 << 10)
        if red is not None:
            red.arm()
        loss, m, s, nrm = _loss(pkg, mod, y0[lo:hi].contiguous(), t, dl[:, lo:hi].contiguous(), WORLD)
        loss.backward()
        if red is not None:
            # the overlapped path: bucket all-reduces issued from the gradient hooks on a side stream
            red.finish()
        else:
            udist.all_reduce_grads(mod.parameters(), average=False)
        q.put((rank, m.cpu().numpy(), s.cpu().numpy(), nrm.cpu().numpy(), [p.grad.cpu().numpy() for p in mod.parameters()]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


@pytest.mark.parametrize("materialize", [False, True], ids=["stats", "materialized"])
def test_two_rank_dp_matches_single_process(pkg, materialize):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 1000 + (7 if materialize else 0)
    procs = [ctx.Process(target=_worker, args=(r, port, q, materialize)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(WORLD)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[0] != "err" for r in res), [r[1] for r in res if r[0] == "err"]
    mod, y0, t, dl = _setup(pkg, torch.device("cuda", 0), materialize)
    loss, m, s, nrm = _loss(pkg, mod, y0, t, dl, 1)
    loss.backward()
    ref = [p.grad.cpu() for p in mod.parameters()]
    for rank, rm, rs, rn, grads in res:
        rm, rs, rn = torch.from_numpy(rm), torch.from_numpy(rs), torch.from_numpy(rn)
        grads = [torch.from_numpy(g) for g in grads]
        assert torch.allclose(rm, m.cpu(), rtol=1e-5, atol=1e-7)
        assert torch.allclose(rs, s.cpu(), rtol=1e-4, atol=1e-7)
        assert torch.allclose(rn, nrm.cpu().reshape(1), rtol=1e-5)
        for a, b in zip(grads, ref):
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-5 * float(b.abs().max())), float((a - b).abs().max())


def _rccl_worker(port, q):
    try:
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        dev = torch.device("cuda", 0)
        # the payloads of ude_amd.distributed: the fp64 statistics totals (combine_sums), one flat
        # fp32 gradient bucket (all_reduce_grads), parameter / RNG-state broadcasts
        sums = torch.tensor([96.0, 1.5, -2.25, 3.0, 4.5, 0.75], dtype=torch.float64, device=dev)
        flat = torch.randn(300_001, device=dev)
        ref_s, ref_f = sums.clone(), flat.clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        dist.all_reduce(flat, op=dist.ReduceOp.SUM)
        dist.broadcast(flat, src=0)
        torch.cuda.synchronize()
        q.put((dist.get_backend(), torch.equal(sums, ref_s), torch.equal(flat, ref_f)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback
        q.put(("err", traceback.format_exc()))


def test_rccl_single_rank_collectives():
    """The RCCL backend ("nccl" on ROCm) on this box: a one-rank process group runs the collectives the
    data-parallel path issues (fp64 statistics totals, the fp32 gradient bucket, a broadcast) through
    RCCL.  The 1-GPU box cannot host a multi-rank RCCL group (one rank per GPU); the multi-rank
    arithmetic is covered by the gloo tests above and the driver's multi-GPU bench."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(29800 + os.getpid() % 1000, q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] != "err", res[1]
    assert res == ("nccl", True, True)
