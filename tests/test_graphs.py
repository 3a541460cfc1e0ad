"""HIP-graph replay of the fused training step (ude_amd/graphs.py): the replayed
step runs the same kernels on the same buffers, so latent, posterior / |Fa| and every gradient are
bitwise the eager step's -- also after the weights are updated in place between replays (the captured
step re-packs them every replay)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(pkg, R, N, n_t, seed=0):
    torch.manual_seed(seed)
    mod = pkg.FaFp(R, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(DEV)
    gen = torch.Generator().manual_seed(seed + 1)
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, R, 5, generator=gen)], -1)
    y0 = (y0 + 1e-5).to(DEV).requires_grad_(True)
    t = torch.arange(n_t, dtype=torch.float32)
    dl = torch.randn((n_t, N, R, 8), generator=gen).to(DEV)
    cm, cs, cn = (torch.tensor([0.3, -0.2], device=DEV), torch.tensor([0.5, 0.1], device=DEV),
                  torch.tensor(0.1, device=DEV))
    def step():
        # gradients (re)assigned, not accumulated: inside a captured step this makes every replay
        # rewrite the gradient buffers the capture assigned
        mod.zero_grad(set_to_none=True)
        y0.grad = None
        mod.clear_tracking()
        lat = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=t[1] - t[0]))
        post = mod.posterior()
        nrm = torch.norm(torch.stack(mod.tracker))
        torch.autograd.backward([lat, post.loc, post.scale, nrm], [dl, cm, cs, cn])
        # detached: a step's outputs must not keep its autograd graph alive into the next (captured)
        # step, whose parameter AccumulateGrad nodes would then carry the earlier step's stream
        return tuple(o.detach() for o in (lat, post.loc, post.scale, nrm))
    return mod, y0, step


def _snapshot(mod, y0, outs):
    return [o.detach().clone() for o in outs] + [y0.grad.clone()] + [p.grad.clone() for p in mod.parameters()]


@pytest.mark.parametrize("R,N,n_t", [(49, 2048, 9), (1, 4096, 9)], ids=["state49_n2048", "us_n4096"])
def test_graph_replay_is_bitwise_the_eager_step(pkg, R, N, n_t):
    from ude_amd.graphs import GraphedStep
    mod, y0, step = _setup(pkg, R, N, n_t)

    def eager():
        outs = step()
        torch.cuda.synchronize()
        return _snapshot(mod, y0, outs)

    ref = eager()
    gs = GraphedStep(step, warmup=2)
    for _ in range(3):
        outs = gs.replay()
        torch.cuda.synchronize()
        got = _snapshot(mod, y0, outs)
        assert all(torch.equal(a, b) for a, b in zip(got, ref))
    # an in-place weight update between replays (an optimizer step): the replay re-packs
    with torch.no_grad():
        for p in mod.parameters():
            p.mul_(0.97)
    outs = gs.replay()
    torch.cuda.synchronize()
    got = _snapshot(mod, y0, outs)
    ref2 = eager()
    assert all(torch.equal(a, b) for a, b in zip(got, ref2))
    assert not torch.equal(ref2[0], ref[0])
