"""Shared test helpers (build modules from golden fixtures, compare normwise)."""
import numpy as np
import torch


def normwise_rel(a, b):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).detach().double().cpu()
    den = max(float(torch.linalg.vector_norm(b)), 1e-30)
    return float(torch.linalg.vector_norm(a - b)) / den


def module_from_golden(pkg, g, device="cpu"):
    m = g["meta"]
    cls = {"Fp": pkg.Fp, "Fa": pkg.Fa, "FaFp": pkg.FaFp}[m["kind"]]
    kw = {}
    if m["net_sizes"] is not None:
        kw["net_sizes"] = m["net_sizes"]
    if m["aug_net_sizes"] is not None:
        kw["aug_net_sizes"] = m["aug_net_sizes"]
    mod = cls(m["n_regions"], latent_dim=m["latent_dim"], **kw)
    sd = {k: torch.from_numpy(g["w_" + k]) for k in m["state_dict_keys"]}
    mod.load_state_dict(sd, strict=True)
    if m["kind"] == "FaFp":
        mod.Fa_w = m.get("fa_w", 1.0)
    return mod.to(device)


def step_of(g):
    t = torch.from_numpy(g["t"])
    st = g["meta"]["step"]
    return t, (t[1] - t[0]) if st == "t1-t0" else st


def tol(g, key, floor=1e-5):
    """max(floor, 2 x the reference's own fp32-vs-fp64 distance on this case)."""
    return max(floor, 2.0 * g["meta"]["ref32_vs_ref64"].get(key, 0.0))


def kernel_forward_masks(pkg, mod, y0, t, step_size, eps=None):
    """The fused training forward (fp32, on mod's HIP device) of y0 with its training store kept:
    (latent (T, N, R, L) on the host, every evaluation's mask decisions on S, I, R -- (x > 2) |
    (x < -1) of the stage inputs the kernel evaluated, read from the store's stage-input checkpoints
    [tile][step][stage][3R][16] -- as an (E, N, R, 3) bool host tensor, E = 4 steps)."""
    from ude_amd import fused, solvers
    dev = next(mod.parameters()).device
    yd = y0.to(dev).contiguous()
    plan = solvers.plan_for(mod, yd, t, step_size)
    mod.clear_tracking()
    with torch.no_grad():
        if mod.uncertainty == "bayes":          # eps: the solve's (4 n_steps, n_params) draw stream
            mus, sds = mod.ude_mean_std()
            lat, _m, _s, _n, ckpt, _sums = fused.FusedBayesRK4.apply(plan, yd, eps.to(dev), True, *(mus + sds))
        else:
            params = [p for lin in mod.ude_linears() for p in (lin.weight, lin.bias)]
            lat, _m, _s, _n, ckpt, _tok, _sums = fused.FusedRK4.apply(plan, yd, True, *params)
    mod.clear_tracking()
    N, R, _L = y0.shape
    tiles = (N + 15) // 16
    E = 4 * plan.prob.n_steps
    dyn = ckpt[: tiles * E * 3 * R * 16].view(tiles, E, 3 * R, 16)
    x = dyn.permute(1, 0, 3, 2).reshape(E, tiles * 16, R, 3)[:, :N]
    masks = ((x > 2) | (x < -1)).cpu()
    return lat.cpu(), masks


def agreeing_trajectories(masks_a, masks_b):
    """(N,) bool: trajectories whose every evaluation takes the same mask decisions in a and b."""
    E, N = masks_a.shape[:2]
    return (masks_a == masks_b).reshape(E, N, -1).all(2).all(0)


class EvalMaskRecorder:
    """Records every evaluation's mask decisions on S, I, R of a module called one evaluation at a
    time (a forward pre-hook): ``masks`` (E, N, R, 3) bool on the host after ``close``."""

    def __init__(self, mod):
        self._m, self._g = [], []
        self._h = mod.register_forward_pre_hook(self._hook)

    def _hook(self, mod, args):
        x = args[1].detach()[..., :3]
        self._m.append(((x > 2) | (x < -1)).cpu())
        self._g.append(torch.minimum((x - 2).abs(), (x + 1).abs()).reshape(x.shape[0], -1).amin(1).cpu())

    def close(self):
        """(masks (E, N, R, 3), margin (N,): each trajectory's closest approach to the boundary)"""
        self._h.remove()
        self.masks = torch.stack(self._m)
        self.margin = torch.stack(self._g).amin(0)
        return self.masks


def kernel_forward_store(pkg, mod, y0, t, step_size):
    """The fused training forward (deterministic RHS, fp32, on mod's HIP device) with its training store
    kept: (latent (T, N, R, L), every stage input the kernel evaluated (E, N, R, 3) fp32 -- read from the
    store's checkpoints [tile][step][stage][3R][16] --, the solve's (mean, std, |Fa|) outputs), on the host."""
    from ude_amd import fused, solvers
    dev = next(mod.parameters()).device
    yd = y0.to(dev).contiguous()
    plan = solvers.plan_for(mod, yd, t, step_size)
    mod.clear_tracking()
    with torch.no_grad():
        params = [p for lin in mod.ude_linears() for p in (lin.weight, lin.bias)]
        lat, m, s, n, ckpt, _tok, _sums = fused.FusedRK4.apply(plan, yd, True, *params)
    mod.clear_tracking()
    N, R, _L = y0.shape
    tiles = (N + 15) // 16
    E = 4 * plan.prob.n_steps
    dyn = ckpt[: tiles * E * 3 * R * 16].view(tiles, E, 3 * R, 16)
    x = dyn.permute(1, 0, 3, 2).reshape(E, tiles * 16, R, 3)[:, :N]
    return lat.cpu(), x.cpu().contiguous(), (m.cpu(), s.cpu(), n.cpu())
