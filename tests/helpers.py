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
