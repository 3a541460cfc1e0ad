"""North-star accuracy at full size (BASELINE.json north_star: "trajectories within 1e-5 rel-err
of reference" on the 4096-trajectory x 365-step fp32 batch), fused gfx950 forward + VJP against
the fp64 CPU oracle.

* M1: US FaFp R=1 [64,64,32]/[64,64] and Fp [32,32], N = 4096, t = arange(366)/7,
  365 daily RK4 steps (1,460 RHS evaluations per trajectory), forward and backward.  The oracle
  runs chunked over trajectories (exact: the side statistics enter the gradient linearly once
  their global values are known, oracle/ude_oracle.py solve_and_grad_chunked) on spawned CPU
  workers.  The whole batch is also compared with the fp32 oracle (the reference's own
  arithmetic).  Bars (written in each test): trajectories split by whether the kernel took the
  fp64 oracle's mask decision ((x > 2) | (x < -1), lib/models.py:130) at every evaluation --
  the agreeing ones' latent <= 1e-5 and dy0 <= 2e-5; the agreeing ones as a batch: posterior /
  |Fa| <= 1e-5, every weight gradient <= max(2e-5, 2 x the fp32 oracle's own distance).
* BASELINE configs[1] (20,480 trajectories, R = 49): the whole batch against the fp64 oracle,
  reductions included (every dW / db, posterior mean / std, |Fa|).
* R = 1 with more tiles than CUs (16,384 trajectories): the M3 launch of the training forward.
* BASELINE configs[2] (dopri5 on the same batch): bit-reproducible, torchdiffeq's evaluation
  count (2 + 6 per attempt), and within the solve tolerance of the fused RK4 at a fine fixed step.
"""
import os

import pytest
import torch

from helpers import agreeing_trajectories, kernel_forward_masks, normwise_rel
from oracle.ude_oracle import OracleRHS, solve_and_grad_chunked

pytestmark = pytest.mark.gpu

DEV = "cuda"
WORKERS = int(os.environ.get("UDE_ORACLE_WORKERS", "12"))
DM = torch.tensor([0.3, -0.2], dtype=torch.float64)
DS = torch.tensor([0.5, 0.1], dtype=torch.float64)
DN = 0.1


def _y0(N, R, L, seed):
    gen = torch.Generator().manual_seed(seed)
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, R, L - 3, generator=gen)], -1)
    return y0 + 1e-5, gen


def _gpu_vjp(pkg, mod, y0, t, dl, stats=True):
    mg = mod.to(DEV)
    mg.zero_grad(set_to_none=True)
    yg = y0.to(DEV).requires_grad_(True)
    mg.clear_tracking()
    assert pkg.fusable(mg, yg)
    lat = pkg.odeint(mg, yg, t, method="rk4", options=dict(step_size=t[1] - t[0]))
    out = {"latent": lat.detach().cpu()}
    loss = (lat.double() * dl.to(DEV)).sum()
    if stats:
        if mg.ode_type != "Fp":
            nrm = torch.norm(torch.stack(mg.tracker))
            out["fa_norm"] = nrm.detach().cpu()
            loss = loss + DN * nrm
        if mg.ode_type != "Fa":
            post = mg.posterior()
            out["mean"], out["std"] = post.loc.detach().cpu(), post.scale.detach().cpu()
            loss = loss + (post.loc.double() * DM.to(DEV)).sum() + (post.scale.double() * DS.to(DEV)).sum()
    loss.backward()
    out["y0"] = yg.grad.cpu()
    names = []
    lins = mg.ude_linears()
    pref = ["p"] * (len(lins) if mg.ode_type == "Fp" else 0)
    if mg.ode_type == "FaFp":
        n_p = len([m for m in mg.net if isinstance(m, torch.nn.Linear)])
        pref = ["p"] * n_p + ["a"] * (len(lins) - n_p)
    elif mg.ode_type == "Fa":
        pref = ["a"] * len(lins)
    cnt = {"p": 0, "a": 0}
    for lin, pr in zip(lins, pref):
        i = cnt[pr]
        cnt[pr] += 1
        out[f"{pr}_w{i}"] = lin.weight.grad.cpu()
        out[f"{pr}_b{i}"] = lin.bias.grad.cpu()
        names += [f"{pr}_w{i}", f"{pr}_b{i}"]
    mod.cpu()
    return out, names


def _scale_outputs(mod, sp, sa):
    """Rate-net output layer x sp, augmentation-net output layer x sa."""
    with torch.no_grad():
        for name, s in (("net", sp), ("Fp_net", sp), ("aug_net", sa)):
            if hasattr(mod, name) and s != 1.0:
                getattr(mod, name)[-1].weight.mul_(s)
                getattr(mod, name)[-1].bias.mul_(s)


def _oracle(mod, y0, t, dl, dtype, stats=True, masks=True, chunk=512, k_order="torch"):
    """The chunked oracle (oracle/ude_oracle.py solve_and_grad_chunked) in ``dtype`` on spawned
    CPU workers: latent, posterior / |Fa|, every gradient, every evaluation's mask decisions.
    k_order="rev4": the same arithmetic with every Linear's products summed in another order."""
    dm, ds, dn = (DM.to(dtype), DS.to(dtype), DN) if stats else (None, None, None)
    rhs = OracleRHS.from_module(mod, dtype)
    rhs.k_order = k_order
    return solve_and_grad_chunked(rhs, y0.to(dtype), t, t[1] - t[0],
                                  None if dl is None else dl.to(dtype), dm, ds, dn, chunk=chunk,
                                  workers=WORKERS, masks=masks)


def _res_dict(res, names):
    out = {"latent": res.latent, "y0": res.grads["y0"]}
    for k in ("mean", "std", "fa_norm"):
        if getattr(res, k) is not None:
            out[k] = getattr(res, k)
    for k in names:
        out[k] = res.grads[k]
    return out


def _errs(a, b):
    return {k: normwise_rel(a[k], b[k]) for k in b if k in a}


def _fmt(d):
    return ", ".join(f"{k} {v:.2e}" for k, v in d.items())


STAT_KEYS = ("latent", "mean", "std", "fa_norm")
# closest approach of a trajectory's stage inputs to the mask boundary below which its gradient is
# treated as ill-conditioned (fp32 rounding alone moves it by more than the 2e-5 bar there)
MARGIN = 1e-3


def _assert_bars(errs, label, mod, y0, t, dl, names):
    """latent / posterior / |Fa| <= 1e-5 (north_star); every gradient <= max(2e-5, 2 x the fp32
    oracle's own distance to fp64), the fp32 oracle run only when a gradient is above the floor."""
    for k in STAT_KEYS:
        if k in errs:
            assert errs[k] <= 1e-5, f"{label} {k}: {errs[k]:.3e} > 1e-5"
    over = [k for k, v in errs.items() if k not in STAT_KEYS and v > 2e-5]
    if over:
        o64 = _res_dict(_oracle(mod, y0, t, dl, torch.float64, masks=False), names)
        o32 = _res_dict(_oracle(mod, y0, t, dl, torch.float32, masks=False), names)
        for k in over:
            bar = 2.0 * normwise_rel(o32[k], o64[k])
            print(f"  {label} {k}: {errs[k]:.2e} vs the fp32 oracle's own {bar / 2:.2e}")
            assert errs[k] <= bar, f"{label} {k}: {errs[k]:.3e} > max(2e-5, {bar:.3e})"


def _full_batch(pkg, mod, y0, t, dl, label, fp32_whole=False):
    """Whole batch on the GPU (training forward with its store kept, for the kernel's own mask
    decisions; then forward + VJP with the posterior / |Fa| terms) against the fp64 oracle over the
    same batch.  Trajectories are split by whether the kernel took the fp64 oracle's mask decision
    ((x > 2) | (x < -1) on S, I, R, lib/models.py:130 -- a discontinuity of the RHS) at every one of
    their evaluations.  fp32_whole: also the fp32 oracle (the reference's own arithmetic) over the
    whole batch, and the kernel's distance to it."""
    h = t[1] - t[0]
    N = y0.shape[0]
    mg = mod.to(DEV)
    lat_k, mk = kernel_forward_masks(pkg, mg, y0, t, h)
    got, names = _gpu_vjp(pkg, mod, y0, t, dl)
    assert torch.equal(got["latent"], lat_k)          # the same training forward, bit for bit
    r64 = _oracle(mod, y0, t, dl, torch.float64)
    ref = _res_dict(r64, names)
    agree = agreeing_trajectories(mk, r64.masks)
    K = int(agree.sum())
    ever = int(r64.masks.reshape(r64.masks.shape[0], N, -1).any(2).any(0).sum())
    whole = _errs(got, ref)
    lines = [f"{label}: {K}/{N} trajectories take the fp64 oracle's mask decision at every evaluation "
             f"({ever} are masked at some evaluation)",
             "  whole batch, kernel vs fp64: " + _fmt(whole)]
    r32 = None
    if fp32_whole:
        r32 = _oracle(mod, y0, t, dl, torch.float32)
        o32 = _res_dict(r32, names)

        agree32 = agreeing_trajectories(r32.masks, r64.masks)
        k32 = int(agree32.sum())
        lines.append(f"  fp32 oracle: {k32}/{N} trajectories agree with fp64; the kernel and the fp32 "
                     f"oracle decide alike on {int(agreeing_trajectories(mk, r32.masks).sum())}")
        lines.append("  whole batch, fp32 oracle vs fp64: " + _fmt(_errs(o32, ref)))
        lines.append("  whole batch, kernel vs fp32 oracle: " + _fmt(_errs(got, o32)))
        if k32:
            lines.append(f"  fp32 oracle on its {k32} agreeing trajectories: latent "
                         f"{normwise_rel(r32.latent[:, agree32], r64.latent[:, agree32]):.2e}, y0 "
                         f"{normwise_rel(r32.grads['y0'][agree32], r64.grads['y0'][agree32]):.2e}")
    split = {}
    if K:
        split["latent"] = normwise_rel(got["latent"][:, agree], r64.latent[:, agree])
        split["y0"] = normwise_rel(got["y0"][agree], r64.grads["y0"][agree])
    diff = (got["y0"].double() - r64.grads["y0"].double()).reshape(N, -1).pow(2).sum(1)
    share = float(diff[~agree].sum() / diff.sum()) if float(diff.sum()) > 0 else 0.0
    lines.append(f"  kernel on its {K} agreeing trajectories: " + _fmt(split) +
                 f"; the {N - K} disagreeing ones carry {100 * share:.1f}% of the whole-batch dy0 error^2")
    # where the dy0 error sits: the worst trajectories, their share, the fp32 oracle's error on them and
    # their closest approach to the mask boundary (fp64 stage inputs)
    den = float(r64.grads["y0"].double().pow(2).sum())
    top = torch.topk(diff, min(8, N))
    parts = []
    for i in top.indices.tolist():
        e32 = ""
        if r32 is not None:
            d32 = float((r32.grads["y0"][i].double() - r64.grads["y0"][i].double()).pow(2).sum())
            e32 = f"/{(d32 / den) ** 0.5:.1e}"
        parts.append(f"#{i} {(float(diff[i]) / den) ** 0.5:.1e}{e32} m={float(r64.margin[i]):.1e}")
    lines.append(f"  worst dy0 trajectories (kernel/fp32-oracle error, normwise over the batch; m = margin): "
                 + ", ".join(parts) + f"; they carry {100 * float(top.values.sum() / diff.sum()):.1f}%")
    for thr in (1e-4, 1e-3, 1e-2):
        far = agree & (r64.margin > thr)
        if int(far.sum()):
            lines.append(f"  agreeing with margin > {thr:g}: {int(far.sum())} trajectories, dy0 "
                         f"{normwise_rel(got['y0'][far], r64.grads['y0'][far]):.2e}")
    split["near"] = agree & ~(r64.margin > MARGIN)
    split["far"] = agree & (r64.margin > MARGIN)
    split["margin"] = r64.margin
    if fp32_whole and int(split["near"].sum()):
        # the agreeing trajectories that come within MARGIN of the mask boundary: the same fp32
        # arithmetic with another summation order (k_order rev4) samples how far fp32 rounding moves
        # their (ill-conditioned) gradients
        nb = split["near"]
        # (their own batch, the latent term of the loss only: fp32 orders against fp64 of the same loss)
        yn, dn = y0[nb].contiguous(), dl[:, nb].contiguous()
        alt = _oracle(mod, yn, t, dn, torch.float32, stats=False, masks=False, k_order="rev4")
        alt64 = _oracle(mod, yn, t, dn, torch.float64, stats=False, masks=False)
        r32.near_alt = normwise_rel(alt.grads["y0"], alt64.grads["y0"])
        lines.append(f"  the {int(nb.sum())} agreeing trajectories within {MARGIN:g} of the boundary: dy0 kernel "
                     f"{normwise_rel(got['y0'][nb], r64.grads['y0'][nb]):.2e}, fp32 oracle "
                     f"{normwise_rel(r32.grads['y0'][nb], r64.grads['y0'][nb]):.2e}, fp32 oracle in another "
                     f"summation order {r32.near_alt:.2e}")
    print("\n".join(lines))
    return got, ref, r32, agree, names, whole, split


# The whole-batch spread bar: PRE-REGISTERED samples of the fp32 reference
# arithmetic, every one run on every call (nothing stops early, the list does not grow):
#  * the torch oracle (oracle/ude_oracle.py) in fp32 with every Linear's K products summed in torch's
#    own order, in blocks of 4 last block first ("rev4") and first block first ("fwd4");
#  * "korder32": the reference arithmetic in the kernel's own MLP order -- oracle/ude_korder.c with
#    torchdiffeq's fp32 RK4 state (state32) and the exact VJP of that forward.  It differs from the
#    kernel in one thing only, the fp64 RK state the kernel carries (fwd_body), so it measures how far
#    the reference's own fp32 integrator arithmetic lands from fp64 with the kernel's summation order.
# (tests/test_kernel_order.py proves separately that the kernel's forward IS the kernel-order
# arithmetic, bit for bit, and its backward that forward's exact VJP up to fp32 backward rounding.)
FP32_ORDERS = ("torch", "rev4", "fwd4", "korder32")


def _korder32(mod, y0, t, dl, names):
    from oracle.ude_korder import KernelOrderOracle
    h = t[1] - t[0]
    ko = KernelOrderOracle(OracleRHS.from_module(mod, torch.float32), state32=True)
    st = ko.solve(y0, t, h, threads=WORKERS)
    kind = mod.ode_type
    dy0, gr, _ = ko.vjp(y0, t, h, dl, DM if kind != "Fa" else None, DS if kind != "Fa" else None,
                        DN if kind != "Fp" else None, stats=st, threads=WORKERS)
    out = {"latent": st["latent"], "y0": dy0}
    out.update({k: gr[k] for k in names})
    return out


def _assert_whole_within_fp32_spread(label, mod, y0, t, dl, names, whole, ref, r32=None):
    """The WHOLE batch's dy0 and every dW / db (near-boundary trajectories included) vs fp64 within
    max(2e-5, 2 x the farthest of the fixed fp32 samples FP32_ORDERS vs fp64)."""
    sp = []
    for ko in FP32_ORDERS:
        if ko == "korder32":
            sp.append(_errs(_korder32(mod, y0, t, dl, names), ref))
            continue
        r = r32 if (ko == "torch" and r32 is not None) else _oracle(mod, y0, t, dl, torch.float32, masks=False,
                                                                   k_order=ko)
        sp.append(_errs(_res_dict(r, names), ref))
    keys = ["y0"] + list(names)
    bad = [(k, whole[k], max(2e-5, 2.0 * max(s_[k] for s_ in sp))) for k in keys]
    bad = [b for b in bad if b[1] > b[2]]
    lines = [f"{k} {whole[k]:.2e} [" + "/".join(f"{s_[k]:.1e}" for s_ in sp) + "]" for k in keys]
    print(f"  {label}, whole batch vs fp64 [fp32 {' / '.join(FP32_ORDERS)} vs fp64]: " + ", ".join(lines))
    assert not bad, f"{label}: outside max(2e-5, 2 x the fixed fp32 spread {FP32_ORDERS}): {bad}"


def _agreeing_batch(pkg, mod, y0, t, dl, agree, names, label):
    """The given (agreeing, away-from-the-boundary) trajectories solved as a batch of their own:
    posterior / |Fa| and every weight gradient against the fp64 oracle over the same trajectories."""
    yk, dk = y0[agree].contiguous(), dl[:, agree].contiguous()
    gk, _ = _gpu_vjp(pkg, mod, yk, t, dk)
    rk = _res_dict(_oracle(mod, yk, t, dk, torch.float64, masks=False), names)
    errs = _errs(gk, rk)
    print(f"  the {int(agree.sum())} agreeing trajectories as one batch: " + _fmt(errs))
    _assert_bars(errs, label, mod, yk, t, dk, names)


@pytest.mark.timeout(2400)
@pytest.mark.parametrize("kind,net,aug,sa", [("FaFp", [64, 64, 32], [64, 64], 1.0),
                                             ("FaFp", [64, 64, 32], [64, 64], 0.01),
                                             ("Fp", [32, 32], None, 1.0)],
                         ids=["FaFp_64_64_32", "FaFp_64_64_32_Fa_x0.01", "Fp_32_32"])
def test_north_star_m1_full_size(pkg, kind, net, aug, sa):
    """M1 (4096 x 365 daily steps, 1,460 evaluations per trajectory), whole batch, forward + VJP,
    against the fp64 oracle and against the fp32 oracle (the reference's own arithmetic).

    The RHS is masked to zero outside [-1, 2] (lib/models.py:130): with the default init nearly
    every FaFp trajectory crosses that boundary within the year, and a trajectory whose evaluation
    lands next to it is masked or not by rounding -- its gradient then follows another branch of a
    discontinuous map.  Bars: every trajectory whose evaluations all take the fp64
    oracle's mask decisions -- latent <= 1e-5, dy0 <= max(2e-5, 2 x the fp32 oracle's own distance,
    the farther of two fp32 oracle runs that differ only in GEMM blocking: with the default init a few
    ill-conditioned trajectories make that distance swing by ~10x between fp32 roundings); those
    trajectories solved as a batch of their own -- posterior / |Fa| <= 1e-5, every weight gradient
    <= max(2e-5, 2 x the fp32 oracle's own distance); the whole batch's
    latent <= 1e-5, or <= 2 x the fp32 oracle's own distance.  The counts, the fp32 oracle's own
    numbers and the disagreeing trajectories' share of the whole-batch dy0 error are printed."""
    torch.manual_seed(0)
    kw = {"net_sizes": net} if net else {}
    if aug:
        kw["aug_net_sizes"] = aug
    mod = getattr(pkg, kind)(1, latent_dim=8, **kw)
    _scale_outputs(mod, 1.0, sa)
    N, n_t = 4096, 366
    y0, gen = _y0(N, 1, 8, 11)
    t = torch.arange(n_t, dtype=torch.float32) / 7.0
    dl = torch.randn((n_t, N, 1, 8), generator=gen, dtype=torch.float64)
    label = f"north-star {kind} (Fa x{sa})"
    got, ref, r32, agree, names, whole, split = _full_batch(pkg, mod, y0, t, dl, label, fp32_whole=True)
    if whole["latent"] > 1e-5:
        bar = 2.0 * normwise_rel(r32.latent, ref["latent"])
        assert whole["latent"] <= bar, f"whole-batch latent {whole['latent']:.3e} > 2 x the fp32 oracle's {bar / 2:.3e}"
    assert int(agree.sum()) >= 16, "too few agreeing trajectories for the gradient check"
    assert split["latent"] <= 1e-5, split
    # dy0: the agreeing trajectories that keep their distance from the boundary <= 2e-5; those that come
    # within MARGIN of it <= max(2e-5, 2 x the farther of two fp32 roundings of the reference arithmetic)
    far = split["far"]
    e_far = normwise_rel(got["y0"][far], ref["y0"][far])
    assert int(far.sum()) >= 16 and e_far <= 2e-5, (int(far.sum()), e_far)
    nb = split["near"]
    if int(nb.sum()):
        e_nb = normwise_rel(got["y0"][nb], ref["y0"][nb])
        bar = max(2e-5, 2.0 * max(normwise_rel(r32.grads["y0"][nb], ref["y0"][nb]), r32.near_alt))
        assert e_nb <= bar, (e_nb, bar)
    # the batch sums (posterior, |Fa|, every weight gradient) over the well-conditioned trajectories
    _agreeing_batch(pkg, mod, y0, t, dl, far, names, label)
    # and over the whole batch, against the fp32 reference arithmetic's own spread
    _assert_whole_within_fp32_spread(label, mod, y0, t, dl, names, whole, ref, r32)


@pytest.mark.timeout(2400)
def test_state49_full_batch_vs_oracle(pkg):
    """BASELINE configs[1] at full size: 20,480 trajectories x R = 49, 8 weekly steps, forward + VJP
    with the posterior / |Fa| terms, the WHOLE batch against the fp64 oracle (chunked on CPU
    workers): latent, posterior mean / std, |Fa| <= 1e-5; dy0 and every dW / db -- the 1,280-tile
    fixed-order slab reduction + ude_grad_finalize -- <= max(2e-5, 2 x the fp32 oracle's own
    distance).  If some trajectory's mask decisions differed from fp64 the bars would move to the
    agreeing trajectories (the count is printed)."""
    torch.manual_seed(0)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    N = 20480
    y0, gen = _y0(N, 49, 8, 5)
    t = torch.arange(9, dtype=torch.float32)
    dl = torch.randn((9, N, 49, 8), generator=gen, dtype=torch.float64)
    got, ref, r32, agree, names, whole, split = _full_batch(pkg, mod, y0, t, dl, "state49 full batch",
                                                            fp32_whole=True)
    if int(agree.sum()) == N:
        _assert_bars(whole, "state49", mod, y0, t, dl, names)
    else:
        assert split["latent"] <= 1e-5 and split["y0"] <= 2e-5, split
        _agreeing_batch(pkg, mod, y0, t, dl, agree, names, "state49 agreeing")
    for k in STAT_KEYS[1:]:
        assert whole[k] <= 1e-5, (k, whole[k])
    # the whole batch's latent too, <= max(1e-5, 2 x the fp32 reference arithmetic's)
    bar = max(1e-5, 2.0 * normwise_rel(r32.latent, ref["latent"]))
    assert whole["latent"] <= bar, f"state49 whole-batch latent {whole['latent']:.3e} > {bar:.3e}"
    # the batch's dy0 and every dW / db within the fixed fp32 spread
    _assert_whole_within_fp32_spread("state49", mod, y0, t, dl, names, whole, ref, r32)


@pytest.mark.timeout(1500)
@pytest.mark.parametrize("kind,net,aug", [("FaFp", [64, 64, 32], [64, 64]), ("Fp", [32, 32], None)],
                         ids=["FaFp_64_64_32", "Fp_32_32"])
def test_r1_more_tiles_than_cus_full_batch(pkg, kind, net, aug):
    """R = 1 with more tiles than CUs (16,384 trajectories = 1,024 tiles): the 4-wave training forward
    at two workgroups per CU (ude_entry.h, the M3 launch) instead of the one-tile-per-CU split
    forward the smaller R = 1 tests take.  Whole batch, 8 weekly steps, against the fp64 oracle:
    latent / posterior / |Fa| <= 1e-5, dy0 and every weight gradient <= max(2e-5, 2 x fp32 oracle)."""
    torch.manual_seed(1)
    kw = {"net_sizes": net}
    if aug:
        kw["aug_net_sizes"] = aug
    mod = getattr(pkg, kind)(1, latent_dim=8, **kw)
    N = 16384
    y0, gen = _y0(N, 1, 8, 13)
    t = torch.arange(9, dtype=torch.float32)
    dl = torch.randn((9, N, 1, 8), generator=gen, dtype=torch.float64)
    got, ref, _, agree, names, whole, split = _full_batch(pkg, mod, y0, t, dl, f"R=1 {kind} N={N}")
    if int(agree.sum()) == N:
        _assert_bars(whole, f"R=1 {kind}", mod, y0, t, dl, names)
    else:
        assert split["latent"] <= 1e-5 and split["y0"] <= 2e-5, split
        _agreeing_batch(pkg, mod, y0, t, dl, agree, names, f"R=1 {kind} agreeing")


@pytest.mark.timeout(600)
def test_dopri5_full_batch_properties(pkg):
    torch.manual_seed(0)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    # output layers scaled by 0.1: slow rates, so S, I, R stay inside [-1, 2] (the RHS is masked,
    # i.e. discontinuous, at that boundary, where two solvers' crossing times differ)
    with torch.no_grad():
        mod.net[-1].weight.mul_(0.1); mod.net[-1].bias.mul_(0.1)
        mod.aug_net[-1].weight.mul_(0.1); mod.aug_net[-1].bias.mul_(0.1)
    mod = mod.to(DEV)
    y0, _ = _y0(20480, 49, 8, 5)
    y0 = y0.to(DEV)
    t = torch.arange(9, dtype=torch.float32).to(DEV)
    runs = []
    for _ in range(2):
        mod.clear_tracking()
        with torch.no_grad():
            lat = pkg.odeint(mod, y0, t, method="dopri5", rtol=1e-6, atol=1e-8)
        post = mod.posterior()
        runs.append((lat, post.loc.clone(), post.scale.clone(), dict(mod.last_solve_info)))
    (l1, m1, s1, i1), (l2, m2, s2, i2) = runs
    assert torch.equal(l1, l2) and torch.equal(m1, m2) and torch.equal(s1, s2) and i1 == i2
    assert i1["n_evals"] == 2 + 6 * i1["n_steps"], i1
    assert i1["n_accepted"] <= i1["n_steps"]
    # the fused RK4 at a fine fixed step (1/16) is an independent solution of the same IVP
    mod.clear_tracking()
    with torch.no_grad():
        fine = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=1.0 / 16))
    sir = fine[..., :3]
    inside = bool(((sir > -1) & (sir < 2)).all())
    err = normwise_rel(l1[..., :3], fine[..., :3])
    print(f"dopri5 full batch: {i1}, S/I/R vs fine RK4 {err:.2e} (every state inside [-1, 2]: {inside})")
    assert inside and err < 1e-5
