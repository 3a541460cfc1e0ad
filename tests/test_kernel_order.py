"""The kernel computes exactly the arithmetic it claims.

oracle/ude_korder.c restates the reference RHS (lib/models.py:109-265) under torchdiffeq's RK4
(lib/VAE.py:137) in the kernels' own operation order: fp32 fmaf chains in the MFMA K order, the
static-feature hoist, ROCm's expm1f, fp64 RK4 state with fp32 stage inputs.

* CPU (the checker is pinned before it is trusted): the restatement against the golden fixtures the
  reference generated (tests/golden, fp64): latent, dy0 and every weight gradient within the same bars
  as the kernel's own golden tests; its expm1f within 1 ulp of the correctly rounded value.
* GPU, arithmetic probes (tests/native/ude_probe.hip): one v_mfma_f32_16x16x4_f32 is the fmaf chain
  over its 4 K lanes in lane-group order 0..3, bitwise, on random operands spread over 2^±12; the device
  expm1f equals the restated one on EVERY float in [-17.5, 0] (and beyond -17.5 it is -1).
* GPU, whole solves: the fused training forward equals the restatement BIT FOR BIT -- every latent
  value and every stage input the kernel evaluated (so every mask decision of lib/models.py:130), on
  every golden shape and on the whole M1 north-star batches (4,096 x 365 daily steps, FaFp default
  init -- the batch with the ill-conditioned near-boundary trajectories -- and Fp [32, 32]) and the
  whole state49 batch (20,480 x R49); the statistics (posterior mean / std, |Fa|) to the last bit
  of their fp32 rounding.  The fused backward against the restatement's exact (fp64) VJP of that same
  fp32 forward -- no mask flip, no different branch, only the backward's own rounding left: dy0 and
  every dW / db within max(1e-6, 2 x the distance of ONE fp32 execution of the same VJP in the
  kernel's association from the exact one), and a weight gradient also within 1e-6 of its summed
  terms' magnitude.  The second term is the size of fp32 backward rounding on this forward: it
  matters only on the 4,096 x 365-step M1 batches, whose 1,460-evaluation adjoint recursions and
  6M-term weight-gradient sums are ~1e-5 from exact in any fp32 execution; on every golden shape and
  the state49 batch the kernel is within ~1e-6 outright.
  This comparison found the round-5 backward adding each stage's flux and MLP input gradients to the
  fp32 adjoint separately: on M1 Fp [32, 32] trajectories whose infected share grows exponentially the
  two nearly cancel, and dy0 was 5e-6 from exact (20x an fp32 execution that joins them first); the
  kernel now joins them first (Model::DYF).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import REPO, load_golden, solver_cases
from helpers import kernel_forward_store, module_from_golden, normwise_rel, step_of, tol
from oracle.ude_korder import KernelOrderOracle, expm1f, lib as ko_lib
from oracle.ude_oracle import OracleRHS

DEV = "cuda"
THREADS = int(os.environ.get("UDE_ORACLE_THREADS", "16"))
PROBE = os.path.join(REPO, "tests", "native", "_build", "libude_probe.so")
DM = torch.tensor([0.3, -0.2], dtype=torch.float64)
DS = torch.tensor([0.5, 0.1], dtype=torch.float64)
DN = 0.1
BAR_BWD = 1e-6


def _names_to_torch(mod, ko):
    """korder name (p_w0 ...) -> the module's parameter (ude_linears order: rate net, then aug net)."""
    lins = mod.ude_linears()
    out = {}
    for i, nm in enumerate([n for n in ko.names if "_w" in n]):
        out[nm] = lins[i].weight
        out[nm.replace("_w", "_b")] = lins[i].bias
    return out


# ---------------------------------------------------------------------------------------------------
# CPU: the restatement pinned by the reference's golden vectors

def test_korder_expm1f_within_one_ulp():
    x = -np.linspace(1e-7, 17.4, 1_000_001).astype(np.float32)
    y = expm1f(x)
    ref = np.expm1(x.astype(np.float64)).astype(np.float32)
    ulp = np.abs(y.view(np.int32).astype(np.int64) - ref.view(np.int32).astype(np.int64))
    assert ulp.max() <= 1, ulp.max()
    assert expm1f(np.array([-20.0, -0.0], np.float32)).tolist() == [-1.0, 0.0]


@pytest.mark.parametrize("case", solver_cases())
def test_korder_oracle_matches_golden(pkg, case):
    """The kernel-order restatement against the reference-generated fixtures (fp64): the same bars as
    the fused kernel's golden test (tests/test_gpu_parity.py)."""
    g = load_golden(case)
    mod = module_from_golden(pkg, g)
    t, h = step_of(g)
    ko = KernelOrderOracle(OracleRHS.from_module(mod, torch.float32))
    y0 = torch.from_numpy(g["y0"])
    out = ko.solve(y0, t, h, threads=4)
    assert normwise_rel(out["latent"], g["ref64_latent"]) <= tol(g, "latent")
    for key in ("mean", "std", "fa_norm"):
        if "ref64_" + key in g:
            assert normwise_rel(out[key], g["ref64_" + key]) <= tol(g, key)
    dm = torch.from_numpy(g["dmean"]) if "dmean" in g else None
    ds = torch.from_numpy(g["dstd"]) if "dstd" in g else None
    dn = float(g["dnorm"][0]) if "dnorm" in g else None
    dy0, gr, _ = ko.vjp(y0, t, h, torch.from_numpy(g["dlatent"]), dm, ds, dn, stats=out, threads=4)
    assert normwise_rel(dy0, g["ref64_d_y0"]) <= tol(g, "d_y0", 2e-5)
    tn = {id(p): n for n, p in mod.named_parameters()}
    for nm, p in _names_to_torch(mod, ko).items():
        k = "d_" + tn[id(p)]
        assert normwise_rel(gr[nm], g["ref64_" + k]) <= tol(g, k, 2e-5), (nm, k)


# ---------------------------------------------------------------------------------------------------
# GPU: arithmetic probes

def _probe():
    if not os.path.exists(PROBE):
        pytest.fail(f"{PROBE} missing: run __graft_entry__.build()")
    lp = ctypes.CDLL(PROBE)
    vp = ctypes.c_void_p
    lp.ude_probe_mfma.argtypes = [vp, vp, vp, vp, ctypes.c_int, vp]
    lp.ude_probe_expm1_bits.argtypes = [ctypes.c_uint32, ctypes.c_long, vp, vp]
    return lp


@pytest.mark.gpu
def test_mfma_f32_16x16x4_is_an_fmaf_chain_in_lane_order():
    lp = _probe()
    gen = torch.Generator().manual_seed(7)
    n = 512

    def spread(*shape):
        # mantissas in [1, 2), exponents over 2^-12 .. 2^12, random signs: partial sums of very
        # different magnitude, so every summation order rounds differently
        m = 1.0 + torch.rand(*shape, generator=gen)
        e = torch.randint(-12, 13, shape, generator=gen).double()
        s = torch.randint(0, 2, shape, generator=gen).double() * 2 - 1
        return (s * m.double() * torch.pow(2.0, e)).float()
    A, B, C = spread(n, 16, 4), spread(n, 4, 16), spread(n, 16, 16)
    D = torch.empty(n, 16, 16, device=DEV)
    Ad, Bd, Cd = A.to(DEV), B.to(DEV), C.to(DEV)
    assert lp.ude_probe_mfma(Ad.data_ptr(), Bd.data_ptr(), Cd.data_ptr(), D.data_ptr(), n,
                             torch.cuda.current_stream().cuda_stream) == 0
    D = D.cpu()
    import itertools
    f = ko_lib().ko_mfma_elem
    match = {}
    An, Bn, Cn, Dn = A.numpy(), B.numpy(), C.numpy(), D.numpy()
    for perm in itertools.permutations(range(4)):
        pa = (ctypes.c_int * 4)(*perm)
        ok = 0
        for c in range(0, n, 8):
            for i in range(16):
                for j in range(16):
                    a = np.ascontiguousarray(An[c, i, :])
                    b = np.ascontiguousarray(Bn[c, :, j])
                    acc = np.array([Cn[c, i, j]], np.float32)
                    f(a.ctypes.data, b.ctypes.data, pa, acc.ctypes.data)
                    ok += int(acc.view(np.int32)[0] == Dn[c:c + 1, i, j].view(np.int32)[0])
        match[perm] = ok
    total = (n // 8) * 256
    print("MFMA f32 16x16x4: elements matching an fmaf chain in lane order", {k: v for k, v in match.items() if v})
    assert match[(0, 1, 2, 3)] == total, (match[(0, 1, 2, 3)], total)


@pytest.mark.gpu
def test_device_expm1f_equals_restatement_on_every_float():
    """__ocml_expm1_f32 on the device vs ko_expm1f on every float in [-17.5, 0] (+0, -0, and the
    negative floats up to magnitude 17.5: the elu1 argument min(x, 0) on the range where expm1f is not
    the constant -1), bit for bit."""
    lp = _probe()
    start = 0x80000000                                  # -0.0
    stop = int(np.array([-17.5], np.float32).view(np.uint32)[0])
    total, chunk, bad = stop - start + 1, 1 << 27, 0
    y = torch.empty(chunk, dtype=torch.float32, device=DEV)
    first = ctypes.c_long(-1)
    for off in range(0, total, chunk):
        n = min(chunk, total - off)
        assert lp.ude_probe_expm1_bits(start + off, n, y.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        yh = y[:n].cpu().numpy()
        b = ko_lib().ko_expm1f_compare_bits(ctypes.c_uint32(start + off), ctypes.c_long(n), yh.ctypes.data,
                                            ctypes.byref(first))
        assert b == 0, f"{b} mismatches from bits {start + off + first.value:#x}"
        bad += b
    # +0 and the saturated range
    xs = torch.tensor([0.0, -17.6, -50.0, -1e30], dtype=torch.float32)
    ys = torch.empty(len(xs), device=DEV)
    for i, v in enumerate(xs.numpy()):
        assert lp.ude_probe_expm1_bits(int(np.array([v], np.float32).view(np.uint32)[0]), 1, ys[i:].data_ptr(),
                                       torch.cuda.current_stream().cuda_stream) == 0
    assert ys.cpu().numpy().tolist() == expm1f(xs.numpy()).tolist()
    print(f"device expm1f == restated expm1f on all {total} floats in [-17.5, -0]")


# ---------------------------------------------------------------------------------------------------
# GPU: whole solves, forward bitwise, backward against the exact VJP of the same forward

def _gpu_vjp(pkg, mod, y0, t, dl, h=None):
    """fused forward + VJP with the posterior / |Fa| terms; the cotangents the kernel receives are the
    fp32 roundings of dl, DM, DS, DN (returned, for the oracle)."""
    mg = mod.to(DEV)
    mg.zero_grad(set_to_none=True)
    yg = y0.to(DEV).requires_grad_(True)
    mg.clear_tracking()
    assert pkg.fusable(mg, yg)
    lat = pkg.odeint(mg, yg, t, method="rk4", options=dict(step_size=t[1] - t[0] if h is None else h))
    loss = (lat * dl.float().to(DEV)).sum()
    if mg.ode_type != "Fp":
        loss = loss + np.float32(DN) * torch.norm(torch.stack(mg.tracker))
    if mg.ode_type != "Fa":
        post = mg.posterior()
        loss = loss + (post.loc * DM.float().to(DEV)).sum() + (post.scale * DS.float().to(DEV)).sum()
    loss.backward()
    out = {"y0": yg.grad.cpu()}
    for lin_i, lin in enumerate(mg.ude_linears()):
        out[("w", lin_i)] = lin.weight.grad.cpu()
        out[("b", lin_i)] = lin.bias.grad.cpu()
    mod.cpu()
    return lat.detach().cpu(), out


def _check(pkg, mod, y0, t, dl, label, h=None):
    h = t[1] - t[0] if h is None else h
    mod = mod.to(DEV)
    lat_k, X_k, (m_k, s_k, n_k) = kernel_forward_store(pkg, mod, y0, t, h)
    lat_v, got = _gpu_vjp(pkg, mod, y0, t, dl, h)
    assert torch.equal(lat_v, lat_k)                      # the same forward, bit for bit
    mod = mod.cpu()
    ko = KernelOrderOracle(OracleRHS.from_module(mod, torch.float32))
    out = ko.solve(y0, t, h, stage_inputs=True, threads=THREADS)
    n_lat = int((out["latent"] != lat_k).sum())
    n_x = int((out["stage_inputs"] != X_k).sum())
    bad_traj = ((out["stage_inputs"] != X_k).reshape(X_k.shape[0], X_k.shape[1], -1).any(2).any(0)).nonzero()
    print(f"{label}: latent {lat_k.numel()} values, {n_lat} differ from the kernel-order restatement; "
          f"stage inputs {X_k.numel()} values, {n_x} differ (trajectories {bad_traj.flatten()[:8].tolist()})")
    assert n_lat == 0 and n_x == 0
    kind = mod.ode_type
    if kind != "Fa":
        assert torch.equal(out["mean"], m_k) and torch.equal(out["std"], s_k), (out["mean"], m_k, out["std"], s_k)
    if kind != "Fp":
        assert torch.equal(out["fa_norm"], n_k), (out["fa_norm"], n_k)
    dl32 = dl.float().double()
    dy0, gr, mag = ko.vjp(y0, t, h, dl32, DM.float().double(), DS.float().double(), float(np.float32(DN)),
                          stats=out, threads=THREADS)
    errs = {"y0": normwise_rel(got["y0"], dy0)}
    rel_mag = {}
    wn = [n for n in ko.names if "_w" in n]
    for i, nm in enumerate(wn):
        for kk, key in ((nm, ("w", i)), (nm.replace("_w", "_b"), ("b", i))):
            errs[kk] = normwise_rel(got[key], gr[kk])
            # the same difference against the magnitude of the summed terms (the scale of fp32 rounding)
            rel_mag[kk] = float((got[key].double() - gr[kk]).norm() / max(float(mag[kk].norm()), 1e-30))
    # the size of fp32 backward rounding on this very forward: the same VJP executed in fp32 in the
    # kernel's association (ko_set_assoc(1): the step's adjoint accumulated as the kernel's bwd_body does,
    # one update per stage; per-tile fp32 weight-gradient sums, then the tiles, like the kernel's slabs)
    ko_lib().ko_set_assoc(1)
    try:
        dy0_32, gr32, _ = ko.vjp(y0, t, h, dl32, DM.float().double(), DS.float().double(), float(np.float32(DN)),
                                 stats=out, threads=THREADS, fp32=True)
    finally:
        ko_lib().ko_set_assoc(0)
    ref32 = {"y0": normwise_rel(dy0_32, dy0)}
    ref32.update({k: normwise_rel(gr32[k], gr[k]) for k in gr})
    dd = lambda a, b: normwise_rel(a, b)
    d2 = (got["y0"].double() - dy0).reshape(dy0.shape[0], -1).pow(2).sum(1)
    top = torch.topk(d2, min(4, dy0.shape[0]))
    print(f"  dy0 split: S, I, R dims {dd(got['y0'][..., :3], dy0[..., :3]):.1e} [{dd(dy0_32[..., :3], dy0[..., :3]):.1e}], "
          f"static dims {dd(got['y0'][..., 3:], dy0[..., 3:]):.1e} [{dd(dy0_32[..., 3:], dy0[..., 3:]):.1e}]; worst "
          f"trajectories {top.indices.tolist()} carry {float(top.values.sum() / d2.sum()):.2f} of the kernel's dy0 error^2")
    print(f"  kernel backward vs the exact VJP of the kernel-order forward [fp32 execution of that VJP]: "
          + ", ".join(f"{k} {v:.1e} [{ref32[k]:.1e}]" for k, v in errs.items()))
    print("  (kernel difference / |summed terms|: " + ", ".join(f"{k} {v:.1e}" for k, v in rel_mag.items()) + ")")
    # bar: max(1e-6, 2 x the fp32 execution's distance) normwise; for a weight gradient (a sum of
    # N x E terms) also 1e-6 of the summed terms' magnitude -- the standard measure of a long fp32
    # summation's rounding, which cancellation in the sum does not shrink (Higham, ch. 4)
    bars = {k: max(BAR_BWD, 2.0 * ref32[k]) for k in errs}
    for k in rel_mag:
        bars[k] = max(bars[k], BAR_BWD * float(mag[k].norm()) / max(float(gr[k].norm()), 1e-30))
    over = {k: (v, bars[k]) for k, v in errs.items() if v > bars[k]}
    assert not over, f"{label}: kernel backward vs the exact VJP of its own forward above its bar: {over}"


def _y0(N, R, L, seed):
    gen = torch.Generator().manual_seed(seed)
    S = torch.rand(N, R, generator=gen) * 0.4 + 0.5
    I = torch.rand(N, R, generator=gen) * 0.05
    y0 = torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, R, L - 3, generator=gen)], -1)
    return y0 + 1e-5, gen


@pytest.mark.gpu
@pytest.mark.parametrize("case", solver_cases())
def test_kernel_equals_korder_on_golden_shapes(pkg, case):
    g = load_golden(case)
    mod = module_from_golden(pkg, g)
    t, h = step_of(g)
    y0 = torch.from_numpy(g["y0"]).float()
    _check(pkg, mod, y0, t, torch.from_numpy(g["dlatent"]), case, h)


@pytest.mark.gpu
@pytest.mark.timeout(1500)
@pytest.mark.parametrize("kind,net,aug", [("FaFp", [64, 64, 32], [64, 64]), ("Fp", [32, 32], None)],
                         ids=["FaFp_64_64_32", "Fp_32_32"])
def test_kernel_equals_korder_m1_whole_batch(pkg, kind, net, aug):
    """M1 (4,096 x 365 daily steps), the batch and seed of tests/test_north_star.py (FaFp default init:
    trajectory #2994 passes 4e-5 from the mask boundary with |dy0| = 1.8e5)."""
    torch.manual_seed(0)
    kw = {"net_sizes": net}
    if aug:
        kw["aug_net_sizes"] = aug
    mod = getattr(pkg, kind)(1, latent_dim=8, **kw)
    y0, gen = _y0(4096, 1, 8, 11)
    t = torch.arange(366, dtype=torch.float32) / 7.0
    dl = torch.randn((366, 4096, 1, 8), generator=gen, dtype=torch.float64)
    _check(pkg, mod, y0, t, dl, f"M1 {kind}")


@pytest.mark.gpu
@pytest.mark.timeout(1500)
def test_kernel_equals_korder_state49_whole_batch(pkg):
    """BASELINE configs[1]: 20,480 trajectories x R = 49, 8 weekly steps (tests/test_north_star.py's batch)."""
    torch.manual_seed(0)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    y0, gen = _y0(20480, 49, 8, 5)
    t = torch.arange(9, dtype=torch.float32)
    dl = torch.randn((9, 20480, 49, 8), generator=gen, dtype=torch.float64)
    _check(pkg, mod, y0, t, dl, "state49")
