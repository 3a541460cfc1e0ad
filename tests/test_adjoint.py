"""odeint_adjoint (torchdiffeq's adjoint API; BASELINE configs[2] "adjoint backward").

CPU: known-answer tests of the adjoint gradient (linear ODE vs the matrix exponential), the
product adjoint (ude_amd/adjoint.py) against the oracle's independent restatement
(oracle/ude_oracle_adjoint.py), and the adjoint against autograd through the forward solve
at tight tolerances.  GPU: UDE modules on the MI355X -- forward = the fused dopri5 solve,
backward = the augmented solve whose every evaluation is the gfx950 evaluation + VJP kernels
-- against the oracle adjoint in fp64 on the host.

torchdiffeq is absent (unpinned dependency of the reference), so parity with torchdiffeq
itself is unpinned; the KATs pin the algorithm."""
import pytest
import torch

from helpers import normwise_rel
from oracle.ude_oracle import OracleRHS
from oracle.ude_oracle_adjoint import adjoint_backward
from oracle.ude_oracle_dopri5 import odeint_dopri5


class _Linear(torch.nn.Module):
    def __init__(self, A):
        super().__init__()
        self.A = torch.nn.Parameter(A.clone())

    def forward(self, t, y):
        return y @ self.A.T


def test_adjoint_linear_ode_matches_matrix_exponential(pkg):
    from torchdiffeq import odeint_adjoint
    torch.manual_seed(0)
    A = torch.randn(3, 3, dtype=torch.float64) * 0.5
    y0 = torch.randn(4, 3, dtype=torch.float64).requires_grad_(True)
    t = torch.tensor([0.0, 0.4, 1.1], dtype=torch.float64)
    c = torch.randn(3, 4, 3, dtype=torch.float64)
    f = _Linear(A)
    ys = odeint_adjoint(f, y0, t, rtol=1e-10, atol=1e-12, method="dopri5")
    (ys * c).sum().backward()
    Ar = A.clone().requires_grad_(True)
    y0r = y0.detach().clone().requires_grad_(True)
    yr = torch.stack([y0r @ torch.linalg.matrix_exp(Ar * float(tt)).T for tt in t])
    (yr * c).sum().backward()
    assert normwise_rel(ys.detach(), yr.detach()) < 1e-8
    assert normwise_rel(y0.grad, y0r.grad) < 1e-7
    assert normwise_rel(f.A.grad, Ar.grad) < 1e-7


def test_adjoint_time_gradient_matches_analytic(pkg):
    """dL/dt for L = sum_i c_i . y(t_i), y(t) = expm(A (t - t0)) y0: dL/dt_i = c_i . A y(t_i) for i >= 1
    and dL/dt0 = -sum_{i>=1} c_i . A y(t_i) (torchdiffeq's time_vjps)."""
    from torchdiffeq import odeint_adjoint
    torch.manual_seed(3)
    A = torch.randn(3, 3, dtype=torch.float64) * 0.5
    y0 = torch.randn(4, 3, dtype=torch.float64)
    t = torch.tensor([0.2, 0.7, 1.5], dtype=torch.float64).requires_grad_(True)
    c = torch.randn(3, 4, 3, dtype=torch.float64)
    ys = odeint_adjoint(_Linear(A), y0, t, rtol=1e-11, atol=1e-13, method="dopri5")
    (ys * c).sum().backward()
    with torch.no_grad():
        yt = torch.stack([y0 @ torch.linalg.matrix_exp(A * float(tt - t[0])).T for tt in t])
        dti = torch.stack([(c[i] * (yt[i] @ A.T)).sum() for i in range(3)])
        want = dti.clone()
        want[0] = -dti[1:].sum()
    assert normwise_rel(t.grad, want) < 1e-8, (t.grad, want)


def _uoracle(pkg, kind, R, dtype):
    torch.manual_seed(2)
    if kind == "FaFp":
        m = pkg.FaFp(R, latent_dim=8, net_sizes=[16, 16, 8], aug_net_sizes=[16, 12])
        m.Fa_w = 0.6
    elif kind == "Fp":
        m = pkg.Fp(R, latent_dim=8, net_sizes=[16, 16, 8])
    else:
        m = pkg.Fa(R, latent_dim=8, aug_net_sizes=[16, 12])
    return m.to(dtype)


def _y0(N, R, dtype, seed=4):
    g = torch.Generator().manual_seed(seed)
    S = torch.rand(N, R, generator=g) * 0.4 + 0.5
    I = torch.rand(N, R, generator=g) * 0.05
    return torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, R, 5, generator=g)],
                     -1).to(dtype)


@pytest.mark.parametrize("kind", ["FaFp", "Fp", "Fa"])
def test_adjoint_matches_oracle_restatement_cpu(pkg, kind):
    """Product adjoint (eager RHS on the host) vs the oracle's restatement, fp64."""
    from torchdiffeq import odeint_adjoint
    mod = _uoracle(pkg, kind, 1, torch.float64)
    y0 = _y0(6, 1, torch.float64).requires_grad_(True)
    t = torch.tensor([0.0, 0.5, 1.0, 2.0], dtype=torch.float64)
    c = torch.randn((4,) + tuple(y0.shape), generator=torch.Generator().manual_seed(9), dtype=torch.float64)
    ys = odeint_adjoint(mod, y0, t, rtol=1e-8, atol=1e-10)
    (ys * c).sum().backward()
    rhs = OracleRHS.from_module(mod, torch.float64).requires_grad_()
    with torch.no_grad():
        yr = odeint_dopri5(rhs, y0.detach(), t, rtol=1e-8, atol=1e-10)
    dy0, dps = adjoint_backward(rhs, rhs.weights(), t, yr, c, 1e-8, 1e-10)
    # same algorithm, different fp64 operation orders (matmul vs sum of products in the
    # stage combinations): step sizes agree to rounding
    assert normwise_rel(ys.detach(), yr) < 1e-10
    assert normwise_rel(y0.grad, dy0) < 1e-7
    grads = [p.grad for lin in mod.ude_linears() for p in (lin.weight, lin.bias)]
    for a, b in zip(grads, dps):
        assert normwise_rel(a, b) < 1e-7


def test_adjoint_converges_to_true_gradient(pkg):
    """Adjoint gradients approach the exact gradient (backprop through a fine fixed-step RK4,
    O(h^4)) as the tolerances shrink.  (Backprop through the adaptive solve itself is not the
    reference: it also differentiates the step-size controller.)"""
    from torchdiffeq import odeint, odeint_adjoint
    mod = _uoracle(pkg, "FaFp", 1, torch.float64)
    y0 = _y0(5, 1, torch.float64)
    t = torch.tensor([0.0, 1.0, 2.5], dtype=torch.float64)
    c = torch.randn((3,) + tuple(y0.shape), generator=torch.Generator().manual_seed(1), dtype=torch.float64)
    gt = y0.clone().requires_grad_(True)
    (odeint(mod, gt, t, method="rk4", options=dict(step_size=2.5e-3)) * c).sum().backward()
    errs = []
    for tol in (1e-5, 1e-9):
        ga = y0.clone().requires_grad_(True)
        (odeint_adjoint(mod, ga, t, rtol=tol, atol=tol * 1e-2) * c).sum().backward()
        errs.append(normwise_rel(ga.grad, gt.grad))
    assert errs[1] < 1e-7 and errs[1] < 1e-2 * errs[0], errs


@pytest.mark.gpu
@pytest.mark.parametrize("kind,R", [("FaFp", 1), ("Fp", 1), ("Fa", 1), ("FaFp", 49)])
def test_fused_adjoint_matches_oracle(pkg, kind, R):
    from torchdiffeq import odeint_adjoint
    if R == 49:
        torch.manual_seed(2)
        mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    else:
        mod = _uoracle(pkg, kind, R, torch.float32)
        if kind == "Fp":
            mod = pkg.Fp(1, latent_dim=8, net_sizes=[32, 32])
        elif kind == "Fa":
            mod = pkg.Fa(1, latent_dim=8, aug_net_sizes=[64, 64])
        else:
            mod = pkg.FaFp(1, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    N = 24 if R == 49 else 40
    y0 = _y0(N, R, torch.float32)
    t = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float32)
    c = torch.randn((3,) + tuple(y0.shape), generator=torch.Generator().manual_seed(3))
    rtol, atol = 1e-6, 1e-8
    rhs = OracleRHS.from_module(mod, torch.float64).requires_grad_()
    with torch.no_grad():
        yr = odeint_dopri5(rhs, y0.double(), t, rtol=rtol, atol=atol)
    dy0, dps = adjoint_backward(rhs, rhs.weights(), t, yr, c.double(), rtol, atol)
    # the same adjoint restated in fp32: the bar is max(1e-4, 2 x its distance to fp64)
    r32 = OracleRHS.from_module(mod, torch.float32).requires_grad_()
    with torch.no_grad():
        y32 = odeint_dopri5(r32, y0, t, rtol=rtol, atol=atol)
    d32, p32 = adjoint_backward(r32, r32.weights(), t, y32, c, rtol, atol)
    bar = lambda a, b: max(1e-4, 2.0 * normwise_rel(a, b))
    mg = mod.to("cuda")
    yg = y0.to("cuda").requires_grad_(True)
    ys = odeint_adjoint(mg, yg, t.to("cuda"), rtol=rtol, atol=atol)
    (ys * c.to("cuda")).sum().backward()
    assert mg.last_adjoint_info["fused"], mg.last_adjoint_info     # one eval+VJP launch per evaluation
    assert normwise_rel(ys.detach(), yr) < 1e-5
    assert normwise_rel(yg.grad, dy0) < bar(d32, dy0), normwise_rel(yg.grad, dy0)
    grads = [p.grad for lin in mg.ude_linears() for p in (lin.weight, lin.bias)]
    for i, (a, b) in enumerate(zip(grads, dps)):
        assert normwise_rel(a, b) < bar(p32[i], b), (i, normwise_rel(a, b), bar(p32[i], b))


@pytest.mark.gpu
@pytest.mark.parametrize("norm", [None, "seminorm"])
def test_fused_adjoint_matches_autograd_adjoint(pkg, norm):
    """The fused backward (ude_rhs_eval_vjp per augmented evaluation, ude_lincomb / ude_scaled_sumsq
    controller passes) against the generic one (module call + torch.autograd.grad per evaluation,
    PyTorch controller), selected by handing the parameters in another order: same gradients."""
    from torchdiffeq import odeint_adjoint
    torch.manual_seed(4)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to("cuda")
    y0 = _y0(300, 49, torch.float32).to("cuda")
    t = torch.tensor([0.0, 0.7, 1.5], device="cuda")
    c = torch.randn((3,) + tuple(y0.shape), generator=torch.Generator().manual_seed(5)).to("cuda")
    opts = None if norm is None else dict(norm=norm)
    params = [p for lin in mod.ude_linears() for p in (lin.weight, lin.bias)]
    out = []
    for order in (params, params[::-1]):
        mod.zero_grad(set_to_none=True)
        yg = y0.clone().requires_grad_(True)
        ys = odeint_adjoint(mod, yg, t, rtol=1e-6, atol=1e-8, adjoint_params=order, adjoint_options=opts)
        (ys * c).sum().backward()
        out.append((mod.last_adjoint_info["fused"], yg.grad.clone(), [p.grad.clone() for p in params]))
    assert out[0][0] and not out[1][0]
    assert normwise_rel(out[0][1], out[1][1]) < 1e-5
    for a, b in zip(out[0][2], out[1][2]):
        assert normwise_rel(a, b) < 1e-5


@pytest.mark.gpu
def test_controller_vector_passes_match_torch(pkg):
    """ude_lincomb (out = base + sum_j c_j k_j, one pass; 16-byte and scalar kernels) and
    ude_scaled_sumsq (sum of squared error ratios, fp32 tolerance, fp64 sums) against PyTorch on a
    ragged length."""
    from ude_amd import _native, fused
    lib = _native.prebuilt()
    g = torch.Generator(device="cuda").manual_seed(6)
    n = 1_000_003
    ks = [torch.randn(n, device="cuda", generator=g) for _ in range(7)]
    base = torch.randn(n, device="cuda", generator=g)
    c = torch.randn(7, device="cuda", generator=g)
    out = torch.empty(n, device="cuda")
    st = fused._stream(torch.device("cuda"))
    for nk in (1, 4, 7):
        lib.lincomb(n, base.data_ptr(), [k.data_ptr() for k in ks[:nk]], c.data_ptr(), out.data_ptr(), st)
        ref = base + sum(ks[j] * c[j] for j in range(nk))
        assert torch.allclose(out, ref, rtol=1e-6, atol=1e-6)
        # pointers 4 bytes off 16-byte alignment take the scalar kernel: the same per-element
        # operation order, so bitwise the 16-byte kernel's elements 1..n-1
        out2 = torch.zeros(n, device="cuda")
        lib.lincomb(n - 1, base.data_ptr() + 4, [k.data_ptr() + 4 for k in ks[:nk]], c.data_ptr(),
                    out2.data_ptr() + 4, st)
        torch.cuda.synchronize()
        assert torch.equal(out2[1:], out[1:])
    ssq = torch.empty(_native.SUMSQ_WS, dtype=torch.float64, device="cuda")
    y0, y1 = ks[1], ks[2]
    lib.scaled_sumsq(n, ks[0].data_ptr(), y0.data_ptr(), y1.data_ptr(), 1e-8, 1e-6, ssq.data_ptr(), st)
    r = (ks[0] / (1e-8 + 1e-6 * torch.max(y0.abs(), y1.abs()))).double()
    assert abs(float(ssq[0]) / float((r * r).sum()) - 1) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("seminorm", [False, True])
def test_host_scalar_controller_equals_operator_chain(pkg, seminorm):
    """adaptive.host_scalar_dopri5 (odeint_adjoint's fused backward: controller scalars mirrored on the
    host, ude_lincomb_hc / ude_dopri_ratio) against eager_dopri5 with the fused evaluation and the
    device-scalar operator chain (ude_lincomb with device coefficients, PyTorch ratio and step-size
    update): the same attempts and bitwise the same solution, mixed norm and seminorm."""
    from ude_amd import adaptive
    from ude_amd import adjoint as A
    torch.manual_seed(7)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to("cuda")
    y = _y0(300, 49, torch.float32).to("cuda")
    a = torch.randn(y.shape, generator=torch.Generator().manual_seed(8)).to("cuda")
    params = tuple(p for lin in mod.ude_linears() for p in (lin.weight, lin.bias))
    rtol, atol = 1e-6, 1e-8
    fused = A._FusedAug(mod, y, params, seminorm)
    fused.atol, fused.rtol = atol, rtol
    zero = torch.zeros((), device="cuda")
    state = [zero, y, a] + [torch.zeros_like(p) for p in params]
    flat = A._Flat([x.shape for x in state])
    y0 = flat.flat(state)
    s_pair = torch.tensor([-1.5, -0.7], dtype=torch.float64, device="cuda")

    def norm(v):
        vt, yy, ay, *ap = flat.split(v)
        n = torch.max(torch.stack([vt.abs().reshape(()), A._rms(yy), A._rms(ay)]))
        return n if seminorm else torch.max(n, A._mixed_norm(ap))

    class Vec:
        comb = staticmethod(fused.comb)
        ratio = staticmethod(lambda err, yy, y1: fused.ratio(err, yy, y1, atol, rtol))
    e0 = fused.evals
    r_old = adaptive.eager_dopri5(fused, y0, s_pair, rtol, atol, None, adaptive.MAX_NUM_STEPS, norm=norm, vec=Vec)
    e1 = fused.evals
    r_new = adaptive.host_scalar_dopri5(fused, y0, s_pair, rtol, atol, None, adaptive.MAX_NUM_STEPS, norm, fused)
    e2 = fused.evals
    assert e2 - e1 == e1 - e0 and e1 - e0 > 20
    assert torch.equal(r_new, r_old), float((r_new - r_old).abs().max())


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_fused_adjoint_state49_slice_matches_oracle(pkg):
    """odeint_adjoint on a 1,024-trajectory slice of the state49 batch (R = 49, the
    bench's model with its output layers x 0.1 so no trajectory crosses the mask boundary, as
    tests/test_full_size.py's whole-batch adjoint) against the fp64 oracle adjoint
    (oracle/ude_oracle_adjoint.py: torchdiffeq's augmented backward restated) on the same slice -- the
    same batch-shared step control, so the same step sequence up to rounding: latent <= 1e-5, dy0 and
    every weight gradient <= max(1e-4, 2 x the fp32 oracle's own distance)."""
    from torchdiffeq import odeint_adjoint
    torch.manual_seed(0)
    mod = pkg.FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    with torch.no_grad():
        for seq in (mod.net, mod.aug_net):
            seq[-1].weight.mul_(0.1)
            seq[-1].bias.mul_(0.1)
    y0 = _y0(1024, 49, torch.float32, seed=5)
    t = torch.tensor([0.0, 1.0], dtype=torch.float32)
    c = torch.randn((2,) + tuple(y0.shape), generator=torch.Generator().manual_seed(6))
    rtol, atol = 1e-6, 1e-8
    rhs = OracleRHS.from_module(mod, torch.float64).requires_grad_()
    with torch.no_grad():
        yr = odeint_dopri5(rhs, y0.double(), t, rtol=rtol, atol=atol)
    dy0, dps = adjoint_backward(rhs, rhs.weights(), t, yr, c.double(), rtol, atol)
    r32 = OracleRHS.from_module(mod, torch.float32).requires_grad_()
    with torch.no_grad():
        y32 = odeint_dopri5(r32, y0, t, rtol=rtol, atol=atol)
    d32, p32 = adjoint_backward(r32, r32.weights(), t, y32, c, rtol, atol)
    bar = lambda a, b: max(1e-4, 2.0 * normwise_rel(a, b))
    mg = mod.to("cuda")
    yg = y0.to("cuda").requires_grad_(True)
    ys = odeint_adjoint(mg, yg, t.to("cuda"), rtol=rtol, atol=atol)
    (ys * c.to("cuda")).sum().backward()
    info = dict(mg.last_adjoint_info)
    assert info["fused"], info
    e_lat = normwise_rel(ys.detach(), yr)
    e_dy0 = normwise_rel(yg.grad, dy0)
    grads = [p.grad for lin in mg.ude_linears() for p in (lin.weight, lin.bias)]
    e_p = [normwise_rel(a, b) for a, b in zip(grads, dps)]
    print(f"adjoint state49 slice (1024 x R49, {info}): latent {e_lat:.1e}, dy0 {e_dy0:.1e} "
          f"[fp32 oracle {normwise_rel(d32, dy0):.1e}], weights " +
          ", ".join(f"{e:.1e} [{normwise_rel(p, b):.1e}]" for e, p, b in zip(e_p, p32, dps)))
    assert e_lat < 1e-5
    assert e_dy0 < bar(d32, dy0)
    for i, (e, p, b) in enumerate(zip(e_p, p32, dps)):
        assert e < bar(p, b), (i, e, bar(p, b))
