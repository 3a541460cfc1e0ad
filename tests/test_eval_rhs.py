"""One RHS evaluation + VJP on the gfx950 kernels (csrc/ude_eval.h, ude_amd/eval_rhs.py) against
the reference's forward() restated in fp64 (oracle/ude_oracle.py OracleRHS, pinned to the
reference's own classes by the rhs_* golden fixtures): the returned derivative, the rates and
Fa the forward appends to params / tracker, and autograd's gradients through all three
(w.r.t. the state and every weight), including states on / outside the [-1, 2] mask.

Tolerance: normwise relative 1e-5 (fp32 kernel vs fp64 reference)."""
import pytest
import torch

from conftest import load_golden, rhs_cases
from helpers import normwise_rel
from oracle.ude_oracle import OracleRHS

DEV = "cuda"
CASES = [  # kind, R, L, net, aug
    ("FaFp", 1, 8, [64, 64, 32], [64, 64]), ("Fp", 1, 8, [32, 32], None), ("Fa", 1, 8, None, [64, 64]),
    ("FaFp", 3, 5, [40, 24], [36]), ("FaFp", 10, 8, [64, 64, 32], [64, 64]), ("FaFp", 49, 8, [64, 64, 32], [64, 64]),
    ("Fp", 49, 8, [64, 64, 32], None), ("Fa", 10, 8, None, [64, 64]),
    ("Fa", 49, 8, None, [64, 64]),     # the three R = 49 kinds run the split (8-wave) evaluation + VJP
]


def _module(pkg, kind, R, L, net, aug, fa_w=0.7):
    torch.manual_seed(R * 7 + L)
    if kind == "FaFp":
        m = pkg.FaFp(R, latent_dim=L, net_sizes=net, aug_net_sizes=aug)
        m.Fa_w = fa_w
    elif kind == "Fp":
        m = pkg.Fp(R, latent_dim=L, net_sizes=net)
    else:
        m = pkg.Fa(R, latent_dim=L, aug_net_sizes=aug)
    return m


def _x(N, R, L, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(N, R, L, generator=g) * 1.6 - 0.3
    x[0, 0, 0] = 2.0            # on the mask boundary: not masked
    x[1, 0, 1] = 2.5            # outside: masked
    x[2, -1, 2] = -1.2
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}_R{c[1]}_L{c[2]}")
def test_fused_eval_and_vjp_match_reference(pkg, case):
    kind, R, L, net, aug = case
    mod = _module(pkg, kind, R, L, net, aug)
    N = 45                                           # ragged tile
    x = _x(N, R, L, 100 + R)
    g = torch.Generator().manual_seed(5)
    cf, cr, ca = torch.randn(N, R, L, generator=g), torch.randn(N, R, 2, generator=g), torch.randn(N, R, 3, generator=g)
    # reference (fp64)
    ref = OracleRHS.from_module(mod, torch.float64).requires_grad_()
    xr = x.double().requires_grad_(True)
    f_ref = ref(0.0, xr)
    loss = (f_ref * cf.double()).sum()
    if kind != "Fa":
        loss = loss + (ref.params[0] * cr.double()).sum()
    if kind != "Fp":
        loss = loss + (ref.tracker[0] * ca.double()).sum()
    gr = torch.autograd.grad(loss, [xr] + ref.weights())
    # fused kernel through the module's forward
    mg = mod.to(DEV)
    mg.clear_tracking()
    xg = x.to(DEV).requires_grad_(True)
    f = mg(0.0, xg)
    assert len(mg.params) == (0 if kind == "Fa" else 1) and len(mg.tracker) == (0 if kind == "Fp" else 1)
    loss = (f * cf.to(DEV)).sum()
    if kind != "Fa":
        assert normwise_rel(mg.params[0], ref.params[0]) < 1e-5
        loss = loss + (mg.params[0] * cr.to(DEV)).sum()
    if kind != "Fp":
        assert normwise_rel(mg.tracker[0], ref.tracker[0]) < 1e-5
        loss = loss + (mg.tracker[0] * ca.to(DEV)).sum()
    assert normwise_rel(f, f_ref) < 1e-5
    assert torch.equal(f[..., 3:].cpu(), torch.zeros(N, R, L - 3))
    assert float(f[1, 0, 1]) == 0.0 and float(f[2, -1, 2]) == 0.0
    lins = mg.ude_linears()
    params = [p for lin in lins for p in (lin.weight, lin.bias)]
    gk = torch.autograd.grad(loss, [xg] + params)
    assert normwise_rel(gk[0], gr[0]) < 1e-5, ("dx", normwise_rel(gk[0], gr[0]))
    for i, (a, b) in enumerate(zip(gk[1:], gr[1:])):
        assert normwise_rel(a, b) < 1e-5, (i, normwise_rel(a, b))


@pytest.mark.gpu
@pytest.mark.parametrize("name", rhs_cases())
def test_fused_eval_matches_reference_fixture(pkg, name):
    """The reference's own forward outputs (tests/golden/rhs_*.npz, made by lib/models.py)."""
    d = load_golden(name)
    m = d["meta"]
    mod = _module(pkg, m["kind"], m["n_regions"], m["latent_dim"], m["net_sizes"], m["aug_net_sizes"], fa_w=1.0)
    mod.load_state_dict({k: torch.from_numpy(d["w_" + k]) for k in m["state_dict_keys"]})
    mod = mod.to(DEV)
    mod.clear_tracking()
    res = mod(0.0, torch.from_numpy(d["x"]).to(DEV))
    assert normwise_rel(res, d["res"]) < 1e-5
    if "p" in d:
        assert normwise_rel(mod.params[0], d["p"]) < 1e-5
    if "fa" in d:
        assert normwise_rel(mod.tracker[0], d["fa"]) < 1e-5


@pytest.mark.gpu
def test_bayes_large_r_eval_uses_sampled_weights(pkg):
    """Bayes_FaFp at the state model's size (R = 49; its two dW accumulator sets do not fit the
    fused whole-solve kernel): forward() draws the layer samples exactly as the reference and
    evaluates them on the kernel; gradients reach mean and std through the samples."""
    from ude_amd import bayes
    torch.manual_seed(3)
    mod = bayes.Bayes_FaFp(49, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    x = _x(20, 49, 8, 9)
    torch.manual_seed(11)
    mod.clear_tracking()
    f_ref = mod(0.0, x.clone())                       # eager (CPU): the reference's code path
    loss_ref = (f_ref ** 2).sum() + mod.params[0].sum() + mod.tracker[0].pow(2).sum()
    g_ref = torch.autograd.grad(loss_ref, list(mod.parameters()))
    mg = mod.to(DEV)
    torch.manual_seed(11)
    mg.clear_tracking()
    # the CPU generator drew the reference's samples; on the device the layers draw from the
    # device generator: replay the same draws by seeding make_z's randn_like from CPU draws
    draws = []
    gen = torch.Generator().manual_seed(11)
    for lay in mg._variational():
        draws.append([torch.randn(lay.w_mean.shape, generator=gen), torch.randn(lay.b_mean.shape, generator=gen)])
    it = iter(draws)

    def make_z(self):
        z = next(it)
        self.z = [z[0].to(DEV), z[1].to(DEV)]
    for lay in mg._variational():
        lay.make_z = make_z.__get__(lay)
    f = mg(0.0, x.to(DEV))
    loss = (f ** 2).sum() + mg.params[0].sum() + mg.tracker[0].pow(2).sum()
    g = torch.autograd.grad(loss, list(mg.parameters()))
    assert normwise_rel(f, f_ref) < 1e-5
    for a, b in zip(g, g_ref):
        assert normwise_rel(a, b) < 2e-5
