"""Host-side logic and the C-ABI boundary (no GPU needed).

* the drop-in modules keep the reference's state_dict keys, initialisation and
  eager semantics (pinned by the golden fixtures);
* the schedule builder reproduces torchdiffeq's grid / output rule;
* odeint's argument checking follows torchdiffeq;
* the C-ABI library loads and exports every symbol include/ude_rk4.h declares,
  and its registry holds every prebuilt configuration.
"""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import REPO, load_golden, rhs_cases, solver_cases
from helpers import module_from_golden, normwise_rel, step_of
from oracle.ude_oracle import make_grid, output_schedule


@pytest.fixture(scope="session")
def native(pkg):
    from ude_amd import _native
    if not os.path.exists(_native.PREBUILT_LIB):
        _native.build_prebuilt()
    return _native


@pytest.mark.parametrize("case", solver_cases())
def test_state_dict_keys_match_reference(pkg, case):
    g = load_golden(case)
    mod = module_from_golden(pkg, g)
    assert list(mod.state_dict().keys()) == g["meta"]["state_dict_keys"]


def test_default_init_draws_reference_weights(pkg):
    # golden case 0 was generated with torch.manual_seed(1000) + reference ctor
    g = load_golden("fafp_r1_weekly")
    torch.manual_seed(1000)
    mod = pkg.FaFp(1, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
    for k, v in mod.state_dict().items():
        assert torch.equal(v, torch.from_numpy(g["w_" + k])), k


@pytest.mark.parametrize("case", rhs_cases())
def test_eager_forward_matches_reference(pkg, case):
    g = load_golden(case)
    m = g["meta"]
    cls = getattr(pkg, m["kind"])
    mod = cls(m["n_regions"], latent_dim=8, net_sizes=m["net_sizes"], aug_net_sizes=m["aug_net_sizes"])
    mod.load_state_dict({k: torch.from_numpy(g["w_" + k]) for k in m["state_dict_keys"]})
    res = mod(0.0, torch.from_numpy(g["x"]).clone())
    assert torch.equal(res, torch.from_numpy(g["res"]))
    if "p" in g:
        assert torch.equal(mod.params[0], torch.from_numpy(g["p"]))
    if "fa" in g:
        assert torch.equal(mod.tracker[0], torch.from_numpy(g["fa"]))


@pytest.mark.parametrize("case", ["fafp_r1_weekly", "fp_r1_daily", "fafp_r1_interp", "fafp_r3_l5_ragged"])
def test_eager_odeint_matches_reference_fp32(pkg, case):
    g = load_golden(case)
    mod = module_from_golden(pkg, g)
    t, h = step_of(g)
    lat = pkg.odeint(mod, torch.from_numpy(g["y0"]), t, method="rk4", options=dict(step_size=h))
    assert normwise_rel(lat, g["ref32_latent"]) < 1e-6


def test_schedule_matches_torchdiffeq_rule(pkg):
    from ude_amd.schedule import build_schedule
    for t, h in [(torch.arange(9, dtype=torch.float32), 1.0),
                 (torch.arange(57, dtype=torch.float32) / 7, None),
                 (torch.linspace(1, 20, 20) / 7, 1.0),
                 (torch.arange(366, dtype=torch.float32) / 7, "t1-t0")]:
        hh = (t[1] - t[0]) if h == "t1-t0" else h
        s = build_schedule(t, hh)
        grid = t if hh is None else make_grid(t, hh)
        assert torch.equal(s.grid, grid)
        ref = output_schedule(t, grid)
        assert [r[0] for r in ref] == list(s.out_j)
        assert [r[2] for r in ref] == list(s.out_mode)
        assert np.allclose([r[3] for r in ref], s.out_slope)
        for n in range(s.n_steps):
            rows = [r for r in ref if r[1] == n]
            assert s.out_start[n + 1] - s.out_start[n] == len(rows)
        assert np.array_equal(s.dt, (grid[1:] - grid[:-1]).numpy())
        b = s.to_bytes()
        assert b.nbytes == 4 * s.n_steps + 4 * (s.n_steps + 1) + 12 * s.n_out


def test_odeint_argument_checks(pkg):
    mod = pkg.FaFp(1)
    y0 = torch.rand(4, 1, 8)
    with pytest.raises(ValueError):
        pkg.odeint(mod, y0, torch.arange(3.0), method="rk5")
    with pytest.raises(AssertionError):
        pkg.odeint(mod, y0, torch.tensor([0.0, 2.0, 1.0]), method="rk4")
    with pytest.raises(NotImplementedError):
        pkg.odeint(mod, y0, torch.arange(3.0), method="bosh3")


def test_cpu_tensors_do_not_take_the_fused_path(pkg):
    mod = pkg.FaFp(1)
    assert not pkg.fusable(mod, torch.rand(4, 1, 8))


def test_posterior_pools_fused_groups(pkg):
    mod = pkg.FaFp(1)
    gen = torch.Generator().manual_seed(3)
    a = torch.rand(100, 2, generator=gen, dtype=torch.float64)
    b = torch.rand(60, 2, generator=gen, dtype=torch.float64) * 2
    mod._fused_rates = [(100.0, a.mean(0), a.std(0)), (60.0, b.mean(0), b.std(0))]
    post = mod.posterior()
    allv = torch.cat([a, b])
    assert torch.allclose(post.loc, allv.mean(0)) and torch.allclose(post.scale, allv.std(0))
    assert mod._fused_rates == []


def _header_symbols():
    src = open(os.path.join(REPO, "include", "ude_rk4.h")).read()
    return sorted(set(re.findall(r"\b(ude_[a-z0-9_]+)\s*\(", src)))


def test_cabi_exports_every_declared_symbol(native):
    lib = ctypes.CDLL(native.PREBUILT_LIB)
    syms = _header_symbols()
    assert set(syms) == set(native.EXPORTED_SYMBOLS)
    for s in syms:
        assert hasattr(lib, s), s


def test_registry_has_every_prebuilt_config(native):
    lib = native.prebuilt()
    for cfg in native._cfgs.PREBUILT:
        assert lib.supported(native.make_desc(cfg)), cfg
    assert not lib.supported(native.make_desc(("FaFp", 7, 8, (13,), (11,))))
    assert "gfx950" in lib.build_info()


def test_host_t_cache_tracks_inplace_updates(pkg):
    """odeint's host copy of t is cached per tensor version: an in-place update is
    seen (here it makes t non-increasing, which must raise like torchdiffeq)."""
    from ude_amd import solvers
    t = torch.arange(6, dtype=torch.float32)
    h1 = solvers._host_t(t)
    assert solvers._host_t(t) is h1            # cached
    t[3] = 0.0
    with pytest.raises(AssertionError):
        solvers._host_t(t)


def test_prebuilt_library_matches_the_tree(native):
    """ude_build_info embeds the hash of the sources the library was compiled from; prebuilt()
    refuses a library whose hash differs from the tree's."""
    lib = native.prebuilt()
    assert native.built_hash(lib) == native.source_hash()


def test_stale_prebuilt_library_is_refused(native, monkeypatch):
    lib = native.prebuilt()
    monkeypatch.setattr(native, "source_hash", lambda *a, **k: "0" * 16)
    monkeypatch.setattr(native, "_verified", {})
    with pytest.raises(native.UdeStaleLibrary):
        native.prebuilt()
    native._SUPPORTED.clear()
    with pytest.raises(native.UdeStaleLibrary):      # not silently reported as "unsupported"
        native.config_supported(native._cfgs.PREBUILT[0])
    native._SUPPORTED.clear()


def test_prebuilt_check_runs_once_per_process(native, monkeypatch):
    """library_for() runs every training step; the source hash is read once per process
    and the loaded library verified once (editing a source mid-run does not fail the next step)."""
    native.prebuilt()
    calls = []
    monkeypatch.setattr(native, "source_hash", lambda *a, **k: calls.append(1) or "0" * 16)
    for _ in range(3):
        native.prebuilt()
    assert calls == []
    assert native.source_hash.__name__ == "<lambda>"


def test_development_build_at_product_path_is_refused(native, monkeypatch):
    """a library built with extra flags (-DUDE_ABL, -DUDE_PROFILE ...) carries the same
    source hash; prebuilt() refuses it by its recorded extra flags."""
    lib = native.prebuilt()
    info = lib.build_info()
    assert "extra_flags=[]" in info
    monkeypatch.setattr(native, "_verified", {})
    monkeypatch.setattr(native.NativeLib, "build_info", lambda self: info.replace("extra_flags=[]",
                                                                                   "extra_flags=[-DUDE_ABL=14]"))
    with pytest.raises(native.UdeStaleLibrary):
        native.prebuilt()
    assert native._c_string('a "b" \\c') == 'a \\"b\\" \\\\c'


def test_pack_key_requires_the_same_tensor_objects():
    """the cached weight pack's key holds weak references to the very parameters it
    was packed from: a parameter object that replaced a freed one at the same address and version
    does not match, an in-place update (version bump) does not match, the same unmodified tensors do."""
    import gc
    import weakref
    from ude_amd.fused import _pack_key_matches
    ps = [torch.nn.Parameter(torch.randn(4, 3)), torch.nn.Parameter(torch.randn(4))]
    key = tuple((weakref.ref(p), p.data_ptr(), p._version) for p in ps)
    assert _pack_key_matches(key, ps)
    with torch.no_grad():
        ps[1].add_(1.0)
    assert not _pack_key_matches(key, ps)
    key = tuple((weakref.ref(p), p.data_ptr(), p._version) for p in ps)
    ptrs = [p.data_ptr() for p in ps]
    del ps
    gc.collect()
    qs = [torch.nn.Parameter(torch.randn(4, 3)), torch.nn.Parameter(torch.randn(4))]
    assert not _pack_key_matches(key, qs), (ptrs, [q.data_ptr() for q in qs])
