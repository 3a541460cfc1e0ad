"""Kernel-order oracle -- TEST INFRASTRUCTURE ONLY (ctypes binding of oracle/ude_korder.c).

Only ``tests/`` load this module, as the checker of the fused gfx950 solve.  The package never
imports it.

``KernelOrderOracle`` restates the reference RHS (lib/models.py:109-265) under torchdiffeq's RK4
(lib/VAE.py:137) in the operation order the kernels claim for their training forward: fp32 fmaf
chains in the MFMA K order, the static-feature hoist, ROCm's expm1f, fp64 RK4 state.  Its forward
(``solve``) is meant to equal the kernel's bit for bit; its backward (``vjp``) is the exact fp64
vector-Jacobian product of that fp32 forward at its own linearisation points (the fp32 stage inputs,
pre-activations, rates and mask decisions), so the kernel's fp32 backward differs from it by the
kernel's own backward rounding only.  ``solve`` / ``vjp`` also return what a test needs to bound
that rounding: every parameter's sum of term magnitudes.

The schedule is rebuilt here from ``ude_oracle.make_grid`` / ``output_schedule`` (torchdiffeq's
``_grid_constructor_from_step_size`` / ``integrate``), independently of the package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Dict, Optional

import numpy as np
import torch

from .ude_oracle import OracleRHS, make_grid, output_schedule

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libude_korder.so")
MAXLIN = 5


class KoModel(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("R", ctypes.c_int32), ("L", ctypes.c_int32), ("fa_w", ctypes.c_float),
                ("nl", ctypes.c_int32 * 2),
                ("in_dim", (ctypes.c_int32 * MAXLIN) * 2), ("out_dim", (ctypes.c_int32 * MAXLIN) * 2),
                ("act", (ctypes.c_int32 * MAXLIN) * 2),
                ("w", (ctypes.c_void_p * MAXLIN) * 2), ("b", (ctypes.c_void_p * MAXLIN) * 2)]


class KoSched(ctypes.Structure):
    _fields_ = [("n_steps", ctypes.c_int32), ("n_out", ctypes.c_int32), ("n_times", ctypes.c_int32),
                ("dt", ctypes.c_void_p), ("out_start", ctypes.c_void_p), ("out_j", ctypes.c_void_p),
                ("out_mode", ctypes.c_void_p), ("out_slope", ctypes.c_void_p)]


_lib = None


def build() -> str:
    """Compile the restatement (oracle/Makefile) if the library is missing or older than its source."""
    src = os.path.join(HERE, "ude_korder.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.ko_solve.restype = ctypes.c_int
        _lib.ko_vjp.restype = ctypes.c_int
        _lib.ko_n_params.restype = ctypes.c_int
        _lib.ko_expm1f.restype = ctypes.c_float
        _lib.ko_expm1f.argtypes = [ctypes.c_float]
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        _lib.ko_solve.argtypes = [vp, vp, i32, vp, vp, vp, vp, i32]
        _lib.ko_vjp.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, i32]
        _lib.ko_vjp32.argtypes = [vp, vp, i32, vp, vp, vp, vp, vp, vp, i32]
        _lib.ko_vjp32.restype = ctypes.c_int
        _lib.ko_n_params.argtypes = [vp]
        _lib.ko_expm1f_array.argtypes = [vp, vp, ctypes.c_long]
        _lib.ko_expm1f_array.restype = None
        _lib.ko_expm1f_compare_bits.argtypes = [ctypes.c_uint32, ctypes.c_long, vp, ctypes.POINTER(ctypes.c_long)]
        _lib.ko_expm1f_compare_bits.restype = ctypes.c_long
        _lib.ko_mfma_elem.argtypes = [vp, vp, vp, vp]
        _lib.ko_set_state32.argtypes = [ctypes.c_int]
        _lib.ko_set_assoc.argtypes = [ctypes.c_int]
        _lib.ko_mfma_elem.restype = None
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data


def schedule(t: torch.Tensor, step_size) -> dict:
    """The fixed-grid schedule (dt per step, output CSR) in the kernel's layout."""
    t = t.detach().cpu()
    grid = make_grid(t, step_size) if step_size is not None else t.clone()
    n_steps = len(grid) - 1
    dt = (grid[1:] - grid[:-1]).to(torch.float32).numpy().astype(np.float32) if n_steps else np.zeros(0, np.float32)
    sched = output_schedule(t, grid)
    starts = np.zeros(n_steps + 1, np.int32)
    for (_j, n, _m, _s) in sched:
        starts[n + 1:] += 1
    return {"dt": np.ascontiguousarray(dt, np.float32), "out_start": starts,
            "out_j": np.asarray([s[0] for s in sched], np.int32),
            "out_mode": np.asarray([s[2] for s in sched], np.int32),
            "out_slope": np.asarray([np.float32(s[3]) for s in sched], np.float32), "n_times": len(t)}


class KernelOrderOracle:
    """The kernel-order restatement for the weights of ``rhs`` (an ``OracleRHS`` in any dtype: the
    weights are taken as fp32, the kernels' dtype)."""

    def __init__(self, rhs: OracleRHS, state32: bool = False):
        """state32: the RK4 state and combinations in fp32 in torchdiffeq's operation order (the
        reference's integrator arithmetic around the kernel's MLP order) instead of the kernel's fp64."""
        self.rhs = rhs
        self.state32 = bool(state32)
        m = KoModel()
        m.kind = {"Fp": 1, "Fa": 2, "FaFp": 3}[rhs.kind]
        m.R, m.L = rhs.n_regions, rhs.latent_dim
        m.fa_w = float(rhs.fa_w)
        self._keep = []
        for net, (ws, bs, acts) in enumerate(((rhs.p_w, rhs.p_b, rhs.p_act), (rhs.a_w, rhs.a_b, rhs.a_act))):
            m.nl[net] = len(ws)
            for i, (w, b, a) in enumerate(zip(ws, bs, acts)):
                wn = np.ascontiguousarray(w.detach().cpu().to(torch.float32).numpy())
                bn = np.ascontiguousarray(b.detach().cpu().to(torch.float32).numpy())
                self._keep += [wn, bn]
                m.in_dim[net][i], m.out_dim[net][i], m.act[net][i] = wn.shape[1], wn.shape[0], int(bool(a))
                m.w[net][i], m.b[net][i] = _p(wn), _p(bn)
        self.model = m
        self.n_params = lib().ko_n_params(ctypes.byref(m))
        names = []
        for i in range(len(rhs.p_w)):
            names += [f"p_w{i}", f"p_b{i}"]
        for i in range(len(rhs.a_w)):
            names += [f"a_w{i}", f"a_b{i}"]
        self.names = names
        self.shapes = [tuple(x.shape) for x in rhs.weights()]

    def _sched(self, t, step_size):
        lib().ko_set_state32(int(self.state32))
        s = schedule(t, step_size)
        ks = KoSched()
        ks.n_steps, ks.n_out, ks.n_times = len(s["dt"]), len(s["out_j"]), s["n_times"]
        for k in ("dt", "out_start", "out_j", "out_mode", "out_slope"):
            setattr(ks, k, _p(s[k]) if s[k].size else None)
        return ks, s

    def solve(self, y0: torch.Tensor, t: torch.Tensor, step_size, stage_inputs: bool = False,
              threads: int = 0) -> Dict[str, torch.Tensor]:
        """latent (T, N, R, L) fp32, the fp64 side sums [sum b, sum g, sum b^2, sum g^2, sum Fa^2],
        the statistics as the kernel finalises them (fp32 mean / std / |Fa|), optionally every stage
        input (E, N, R, 3) fp32 (E = 4 n_steps, evaluation order k1..k4 per step)."""
        ks, s = self._sched(t, step_size)
        yn = np.ascontiguousarray(y0.detach().cpu().to(torch.float32).numpy())
        N, R, L = yn.shape
        lat = np.empty((s["n_times"], N, R, L), np.float32)
        E = 4 * ks.n_steps
        X = np.empty((max(E, 1), N, 3 * R), np.float32) if stage_inputs else None
        sums = np.zeros(5, np.float64)
        lib().ko_solve(ctypes.byref(self.model), ctypes.byref(ks), N, _p(yn), _p(lat),
                       None if X is None else _p(X), _p(sums), int(threads))
        out = {"latent": torch.from_numpy(lat), "sums": torch.from_numpy(sums)}
        n = float(E * N * R)
        mean = sums[0:2] / n
        var = (sums[2:4] - n * mean * mean) / (n - 1.0)
        out["mean"] = torch.from_numpy(mean.astype(np.float32))
        out["std"] = torch.from_numpy(np.sqrt(np.maximum(var, 0.0)).astype(np.float32))
        out["fa_norm"] = torch.from_numpy(np.sqrt(sums[4:5]).astype(np.float32))
        out["n"] = n
        if X is not None:
            out["stage_inputs"] = torch.from_numpy(X[:E]).view(E, N, R, 3)
        return out

    def vjp(self, y0: torch.Tensor, t: torch.Tensor, step_size, dlatent: torch.Tensor,
            dmean=None, dstd=None, dnorm=None, stats: Optional[dict] = None, threads: int = 0,
            fp32: bool = False, n_batch: Optional[int] = None):
        """fp64 VJP of the kernel-order forward: (dy0 (N, R, L) fp64, {name: grad fp64}, {name: sum of
        |terms| fp64}).  Side-statistic cotangents enter as the kernel's bwd_body forms them, from the
        solve's fp32 statistics (``stats``: ``solve``'s output, computed when not given).
        fp32=True: the same VJP executed in fp32 (per-tile fp32 weight-gradient sums, then the tiles) --
        its distance to the fp64 one is the size of fp32 backward rounding on this forward (no
        magnitudes: the third value is None)."""
        ks, s = self._sched(t, step_size)
        yn = np.ascontiguousarray(y0.detach().cpu().to(torch.float32).numpy())
        N, R, L = yn.shape
        if stats is None:
            stats = self.solve(y0, t, step_size, threads=threads)
        # the statistics' count is the whole batch's (n_batch: when y0 is a slice of the batch ``stats``
        # came from)
        n = float(4 * ks.n_steps * (N if n_batch is None else int(n_batch)) * R)
        cot = np.zeros(7, np.float64)
        kind = self.rhs.kind
        if kind != "Fa" and dmean is not None:
            cot[0:2] = np.asarray(torch.as_tensor(dmean).double().cpu().numpy()) / n
        if kind != "Fa" and dstd is not None:
            sd = stats["std"].double().numpy()
            cot[2:4] = np.asarray(torch.as_tensor(dstd).double().cpu().numpy()) / ((n - 1.0) * sd)
        if kind != "Fa":
            cot[4:6] = stats["mean"].double().numpy()
        nrm = float(stats["fa_norm"][0])
        if kind != "Fp" and dnorm is not None and nrm > 0.0:
            cot[6] = float(dnorm) / nrm
        dl = np.ascontiguousarray(torch.as_tensor(dlatent).detach().cpu().double().numpy())
        assert dl.shape == (s["n_times"], N, R, L), dl.shape
        dy0 = np.zeros((N, R, L), np.float64)
        gp = np.zeros(self.n_params, np.float64)
        ga = np.zeros(self.n_params, np.float64)
        fn = lib().ko_vjp32 if fp32 else lib().ko_vjp
        fn(ctypes.byref(self.model), ctypes.byref(ks), N, _p(yn), _p(dl), _p(cot), _p(dy0), _p(gp),
           None if fp32 else _p(ga), int(threads))
        grads, mags, off = {}, {}, 0
        for nm, shp in zip(self.names, self.shapes):
            k = int(np.prod(shp))
            grads[nm] = torch.from_numpy(gp[off:off + k].reshape(shp).copy())
            mags[nm] = torch.from_numpy(ga[off:off + k].reshape(shp).copy())
            off += k
        return torch.from_numpy(dy0), grads, (None if fp32 else mags)


def expm1f(x: np.ndarray) -> np.ndarray:
    """ko_expm1f elementwise (the restated __ocml_expm1_f32)."""
    xs = np.ascontiguousarray(x, np.float32)
    ys = np.empty_like(xs)
    lib().ko_expm1f_array(_p(xs), _p(ys), ctypes.c_long(xs.size))
    return ys
