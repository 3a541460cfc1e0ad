"""Loader and builder for the gfx950 C-ABI library (include/ude_rk4.h).

The library is built in-tree with hipcc (``build_prebuilt``), one object per
model configuration of ``configs.PREBUILT`` compiled in parallel and linked
into ``_build/libude_rk4.so``.  A configuration that is not prebuilt is
compiled on first use into ``_build/jit/libude_rk4_<key>.so`` (same C-ABI,
one registry entry).  There is no fallback: if no library for a model can be
loaded, the fused solver raises.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import re
import shutil
import subprocess
import threading
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence

from . import configs as _cfgs

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
INCLUDE = os.path.join(REPO_DIR, "include")
BUILD = os.path.join(PKG_DIR, "_build")
PREBUILT_LIB = os.path.join(BUILD, "libude_rk4.so")
JIT_DIR = os.path.join(BUILD, "jit")
ARCH = os.environ.get("UDE_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", shutil.which("hipcc") or "/opt/rocm/bin/hipcc")
HIP_FLAGS = ["-O3", "-std=c++20", "-fPIC", "-ffp-contract=off", f"--offload-arch={ARCH}"]

UDE_OK, UDE_E_UNSUPPORTED, UDE_E_INVALID, UDE_E_HIP, UDE_E_SOLVER = 0, -1, -2, -3, -4
_ERRS = {UDE_E_UNSUPPORTED: "unsupported model configuration", UDE_E_INVALID: "invalid argument",
         UDE_E_HIP: "HIP runtime error", UDE_E_SOLVER: "adaptive solve failed"}

EXPORTED_SYMBOLS = ("ude_supported", "ude_query", "ude_pack_weights", "ude_pack_weights_bayes",
                    "ude_rk4_forward", "ude_rk4_backward", "ude_rk4_backward_sir", "ude_dopri5_workspace",
                    "ude_dopri5_forward", "ude_loss_head_workspace", "ude_loss_head_forward",
                    "ude_loss_head_backward", "ude_loss_head_backward_sir", "ude_rhs_workspace",
                    "ude_rhs_forward", "ude_rhs_vjp", "ude_pack_decoder", "ude_rk4_forward_dec",
                    "ude_decoder_backward", "ude_nll_workspace", "ude_nll_forward", "ude_nll_backward",
                    "ude_rhs_eval_vjp", "ude_lincomb", "ude_scaled_sumsq", "ude_build_info",
                    "ude_rk4_forward_ex", "ude_rk4_forward_dec_ex", "ude_rk4_backward_ex", "ude_lincomb_hc",
                    "ude_dopri_ratio")
SUMSQ_WS = 1025          # doubles of ude_scaled_sumsq's output / workspace (UDE_SUMSQ_WS)


class UdeModelDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("n_regions", ctypes.c_int32), ("latent_dim", ctypes.c_int32),
                ("n_p_hidden", ctypes.c_int32), ("p_hidden", ctypes.c_int32 * 4),
                ("n_a_hidden", ctypes.c_int32), ("a_hidden", ctypes.c_int32 * 4)]


class UdeProblem(ctypes.Structure):
    _fields_ = [("n_traj", ctypes.c_int32), ("n_steps", ctypes.c_int32), ("n_out", ctypes.c_int32),
                ("fa_w", ctypes.c_float), ("recompute", ctypes.c_int32)]


class UdeDopriInfo(ctypes.Structure):
    _fields_ = [("n_steps", ctypes.c_int32), ("n_accepted", ctypes.c_int32), ("n_evals", ctypes.c_int32),
                ("status", ctypes.c_int32)]


class UdeSizes(ctypes.Structure):
    _fields_ = [("pack_bytes", ctypes.c_int64), ("sched_bytes", ctypes.c_int64), ("ckpt_bytes", ctypes.c_int64),
                ("stats_slab_bytes", ctypes.c_int64), ("grad_slab_bytes", ctypes.c_int64),
                ("n_params", ctypes.c_int64), ("grid_fwd", ctypes.c_int32), ("grid_bwd", ctypes.c_int32),
                ("lds_fwd", ctypes.c_int32), ("lds_bwd", ctypes.c_int32),
                ("dec_pack_bytes", ctypes.c_int64), ("ckpt_final_bytes", ctypes.c_int64),
                ("dec_ws_bytes", ctypes.c_int64), ("act_bytes", ctypes.c_int64), ("ctl_bytes", ctypes.c_int64)]


class UdeSideStats(ctypes.Structure):
    """mean (2) / std (2) / fa_norm (1) float buffers and the fp64 totals (5, nullable)."""
    _fields_ = [("mean", ctypes.c_void_p), ("std", ctypes.c_void_p), ("fa_norm", ctypes.c_void_p),
                ("sums", ctypes.c_void_p)]


class UdeSideStatsGrad(ctypes.Structure):
    """Cotangents of mean / std / fa_norm (each nullable: zero)."""
    _fields_ = [("d_mean", ctypes.c_void_p), ("d_std", ctypes.c_void_p), ("d_fa_norm", ctypes.c_void_p)]


def make_desc(cfg: _cfgs.Config) -> UdeModelDesc:
    kind, R, L, net, aug = cfg
    d = UdeModelDesc()
    d.kind = _cfgs.KIND_CODE[kind]
    d.n_regions = R
    d.latent_dim = L
    net = list(net or [])
    aug = list(aug or [])
    d.n_p_hidden = len(net)
    d.n_a_hidden = len(aug)
    for i, v in enumerate(net):
        d.p_hidden[i] = v
    for i, v in enumerate(aug):
        d.a_hidden[i] = v
    return d


class UdeError(RuntimeError):
    pass


class UdeStaleLibrary(UdeError):
    """The prebuilt library does not match the sources in the tree."""


def check(rc: int, what: str) -> None:
    if rc != UDE_OK:
        raise UdeError(f"{what} failed: {_ERRS.get(rc, rc)} (code {rc})")


class NativeLib:
    """ctypes view of one libude_rk4*.so."""

    def __init__(self, path: str):
        self.path = path
        self.lib = ctypes.CDLL(path)
        L = self.lib
        vp, i32 = ctypes.c_void_p, ctypes.c_int
        pdesc, pprob = ctypes.POINTER(UdeModelDesc), ctypes.POINTER(UdeProblem)
        L.ude_supported.argtypes = [pdesc]
        L.ude_supported.restype = i32
        L.ude_query.argtypes = [pdesc, pprob, i32, ctypes.POINTER(UdeSizes)]
        L.ude_query.restype = i32
        L.ude_pack_weights.argtypes = [pdesc, ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]
        L.ude_pack_weights.restype = i32
        pvp = ctypes.POINTER(vp)
        L.ude_pack_weights_bayes.argtypes = [pdesc, pprob, pvp, pvp, pvp, pvp, vp, vp, vp]
        L.ude_pack_weights_bayes.restype = i32
        L.ude_rk4_forward.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_rk4_forward.restype = i32
        L.ude_rk4_backward.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_rk4_backward.restype = i32
        L.ude_rk4_backward_sir.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_rk4_backward_sir.restype = i32
        L.ude_dopri5_workspace.argtypes = [pdesc, pprob, i32, ctypes.POINTER(ctypes.c_int64)]
        L.ude_dopri5_workspace.restype = i32
        dbl = ctypes.c_double
        L.ude_dopri5_forward.argtypes = [pdesc, pprob, vp, vp, dbl, dbl, dbl, ctypes.c_int32, vp, vp, vp, vp,
                                         ctypes.POINTER(UdeDopriInfo), vp]
        L.ude_dopri5_forward.restype = i32
        L.ude_loss_head_workspace.argtypes = [pdesc, i32, i32, i32, i32, ctypes.POINTER(ctypes.c_int64)]
        L.ude_loss_head_workspace.restype = i32
        L.ude_loss_head_forward.argtypes = [pdesc, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp]
        L.ude_loss_head_forward.restype = i32
        L.ude_loss_head_backward.argtypes = [pdesc, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_loss_head_backward.restype = i32
        L.ude_loss_head_backward_sir.argtypes = [pdesc, i32, i32, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_loss_head_backward_sir.restype = i32
        L.ude_rhs_workspace.argtypes = [pdesc, pprob, i32, ctypes.POINTER(ctypes.c_int64)]
        L.ude_rhs_workspace.restype = i32
        L.ude_rhs_forward.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp]
        L.ude_rhs_forward.restype = i32
        L.ude_rhs_vjp.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_rhs_vjp.restype = i32
        L.ude_pack_decoder.argtypes = [pdesc, vp, vp, vp, vp]
        L.ude_pack_decoder.restype = i32
        L.ude_rk4_forward_dec.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_rk4_forward_dec.restype = i32
        L.ude_decoder_backward.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.ude_decoder_backward.restype = i32
        L.ude_nll_workspace.argtypes = [pdesc, i32, i32, i32, ctypes.POINTER(ctypes.c_int64)]
        L.ude_nll_workspace.restype = i32
        L.ude_nll_forward.argtypes = [pdesc, i32, i32, i32, vp, vp, vp, vp, vp]
        L.ude_nll_forward.restype = i32
        L.ude_nll_backward.argtypes = [pdesc, i32, i32, i32, vp, vp, vp, vp, vp, vp]
        L.ude_nll_backward.restype = i32
        L.ude_rhs_eval_vjp.argtypes = [pdesc, pprob, vp, vp, vp, vp, ctypes.c_float, vp, vp, vp, vp]
        L.ude_rhs_eval_vjp.restype = i32
        L.ude_lincomb.argtypes = [ctypes.c_int64, vp, pvp, ctypes.c_int32, vp, vp, vp]
        L.ude_lincomb.restype = i32
        L.ude_scaled_sumsq.argtypes = [ctypes.c_int64, vp, vp, vp, dbl, dbl, vp, vp]
        L.ude_scaled_sumsq.restype = i32
        L.ude_lincomb_hc.argtypes = [ctypes.c_int64, vp, pvp, ctypes.c_int32, ctypes.POINTER(ctypes.c_float), vp, vp]
        L.ude_lincomb_hc.restype = i32
        L.ude_dopri_ratio.argtypes = [vp, vp, vp, dbl, dbl, vp, ctypes.POINTER(ctypes.c_int64), ctypes.c_int32, vp,
                                      ctypes.c_int32, dbl, vp, vp, vp]
        L.ude_dopri_ratio.restype = i32
        L.ude_build_info.argtypes = []
        L.ude_build_info.restype = ctypes.c_char_p
        pst, pdst = ctypes.POINTER(UdeSideStats), ctypes.POINTER(UdeSideStatsGrad)
        L.ude_rk4_forward_ex.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, pst, vp]
        L.ude_rk4_forward_ex.restype = i32
        L.ude_rk4_forward_dec_ex.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, vp, vp, vp, pst, vp, vp]
        L.ude_rk4_forward_dec_ex.restype = i32
        L.ude_rk4_backward_ex.argtypes = [pdesc, pprob, vp, vp, vp, vp, vp, vp, pst, pdst, vp, vp, vp, vp, vp]
        L.ude_rk4_backward_ex.restype = i32

    def supported(self, desc: UdeModelDesc) -> bool:
        return bool(self.lib.ude_supported(ctypes.byref(desc)))

    def query(self, desc, prob, device: int) -> UdeSizes:
        out = UdeSizes()
        check(self.lib.ude_query(ctypes.byref(desc), ctypes.byref(prob), int(device), ctypes.byref(out)), "ude_query")
        return out

    def pack(self, desc, w_ptrs: Sequence[int], b_ptrs: Sequence[int], pack_ptr: int, stream: int) -> None:
        n = len(w_ptrs)
        W = (ctypes.c_void_p * n)(*w_ptrs)
        B = (ctypes.c_void_p * n)(*b_ptrs)
        check(self.lib.ude_pack_weights(ctypes.byref(desc), W, B, pack_ptr, stream), "ude_pack_weights")

    def pack_bayes(self, desc, prob, w_mean: Sequence[int], b_mean: Sequence[int], w_std: Sequence[int],
                   b_std: Sequence[int], eps_ptr: int, pack_ptr: int, stream: int) -> None:
        n = len(w_mean)
        arr = lambda ptrs: (ctypes.c_void_p * n)(*ptrs)
        check(self.lib.ude_pack_weights_bayes(ctypes.byref(desc), ctypes.byref(prob), arr(w_mean), arr(b_mean),
                                              arr(w_std), arr(b_std), eps_ptr, pack_ptr, stream),
              "ude_pack_weights_bayes")

    def forward(self, desc, prob, pack, sched, y0, latent, ckpt, stats_slab, stats_out, stream) -> None:
        check(self.lib.ude_rk4_forward(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, latent, ckpt,
                                       stats_slab, stats_out, stream), "ude_rk4_forward")

    def backward(self, desc, prob, pack, sched, y0, ckpt, dlatent, stats_out, dstats, dy0, slab, dparams,
                 stream) -> None:
        check(self.lib.ude_rk4_backward(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, ckpt, dlatent,
                                        stats_out, dstats, dy0, slab, dparams, stream), "ude_rk4_backward")

    def backward_sir(self, desc, prob, pack, sched, y0, ckpt, dlatent, dlat_sir, stats_out, dstats, dy0, slab,
                     dparams, stream) -> None:
        check(self.lib.ude_rk4_backward_sir(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, ckpt, dlatent,
                                            dlat_sir, stats_out, dstats, dy0, slab, dparams, stream),
              "ude_rk4_backward_sir")

    def forward_ex(self, desc, prob, pack, sched, y0, latent, ckpt, stats_slab, ctl, stats: UdeSideStats,
                   stream) -> None:
        check(self.lib.ude_rk4_forward_ex(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, latent, ckpt,
                                          stats_slab, ctl, ctypes.byref(stats), stream), "ude_rk4_forward_ex")

    def forward_dec_ex(self, desc, prob, pack, sched, y0, dec_pack, yhat, ckpt, stats_slab, reg_slab, ctl,
                       stats: UdeSideStats, reg_out, stream) -> None:
        check(self.lib.ude_rk4_forward_dec_ex(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, dec_pack,
                                              yhat, ckpt, stats_slab, reg_slab, ctl, ctypes.byref(stats), reg_out,
                                              stream), "ude_rk4_forward_dec_ex")

    def backward_ex(self, desc, prob, pack, sched, y0, ckpt, dlatent, dlat_sir, stats: UdeSideStats,
                    dstats: UdeSideStatsGrad, dy0, slab, ctl, dparams, stream) -> None:
        check(self.lib.ude_rk4_backward_ex(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, ckpt, dlatent,
                                           dlat_sir, ctypes.byref(stats), ctypes.byref(dstats), dy0, slab, ctl,
                                           dparams, stream), "ude_rk4_backward_ex")

    def dopri5_workspace(self, desc, prob, device: int) -> int:
        out = ctypes.c_int64(0)
        check(self.lib.ude_dopri5_workspace(ctypes.byref(desc), ctypes.byref(prob), int(device), ctypes.byref(out)),
              "ude_dopri5_workspace")
        return int(out.value)

    def dopri5_forward(self, desc, prob, pack, t_out, rtol, atol, first_step, max_steps, y0, latent, ws,
                       stats_out, stream) -> UdeDopriInfo:
        info = UdeDopriInfo()
        rc = self.lib.ude_dopri5_forward(ctypes.byref(desc), ctypes.byref(prob), pack, t_out, float(rtol),
                                         float(atol), float(first_step), int(max_steps), y0, latent, ws, stats_out,
                                         ctypes.byref(info), stream)
        if rc == UDE_E_SOLVER:
            why = {1: "underflow in dt", 2: "max_num_steps exceeded", 3: "non-finite values in state `y`"}
            raise AssertionError(f"dopri5: {why.get(info.status, info.status)} "
                                 f"(after {info.n_steps} steps, {info.n_evals} evaluations)")
        check(rc, "ude_dopri5_forward")
        return info

    def loss_workspace(self, desc, T, S, B, device) -> int:
        out = ctypes.c_int64(0)
        check(self.lib.ude_loss_head_workspace(ctypes.byref(desc), int(T), int(S), int(B), int(device),
                                               ctypes.byref(out)), "ude_loss_head_workspace")
        return int(out.value)

    def loss_forward(self, desc, T, S, B, latent, W, b, y, ws, out, stream) -> None:
        check(self.lib.ude_loss_head_forward(ctypes.byref(desc), int(T), int(S), int(B), latent, W, b, y, ws, out,
                                             stream), "ude_loss_head_forward")

    def loss_backward(self, desc, T, S, B, latent, W, b, y, grad, ws, dlat, dW, db, stream) -> None:
        check(self.lib.ude_loss_head_backward(ctypes.byref(desc), int(T), int(S), int(B), latent, W, b, y, grad,
                                              ws, dlat, dW, db, stream), "ude_loss_head_backward")

    def loss_backward_sir(self, desc, T, S, B, latent, W, b, y, grad, ws, dlat_sir, dW, db, stream) -> None:
        check(self.lib.ude_loss_head_backward_sir(ctypes.byref(desc), int(T), int(S), int(B), latent, W, b, y, grad,
                                                  ws, dlat_sir, dW, db, stream), "ude_loss_head_backward_sir")

    def rhs_workspace(self, desc, prob, device: int) -> int:
        out = ctypes.c_int64(0)
        check(self.lib.ude_rhs_workspace(ctypes.byref(desc), ctypes.byref(prob), int(device), ctypes.byref(out)),
              "ude_rhs_workspace")
        return int(out.value)

    def rhs_forward(self, desc, prob, pack, x, f, rates, fa, stream) -> None:
        check(self.lib.ude_rhs_forward(ctypes.byref(desc), ctypes.byref(prob), pack, x, f, rates, fa, stream),
              "ude_rhs_forward")

    def rhs_vjp(self, desc, prob, pack, x, cot_f, cot_rates, cot_fa, dx, ws, dparams, stream) -> None:
        check(self.lib.ude_rhs_vjp(ctypes.byref(desc), ctypes.byref(prob), pack, x, cot_f, cot_rates, cot_fa, dx,
                                   ws, dparams, stream), "ude_rhs_vjp")

    def rhs_eval_vjp(self, desc, prob, pack, x, cot_f, f_out, f_scale, dx, ws, dparams, stream) -> None:
        check(self.lib.ude_rhs_eval_vjp(ctypes.byref(desc), ctypes.byref(prob), pack, x, cot_f, f_out,
                                        float(f_scale), dx, ws, dparams, stream), "ude_rhs_eval_vjp")

    def lincomb(self, n, base, ks: Sequence[int], coef, out, stream) -> None:
        arr = (ctypes.c_void_p * len(ks))(*ks)
        check(self.lib.ude_lincomb(int(n), base, arr, len(ks), coef, out, stream), "ude_lincomb")

    def lincomb_hc(self, n, base, ks: Sequence[int], coef: Sequence[float], out, stream) -> None:
        """ude_lincomb with host coefficients (fp32 values, copied into the launch)."""
        arr = (ctypes.c_void_p * len(ks))(*ks)
        cv = (ctypes.c_float * len(coef))(*coef)
        check(self.lib.ude_lincomb_hc(int(n), base, arr, len(ks), cv, out, stream), "ude_lincomb_hc")

    def dopri_ratio(self, err, y0, y1, atol, rtol, ssq, ns: Sequence[int], extra, n_extra, dt, flag, status,
                    stream) -> None:
        na = (ctypes.c_int64 * max(len(ns), 1))(*ns)
        check(self.lib.ude_dopri_ratio(err, y0, y1, float(atol), float(rtol), ssq, na, len(ns), extra, int(n_extra),
                                       float(dt), flag, status, stream), "ude_dopri_ratio")

    def scaled_sumsq(self, n, err, y0, y1, atol, rtol, out, stream) -> None:
        check(self.lib.ude_scaled_sumsq(int(n), err, y0, y1, float(atol), float(rtol), out, stream),
              "ude_scaled_sumsq")

    def pack_decoder(self, desc, W, b, out, stream) -> None:
        check(self.lib.ude_pack_decoder(ctypes.byref(desc), W, b, out, stream), "ude_pack_decoder")

    def forward_dec(self, desc, prob, pack, sched, y0, dec_pack, yhat, ckpt, stats_slab, reg_slab, stats_out,
                    reg_out, stream) -> None:
        check(self.lib.ude_rk4_forward_dec(ctypes.byref(desc), ctypes.byref(prob), pack, sched, y0, dec_pack, yhat,
                                           ckpt, stats_slab, reg_slab, stats_out, reg_out, stream),
              "ude_rk4_forward_dec")

    def decoder_backward(self, desc, prob, sched, ckpt, dyhat, W, grad_reg, ws, dl3, dW, db, stream) -> None:
        check(self.lib.ude_decoder_backward(ctypes.byref(desc), ctypes.byref(prob), sched, ckpt, dyhat, W, grad_reg,
                                            ws, dl3, dW, db, stream), "ude_decoder_backward")

    def nll_workspace(self, desc, T, S, B) -> int:
        out = ctypes.c_int64(0)
        check(self.lib.ude_nll_workspace(ctypes.byref(desc), int(T), int(S), int(B), ctypes.byref(out)),
              "ude_nll_workspace")
        return int(out.value)

    def nll_forward(self, desc, T, S, B, yhat, y, ws, out, stream) -> None:
        check(self.lib.ude_nll_forward(ctypes.byref(desc), int(T), int(S), int(B), yhat, y, ws, out, stream),
              "ude_nll_forward")

    def nll_backward(self, desc, T, S, B, yhat, y, grad, ws, dyhat, stream) -> None:
        check(self.lib.ude_nll_backward(ctypes.byref(desc), int(T), int(S), int(B), yhat, y, grad, ws, dyhat,
                                        stream), "ude_nll_backward")

    def build_info(self) -> str:
        return self.lib.ude_build_info().decode()


# ---------------------------------------------------------------------------
# building
# ---------------------------------------------------------------------------

def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise UdeError("build command failed:\n" + " ".join(cmd) + "\n" + r.stdout[-8000:])


_SRC_HASH: Optional[str] = None


def source_hash(fresh: bool = False) -> str:
    """sha1 (16 hex digits) of every source the library is compiled from (csrc/*.h, csrc/*.hip,
    include/ude_rk4.h) and of the compile flags.  Embedded in ``ude_build_info`` so a prebuilt
    library that no longer matches the tree is refused at load (``prebuilt``).  Computed once per
    process (the tree the process started from); ``fresh`` re-reads the sources (the builder)."""
    global _SRC_HASH
    if _SRC_HASH is not None and not fresh:
        return _SRC_HASH
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".h", ".hip")))
    srcs.append(os.path.join(INCLUDE, "ude_rk4.h"))
    h = hashlib.sha1()
    for f in srcs:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(HIP_FLAGS).encode())
    _SRC_HASH = h.hexdigest()[:16]
    return _SRC_HASH


_INFO_HASH = re.compile(r"\bsrc=([0-9a-f]+)")
_INFO_EXTRA = re.compile(r"\bextra_flags=\[(.*)\]")


def _c_string(s: str) -> str:
    return s.replace("\\", "\\\\").replace('"', '\\"')


def build_library(cfgs: Sequence[_cfgs.Config], out_path: str, tag: str, jobs: Optional[int] = None,
                  extra_flags: Sequence[str] = ()) -> str:
    """Compile one object per configuration + the C-ABI, link into out_path."""
    if not os.path.exists(HIPCC):
        raise UdeError(f"hipcc not found ({HIPCC}); cannot build the gfx950 library")
    gen = os.path.join(BUILD, "gen_" + tag)
    os.makedirs(gen, exist_ok=True)
    reg = ["// generated by ude_amd/_native.py -- do not edit", "namespace ude {"]
    reg += [f"extern const Entry ude_entry_{i};" for i in range(len(cfgs))]
    reg.append("const Entry* const kEntries[] = {" + ", ".join(f"&ude_entry_{i}" for i in range(len(cfgs))) + "};")
    reg.append(f"constexpr int kNumEntries = {len(cfgs)};")
    reg.append("}  // namespace ude")
    reg.append(f'#define UDE_REGISTRY_TAG "{tag}:{len(cfgs)}"')
    reg.append(f'#define UDE_SRC_HASH "{source_hash(fresh=True)}"')
    reg.append(f'#define UDE_EXTRA_FLAGS "{_c_string(" ".join(extra_flags))}"')
    with open(os.path.join(gen, "ude_registry.inc"), "w") as f:
        f.write("\n".join(reg) + "\n")
    inc = ["-I", INCLUDE, "-I", CSRC, "-I", gen, *extra_flags]

    def compile_cfg(i_cfg):
        i, cfg = i_cfg
        obj = os.path.join(gen, f"cfg_{i}.o")
        _run([HIPCC, *HIP_FLAGS, *inc, "-c", os.path.join(CSRC, "ude_cfg.hip"), f"-DUDE_CFG_ID={i}",
              f"-DUDE_ONE_CONFIG={_cfgs.template_args(cfg)}", "-o", obj])
        return obj

    jobs = jobs or min(16, os.cpu_count() or 4)
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_cfg, list(enumerate(cfgs))))
    capi = os.path.join(gen, "ude_rk4.o")
    _run([HIPCC, *HIP_FLAGS, *inc, "-c", os.path.join(CSRC, "ude_rk4.hip"), "-o", capi])
    tmp = out_path + ".tmp"
    _run([HIPCC, *HIP_FLAGS, "-shared", *objs, capi, "-o", tmp])
    os.replace(tmp, out_path)
    return out_path


def build_prebuilt(jobs: Optional[int] = None) -> str:
    os.makedirs(BUILD, exist_ok=True)
    return build_library(_cfgs.PREBUILT, PREBUILT_LIB, "prebuilt", jobs)


# ---------------------------------------------------------------------------
# loading
# ---------------------------------------------------------------------------

_lock = threading.Lock()
_loaded: Dict[str, NativeLib] = {}


def _load(path: str) -> NativeLib:
    with _lock:
        if path not in _loaded:
            _loaded[path] = NativeLib(path)
        return _loaded[path]


def built_hash(lib: NativeLib) -> Optional[str]:
    m = _INFO_HASH.search(lib.build_info())
    return m.group(1) if m else None


_verified: Dict[str, bool] = {}


def prebuilt() -> NativeLib:
    """The in-tree prebuilt library; refused if it was built from other sources than the tree's
    (a stale binary would silently run old kernels) or with extra compile flags (an A/B or
    diagnostic build -- -DUDE_ABL, -DUDE_PROFILE -- placed at the product path).  Checked once per
    process: the library a process has loaded does not change when the sources are edited."""
    if not os.path.exists(PREBUILT_LIB):
        raise UdeError(f"{PREBUILT_LIB} is missing: run __graft_entry__.build() (hipcc, gfx950)")
    lib = _load(PREBUILT_LIB)
    if not _verified.get(PREBUILT_LIB):
        got, want = built_hash(lib), source_hash()
        if got != want:
            raise UdeStaleLibrary(f"{PREBUILT_LIB} is stale (built from sources {got}, tree is {want}): "
                                  "rebuild it with __graft_entry__.build()")
        m = _INFO_EXTRA.search(lib.build_info())
        if m is None or m.group(1).strip():
            raise UdeStaleLibrary(f"{PREBUILT_LIB} was built with extra flags [{m.group(1) if m else '?'}] "
                                  "(a development build): rebuild it with __graft_entry__.build()")
        _verified[PREBUILT_LIB] = True
    return lib


def jit_library(cfg: _cfgs.Config) -> NativeLib:
    key = _cfgs.config_key(cfg)
    h = source_hash()[:10]
    path = os.path.join(JIT_DIR, f"libude_rk4_{key}_{h}.so")
    if not os.path.exists(path):
        os.makedirs(JIT_DIR, exist_ok=True)
        build_library([cfg], path, f"jit_{key}_{h}", jobs=1)
    return _load(path)


def library_for(cfg: _cfgs.Config) -> NativeLib:
    """The library that has a kernel for this configuration (JIT-compiling if needed)."""
    desc = make_desc(cfg)
    if os.path.exists(PREBUILT_LIB):
        lib = prebuilt()
        if lib.supported(desc):
            return lib
    lib = jit_library(cfg)
    if not lib.supported(desc):
        raise UdeError(f"no gfx950 kernel for {cfg}")
    return lib


_SUPPORTED: Dict[_cfgs.Config, bool] = {}


def config_supported(cfg: _cfgs.Config) -> bool:
    """Whether a fused kernel exists (prebuilt, or JIT-compiled here) for cfg.

    Bayesian models keep a second dW accumulator per tile in registers; models
    too large for that are compiled but report unsupported (Model::FITS)."""
    hit = _SUPPORTED.get(cfg)
    if hit is None:
        try:
            library_for(cfg)
            hit = True
        except UdeStaleLibrary:
            raise
        except UdeError:
            hit = False
        _SUPPORTED[cfg] = hit
    return hit


def loaded_paths() -> List[str]:
    return sorted(_loaded)
