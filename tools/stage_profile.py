"""Diagnostic: per-segment cycle breakdown of the backward and training-forward kernels' stage loops.

Builds a -DUDE_PROFILE copy of one configuration (s_memtime stamps at every
barrier of the stage loop, thread 0 of each workgroup), runs the bench workload
through it and prints the average cycles per stage spent in each segment.  The
stamped build is slower than the real one; read the shares, not the totals.
"""
import ctypes
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native  # noqa: E402
import bench  # noqa: E402

SEG = {0: "stage input (ckpt)", 1: "barrier after ckpt", 2: "fwd d0", 3: "fwd d1", 4: "fwd d2", 5: "fwd d3",
       16: "flux bwd", 17: "  output cotangents", 18: "  stage input staging", 6: "  zero padded rows",
       11: "barrier after flux", 10: "bwd d3 (barrier wait)", 9: "bwd d2 (barrier wait)", 8: "bwd d1 (barrier wait)", 7: "bwd d0 (barrier wait)",
       12: "RK adjoint / split-x0 sum", 13: "step end (RK_A)", 14: "step start (cotangents)", 15: "tile start/end",
       27: "  d3 (previous stamp)", 23: "  d3 reads + MFMA + epilogue", 26: "  d2 (previous stamp)",
       22: "  d2 reads + MFMA + epilogue", 25: "  d1 (previous stamp)", 21: "  d1 reads + MFMA + epilogue",
       24: "  d0 (previous stamp)", 20: "  d0 reads + MFMA + epilogue"}
ORDER = [15, 14, 0, 1, 2, 3, 4, 5, 16, 17, 18, 6, 11, 27, 23, 10, 26, 22, 9, 25, 21, 8, 24, 20, 7, 12, 13]
NPROF = 28
FWD_SLOT = 4096                  # csrc PROF_FWD_SLOT: the training forward's rows
FSEG = {15: "tile start/end", 2: "fwd d0 (+ barrier)", 3: "fwd d1 (+ barrier)", 4: "fwd d2 (+ barrier)",
        5: "fwd d3 (+ barrier)", 0: "act rows (tail stores)", 16: "flux pass", 1: "barrier after flux"}
FORDER = [15, 2, 3, 4, 5, 0, 16, 1]
# SPLIT_BWD_L partner wave 4 (bwd_wbody_l, W = 0): rows 2 * FWD_SLOT + block
PSEG = {15: "tile start/end", 13: "stage loop top", 0: "wait for the stage's DMA (vmcnt)", 2: "stage input copy",
        1: "barrier: stage input", 3: "issue ckpt DMA", 16: "barrier: flux pass", 17: "issue final-layer DMA",
        23: "d3 dW (reads, MFMA, bias)", 10: "d3 barrier wait", 27: "d3 DMA issue",
        22: "d2 dW (reads, MFMA, bias)", 9: "d2 barrier wait", 26: "d2 DMA issue",
        21: "d1 dW (reads, MFMA, bias)", 8: "d1 barrier wait", 25: "d1 DMA issue",
        20: "d0 dW (reads, MFMA, bias)", 7: "d0 barrier wait", 24: "d0 DMA issue"}
PORDER = [15, 13, 0, 2, 1, 3, 16, 17, 23, 10, 27, 22, 9, 26, 21, 8, 25, 20, 7, 24]


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "state49"      # [--build]: compile only (on the host)
    # [--partner]: the partner-wave stamps too (a separate library)
    w = bench.WORKLOADS[wl]
    kind = "B" + w["kind"][len("Bayes_"):] if w["kind"].startswith("Bayes_") else w["kind"]
    cfg = (kind, w["R"], w["L"], tuple(w["net"]) if w["net"] else None, tuple(w["aug"]) if w["aug"] else None)
    partner = "--partner" in sys.argv         # also stamp the SPLIT_BWD_L partner wave 4 (perturbs more)
    path = os.path.join(_native.BUILD, f"libude_rk4_profile_{wl}{'_partner' if partner else ''}.so")
    if "--build" in sys.argv or not os.path.exists(path):
        flags = ["-DUDE_PROFILE"] + (["-DUDE_PROFILE_PARTNER"] if partner else [])
        _native.build_library([cfg], path, "profile_" + wl + ("_partner" if partner else ""), jobs=1,
                              extra_flags=flags)
        if "--build" in sys.argv:
            print("built", path)
            return
    lib = _native.NativeLib(path)
    lib.lib.ude_debug_set_prof.argtypes = [ctypes.c_void_p]
    _native.library_for = lambda c: lib
    dev = torch.device("cuda", 0)
    mod, y0, t, dlat = bench.build(pkg, w, dev, seed=1)
    from ude_amd import distributed as udist
    bench.one_step(pkg, udist, mod, y0, t, dlat, 1)        # warm up (grid size known after)
    buf = torch.zeros(3 * FWD_SLOT * NPROF, dtype=torch.int64, device=dev)
    lib.lib.ude_debug_set_prof(buf.data_ptr())
    bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
    torch.cuda.synchronize()
    lib.lib.ude_debug_set_prof(None)
    tiles = (w["n_traj"] + 15) // 16
    for name, rows, seg, order in (("backward", buf[:FWD_SLOT * NPROF], SEG, ORDER),
                                   ("training forward", buf[FWD_SLOT * NPROF:2 * FWD_SLOT * NPROF], FSEG, FORDER),
                                   ("backward partner wave 4", buf[2 * FWD_SLOT * NPROF:], PSEG, PORDER)):
        v = rows.view(-1, NPROF).double()
        used = v[v.sum(1) > 0]
        if used.shape[0] == 0:
            continue
        stages = tiles * 4 * (len(t) - 1) / used.shape[0]
        per = used.mean(0) / stages
        tot = float(per.sum())
        print(f"{name}: workgroups {used.shape[0]}, stages per WG {stages:.1f}, cycles per stage {tot:.0f}")
        for k in order:
            print(f"  {seg[k]:24s} {float(per[k]):9.0f}  {100 * float(per[k]) / tot:5.1f}%")


if __name__ == "__main__":
    main()
