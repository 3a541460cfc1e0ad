"""Diagnostic: timing ablations of the small-record backward (north-star M1 workload).

`--build` (on the host) compiles the M1 configuration once per ablation id with -DUDE_ABL=<id>
(csrc/ude_kernels.h: the id's component is skipped, so results are wrong); without it, on the
GPU box, each library is timed on the bench's M1 backward and the per-variant kernel time printed.
  0 baseline  1 no weight-gradient waves' work  2 no flux pass  3 no input-gradient MFMAs
  4 no stage-input copy  5 no layer-0 sum / RK adjoint  6 no phase-1 weight gradients
  7 no input-gradient phases
  large records (ABL_WORKLOAD=state49): 21 no partner dW MFMAs  22 no activation-row LDS-DMA
  8 no stage-start activation load (4-wave large path)  12 / 11 / 13 forward ablations (no flux pass /
  no activation-row stores / no layer MFMAs)  14 / 15 / 16 forward flux pass: no fp64 side sums / no
  stage-input checkpoint stores / no latent output stores
"""
import importlib
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native, fused, solvers  # noqa: E402
import bench  # noqa: E402

IDS = [int(a) for a in sys.argv[1:] if a.isdigit()] or [0, 1, 2, 3, 4, 5, 6, 7]
# extra flags per variant id >= 100 (id - 100 = UDE_ABL): UDE_DEFER=1
def flags(i):
    return [f"-DUDE_ABL={i % 100}"] + (["-DUDE_DEFER=1"] if i >= 100 else [])
WL = os.environ.get("ABL_WORKLOAD", "us_northstar")


def lib_path(i):
    return os.path.join(_native.BUILD, f"libude_rk4_abl{i}_{WL}.so")


def main():
    w = bench.WORKLOADS[WL]
    cfg = (w["kind"], w["R"], w["L"], tuple(w["net"]) if w["net"] else None, tuple(w["aug"]) if w["aug"] else None)
    if "--build" in sys.argv:
        with ThreadPoolExecutor(8) as ex:
            list(ex.map(lambda i: _native.build_library([cfg], lib_path(i), f"abl{i}_{WL}", jobs=1,
                                                        extra_flags=flags(i)), IDS))
        print("built", IDS)
        return
    dev = torch.device("cuda", 0)
    mod, y0, t, dlat = bench.build(pkg, w, dev, seed=1)
    from ude_amd import distributed as udist
    for i in IDS:
        lib = _native.NativeLib(lib_path(i))
        _native.library_for = lambda c, lib=lib: lib
        solvers._PLAN_CACHE.clear()
        for _ in range(2):
            bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
        torch.cuda.synchronize()
        fused.EVENTS = []
        for _ in range(5):
            bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
        torch.cuda.synchronize()
        ms = {}
        for name, e0, e1 in fused.EVENTS:
            ms.setdefault(name, []).append(e0.elapsed_time(e1))
        fused.EVENTS = None
        print(f"abl {i}: " + ", ".join(f"{k} {sum(v) / len(v):.3f} ms" for k, v in ms.items()), flush=True)


if __name__ == "__main__":
    main()
