"""A/B (development): the Bayesian R = 1 model's backward as the register dual-dW kernel (default)
vs the GST path (weight gradients per evaluation by ude_gst_dw_kernel, -DUDE_GST_MIN_NDW=0).
`--build` on the host; without it, on the GPU box, times the bayes_us bench step with each."""
import importlib
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native, fused, solvers  # noqa: E402
import bench  # noqa: E402

WL = os.environ.get("AB_WORKLOAD", "bayes_us")
VARIANTS = {"base": [], "gst": ["-DUDE_GST_MIN_NDW=0"]}


def lib_path(v):
    return os.path.join(_native.BUILD, f"libude_rk4_ab_{v}_{WL}.so")


def main():
    w = bench.WORKLOADS[WL]
    kind = "B" + w["kind"][len("Bayes_"):]
    cfg = (kind, w["R"], w["L"], tuple(w["net"]), tuple(w["aug"]))
    if "--build" in sys.argv:
        for v, fl in VARIANTS.items():
            _native.build_library([cfg], lib_path(v), f"ab_{v}_{WL}", jobs=2, extra_flags=fl)
        print("built", list(VARIANTS))
        return
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("AB_N", w["n_traj"]))
    mod, y0, t, dlat = bench.build(pkg, dict(w, n_traj=n), dev, seed=1)
    from ude_amd import distributed as udist
    for v in VARIANTS:
        lib = _native.NativeLib(lib_path(v))
        _native.library_for = lambda c, lib=lib: lib
        solvers._PLAN_CACHE.clear()
        for _ in range(2):
            bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
        torch.cuda.synchronize()
        torch.manual_seed(5)                     # the same eps draws in every variant
        fused.EVENTS = []
        import time
        t0 = time.perf_counter()
        for _ in range(3):
            bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / 3
        ms = {}
        for name, e0, e1 in fused.EVENTS:
            ms.setdefault(name, []).append(e0.elapsed_time(e1))
        fused.EVENTS = None
        grads = [p.grad.detach().clone() for p in mod.parameters()]
        print(f"{v}: step {el * 1e3:.2f} ms, " + ", ".join(f"{k} {sum(x) / len(x):.3f} ms" for k, x in ms.items()),
              flush=True)
        if v == "base":
            ref = grads
        else:
            worst = max(float((a - b).norm() / b.norm()) for a, b in zip(grads, ref) if float(b.norm()) > 0)
            print(f"  max normwise grad difference vs base: {worst:.2e}", flush=True)


if __name__ == "__main__":
    main()
