"""A/B (development): one bench workload's step with the library built under different compile
flags.  `--build` on the host builds every variant; without it, on the GPU box, times the bench
step with each (interleaved rounds, so drift hits every variant alike) and prints the kernel
times and each variant's largest normwise gradient difference from the first.

  AB_WORKLOAD=us_fp32 AB_VARIANTS="a:;b:-DUDE_ABL=14" python tools/ab_flags.py [--build]
"""
import importlib
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native, fused, solvers  # noqa: E402
import bench  # noqa: E402

WL = os.environ.get("AB_WORKLOAD", "us_fp32")
VARIANTS = {}
for item in os.environ.get("AB_VARIANTS", "a:;b:-DUDE_ABL=14").split(";"):
    name, _, flags = item.partition(":")
    VARIANTS[name] = flags.split()


def lib_path(v):
    return os.path.join(_native.BUILD, f"libude_rk4_ab_{v}_{WL}.so")


def cfg_of(w):
    kind = "B" + w["kind"][len("Bayes_"):] if w["kind"].startswith("Bayes_") else w["kind"]
    return (kind, w["R"], w["L"], tuple(w["net"]) if w["net"] else None, tuple(w["aug"]) if w["aug"] else None)


def main():
    w = bench.WORKLOADS[WL]
    if "--build" in sys.argv:
        for v, fl in VARIANTS.items():
            _native.build_library([cfg_of(w)], lib_path(v), f"ab_{v}_{WL}", jobs=2, extra_flags=fl)
        print("built", list(VARIANTS))
        return
    dev = torch.device("cuda", 0)
    n = int(os.environ.get("AB_N", w["n_traj"]))
    mod, y0, t, dlat = bench.build(pkg, dict(w, n_traj=n), dev, seed=1)
    from ude_amd import distributed as udist
    libs = {v: _native.NativeLib(lib_path(v)) for v in VARIANTS}
    steps, rounds = int(os.environ.get("AB_STEPS", 10)), int(os.environ.get("AB_ROUNDS", 3))
    res = {v: {"step": [], "fwd": [], "bwd": []} for v in VARIANTS}
    grads = {}
    for _ in range(rounds):
        for v, lib in libs.items():
            _native.library_for = lambda c, lib=lib: lib
            solvers._PLAN_CACHE.clear()
            for _ in range(2):
                bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
            torch.cuda.synchronize()
            fused.EVENTS = []
            t0 = time.perf_counter()
            for _ in range(steps):
                bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
            torch.cuda.synchronize()
            res[v]["step"].append((time.perf_counter() - t0) / steps * 1e3)
            for name, e0, e1 in fused.EVENTS:
                res[v].setdefault(name, []).append(e0.elapsed_time(e1))
            fused.EVENTS = None
            grads[v] = [p.grad.detach().clone() for p in mod.parameters()] + [y0.grad.detach().clone()]
    first = next(iter(VARIANTS))
    for v, r in res.items():
        line = f"{WL} {v}: " + ", ".join(f"{k} {min(x) if k == 'step' else sum(x) / len(x):.3f} ms"
                                        for k, x in r.items() if x)
        if v != first:
            worst = max(float((a - b).norm() / b.norm()) for a, b in zip(grads[v], grads[first]) if float(b.norm()) > 0)
            line += f"; max normwise grad difference vs {first}: {worst:.2e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
