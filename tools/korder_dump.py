"""Dump the fused kernel's M1 VJP (dy0, every weight gradient) for offline comparison with oracle
variants (development tool; the checks live in tests/test_kernel_order.py)."""
import os, sys, importlib
import numpy as np
import torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
import test_kernel_order as tko
kind = sys.argv[1] if len(sys.argv) > 1 else "Fp"
torch.manual_seed(0)
if kind == "Fp":
    mod = pkg.Fp(1, latent_dim=8, net_sizes=[32, 32])
else:
    mod = pkg.FaFp(1, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64])
y0, gen = tko._y0(4096, 1, 8, 11)
t = torch.arange(366, dtype=torch.float32) / 7.0
dl = torch.randn((366, 4096, 1, 8), generator=gen, dtype=torch.float64)
lat, got = tko._gpu_vjp(pkg, mod, y0, t, dl)
out = {"dy0": got["y0"].numpy()}
for k, v in got.items():
    if k != "y0":
        out[f"{k[0]}{k[1]}"] = v.numpy()
os.makedirs(os.path.join(REPO, "gpurun_out", "dump"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "dump", f"m1_{kind}.npz"), **out)
print("saved", kind)
