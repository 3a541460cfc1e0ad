"""Which part of the fused step captures into a HIP graph (development probe)."""
import os, sys, faulthandler, importlib
faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
mode = sys.argv[1]
emode = sys.argv[2] if len(sys.argv) > 2 else "thread_local"
DEV = "cuda"
torch.manual_seed(0)
R, N = 49, 2048
mod = pkg.FaFp(R, latent_dim=8, net_sizes=[64, 64, 32], aug_net_sizes=[64, 64]).to(DEV)
y0 = (torch.rand(N, R, 8) * 0.3 + 0.1).to(DEV).requires_grad_(mode != "fwd_nograd")
t = torch.arange(9, dtype=torch.float32)
dl = torch.randn(9, N, R, 8, device=DEV)
x = torch.randn(1000, device=DEV)

def f_torch():
    return (x * 2).sum()

def f_fwd():
    mod.clear_tracking()
    with torch.no_grad():
        return pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=1.0))

def f_step():
    mod.zero_grad(set_to_none=True)
    y0.grad = None
    mod.clear_tracking()
    lat = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=1.0))
    if mode == "fwd_grad":
        return lat
    lat.backward(dl)
    return lat

cm, cs, cn = (torch.tensor([0.3, -0.2], device=DEV), torch.tensor([0.5, 0.1], device=DEV),
              torch.tensor(0.1, device=DEV))


def f_stats():
    mod.zero_grad(set_to_none=True)
    y0.grad = None
    mod.clear_tracking()
    lat = pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=1.0))
    post = mod.posterior()
    if mode == "post":
        torch.autograd.backward([lat, post.loc, post.scale], [dl, cm, cs])
        return lat
    nrm = torch.norm(torch.stack(mod.tracker))
    if mode == "norm":
        torch.autograd.backward([lat, nrm], [dl, cn])
        return lat
    torch.autograd.backward([lat, post.loc, post.scale, nrm], [dl, cm, cs, cn])
    return lat


fn = {"torch": f_torch, "fwd_nograd": f_fwd, "fwd_grad": f_step, "step": f_step, "post": f_stats,
      "norm": f_stats, "stats": f_stats}[mode]
if "eagerfirst" in sys.argv:
    fn()
    torch.cuda.synchronize()
    print("eager first done", flush=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        fn()
torch.cuda.current_stream().wait_stream(side)
torch.cuda.synchronize()
print("warm", flush=True)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode=emode):
    out = fn()
print("captured", flush=True)
g.replay()
torch.cuda.synchronize()
print("replayed OK", mode, emode, flush=True)
