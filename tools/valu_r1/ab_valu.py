"""A/B: the R = 1 forward, wave per trajectory on the VALU (tools/valu_r1/valu_fwd.hip)
vs the product's MFMA tiles, M1 Fp [32, 32] (4,096 trajectories x 365 daily RK4 steps)."""
import ctypes, importlib, json, os, sys
import torch
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import fused, solvers
lib = ctypes.CDLL(os.path.join(REPO, "tools", "valu_r1", "_build", "libvalu.so"))
DEV = "cuda"
torch.manual_seed(0)
mod = pkg.Fp(1, latent_dim=8, net_sizes=[32, 32]).to(DEV)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
gen = torch.Generator().manual_seed(11)
S = torch.rand(N, 1, generator=gen) * 0.4 + 0.5
I = torch.rand(N, 1, generator=gen) * 0.05
y0 = (torch.cat([S[..., None], I[..., None], (1 - S - I)[..., None], torch.randn(N, 1, 5, generator=gen)], -1) + 1e-5).to(DEV)
t = torch.arange(366, dtype=torch.float32) / 7.0
lins = mod.ude_linears()
Ws = [l.weight.detach().contiguous() for l in lins]
bs = [l.bias.detach().contiguous() for l in lins]
plan = solvers.plan_for(mod, y0, t, t[1] - t[0])
dts = torch.from_numpy(plan.sched_dev.cpu().numpy()[: 4 * 365].view("float32").copy()).to(DEV)
out = {}


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


lat_v = torch.empty(366, N, 1, 8, device=DEV)
st = torch.empty(N, 4, dtype=torch.float64, device=DEV)
s = torch.cuda.current_stream().cuda_stream
for wpb in (1, 2, 4):
    def run_valu():
        rc = lib.valu_fp32x32_fwd(*[ctypes.c_void_p(x.data_ptr()) for x in (Ws[0], bs[0], Ws[1], bs[1], Ws[2], bs[2], y0)],
                                  ctypes.c_int(N), ctypes.c_int(365), ctypes.c_void_p(dts.data_ptr()),
                                  ctypes.c_void_p(lat_v.data_ptr()), ctypes.c_void_p(st.data_ptr()), ctypes.c_int(wpb),
                                  ctypes.c_void_p(s))
        assert rc == 0
    out[f"valu_fwd_ms_wpb{wpb}"] = timeit(run_valu)


def run_mfma_infer():
    mod.clear_tracking()
    with torch.no_grad():
        return pkg.odeint(mod, y0, t, method="rk4", options=dict(step_size=t[1] - t[0]))


def run_mfma_train():
    mod.clear_tracking()
    yg = y0.clone().requires_grad_(True)
    return pkg.odeint(mod, yg, t, method="rk4", options=dict(step_size=t[1] - t[0]))


out["mfma_fwd_inference_ms"] = timeit(run_mfma_infer)
out["mfma_fwd_training_ms"] = timeit(run_mfma_train)
lat_m = run_mfma_infer()
torch.cuda.synchronize()
rel = float((lat_v[:, :, :, :3].double() - lat_m[..., :3].double()).norm() / lat_m[..., :3].double().norm())
out["latent_rel_diff_valu_vs_mfma"] = rel
out["N"] = N
print(json.dumps(out))
