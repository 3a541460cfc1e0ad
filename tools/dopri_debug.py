"""Debug: fused dopri5 side statistics vs the fp32 oracle, one step at a time (GPU)."""
import sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import torch, importlib
pkg = importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from oracle.ude_oracle import OracleRHS
from oracle.ude_oracle_dopri5 import Dopri5Stats, odeint_dopri5
from helpers import normwise_rel
from test_dopri5 import _module, _y0
mod = _module(pkg, "FaFp", 1, [64, 64, 32], [64, 64]); mod.Fa_w = 0.8
y0 = _y0(16, 1)
mg = None
for tend in (0.05, 0.55, 0.3):
    t = torch.tensor([0.0, tend])
    r32 = OracleRHS.from_module(mod, torch.float32); s32 = Dopri5Stats()
    ref = odeint_dopri5(r32, y0, t, rtol=1e-5, atol=1e-7, stats=s32, first_step=0.05)
    import copy
    mg = copy.deepcopy(mod).cuda() if mg is None else mg
    mg.clear_tracking()
    with torch.no_grad():
        lat = pkg.odeint(mg, y0.cuda(), t.cuda(), rtol=1e-5, atol=1e-7, method="dopri5", options=dict(first_step=0.05))
    p = torch.stack(r32.params).double()          # (E, N, R, 2)
    post = mg.posterior()
    print(tend, mg.last_solve_info, s32.n_evals, "lat err", normwise_rel(lat, ref))
    print("  kernel mean", post.loc.tolist(), "oracle", p.reshape(-1, 2).mean(0).tolist())
    per = p[..., 0].mean(dim=(1, 2))
    print("  oracle per-eval beta", [round(float(v), 6) for v in per])
    # which single eval, if duplicated in place of another, explains the kernel sum?
    E = p.shape[0]; tot = float(post.loc[0]) * E
    print("  kernel*E - oracle sum", tot - float(per.sum()))
# arbitrate with the eager product path on the GPU (tracks per evaluation like the reference)
from ude_amd.adaptive import eager_dopri5
import copy
me = copy.deepcopy(mod).cuda()
for tend in (0.05, 0.3):
    t = torch.tensor([0.0, tend])
    me.clear_tracking()
    with torch.no_grad():
        out = eager_dopri5(me, y0.cuda(), t.cuda(), rtol=1e-5, atol=1e-7, first_step=0.05)
    p = torch.stack(me.params).double()
    print("eager", tend, "evals", p.shape[0], "mean", p.reshape(-1, 2).mean(0).tolist())
    print("  eager per-eval beta", [round(float(v), 6) for v in p[..., 0].mean(dim=(1, 2))])
