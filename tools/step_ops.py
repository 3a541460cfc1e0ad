"""Which host operators launch device work in one bench step (torch.profiler, GPU box).

    python tools/step_ops.py [workload]        # default state49

Prints every device kernel / memcpy of one timed step with the aten operator (and Python frame)
that issued it: the per-step glue the fused path should not have."""
import importlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "state49"
pkg = importlib.import_module(bench.PKG)
from ude_amd import distributed as udist  # noqa: E402

dev = torch.device("cuda", 0)
w = bench.WORKLOADS[wl]
mod, y0, t, dlat = bench.build(pkg, w, dev, seed=1000)
for _ in range(3):
    bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
    torch.cuda.synchronize()
evs = prof.events()
n_dev = 0
for e in evs:
    if e.device_type == torch.autograd.DeviceType.CUDA:
        n_dev += 1
        par = e.cpu_parent
        chain = []
        while par is not None and len(chain) < 4:
            chain.append(par.name)
            par = par.cpu_parent
        print(f"{e.name[:70]:70s} {e.device_time_total:8.1f} us  <- {' <- '.join(chain)}")
print(f"device activities in one step: {n_dev}")
for e in evs:
    if e.name in ("aten::copy_", "aten::fill_", "aten::cat", "aten::clone", "aten::zero_") and e.device_time_total > 0:
        print(e.name, [s for s in e.stack if "torch/" not in s][:4])
