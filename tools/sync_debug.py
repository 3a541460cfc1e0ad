import sys, os, warnings
sys.path.insert(0, "/root/repo")
os.chdir("/root/repo")
import torch, bench, importlib
pkg = importlib.import_module(bench.PKG)
from ude_amd import distributed as udist
w = bench.WORKLOADS["state49"]
mod, y0, t, dlat = bench.build(pkg, w, torch.device("cuda", 0), seed=1)
for _ in range(2):
    bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
warnings.simplefilter("always")
bench.one_step(pkg, udist, mod, y0, t, dlat, 1)
torch.cuda.set_sync_debug_mode(0)
print("done")
