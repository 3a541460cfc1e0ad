"""Diagnostic: run one bench.py extra line (after a warm-up) so rocprofv3 --kernel-trace --stats
can attribute its time to kernels, e.g.
    rocprofv3 --kernel-trace --stats -d gpurun_out/p -o x -- python3 tools/profile_line.py bayes_state49
"""
import importlib
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

pkg = importlib.import_module(bench.PKG)
dev = torch.device("cuda", 0)
which = sys.argv[1]
w = bench.WORKLOADS["state49"]
fn = {"bayes_state49": lambda: bench.bayes_large_line(pkg, dev, steps=2),
      "dopri5_adjoint_state49": lambda: bench.adjoint_line(pkg, w, dev),
      "train_step_head_state49": lambda: bench.train_head_line(pkg, w, dev, reps=3)}[which]
fn()                                # warm-up (plans, attributes, allocator)
torch.cuda.synchronize()
t0 = time.perf_counter()
print(fn())
torch.cuda.synchronize()
print(f"{which}: {time.perf_counter() - t0:.2f} s")
