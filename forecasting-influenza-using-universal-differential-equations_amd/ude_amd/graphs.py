"""One training step of the fused solve replayed as a HIP graph.

At small batches (the reference's own N = 2,048 state batch, the 2,560-trajectory per-GPU shard of
8-way strong scaling) the fused step's kernels take ~0.6 ms, and the Python around them -- odeint's
plan lookup, the autograd Functions, the ctypes launches, posterior() / the tracker norm, the
autograd engine -- takes as long: the step is host-bound.  ``GraphedStep`` captures the whole
steady-state step once (``torch.cuda.graph``; our C-ABI launches on the current stream, so they are
captured like any torch kernel) and replays it with one host call.

What is captured: whatever ``fn`` launches -- for a training step, the weight pack (a captured step
packs on every replay: the parameters may change in place between replays), the fused forward with
its in-launch statistics finalize, the backward and its tail, and the parameter-gradient
accumulation.  The same kernels run on the same buffers in the same order, so the results are
bitwise those of the eager step (tests/test_graphs.py).  As with any CUDA / HIP graph, every tensor
``fn`` reads must be static (update inputs in place), the shapes must not change, and ``fn`` must
not synchronise with the host; gradients are (re)written, not accumulated, by each replay when
``fn`` starts by setting the gradients to None (``zero_grad(set_to_none=True)`` inside ``fn``).
Nothing may keep an earlier step's autograd graph alive into the capture -- return detached outputs,
and let ``fn`` clear the module's tracking first (``clear_tracking()``): a live graph keeps the
parameters' AccumulateGrad nodes of the stream it ran on, and the capture then waits on that stream.  The reference's training step (lib/VAE.py:200-223) is one such step per batch;
data-parallel steps (RCCL all-reduces from autograd hooks) are not captured here.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch


class GraphedStep:
    """``GraphedStep(fn)``: runs ``fn`` ``warmup`` times on a side stream (allocator, plans, kernel
    attributes), then captures one call into a HIP graph; ``replay()`` (or calling the object) runs it.
    ``outputs`` holds ``fn``'s return value from the capture (static tensors, rewritten by every replay)."""

    def __init__(self, fn: Callable[[], Optional[object]], warmup: int = 3, pool=None):
        self.fn = fn
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(warmup, 1)):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        # thread-local capture: host-side HIP calls of other threads (none of ours sync) are not
        # errors; our launches go to the capturing stream
        with torch.cuda.graph(self.graph, pool=pool, capture_error_mode="thread_local"):
            self.outputs = fn()

    def replay(self):
        self.graph.replay()
        return self.outputs

    __call__ = replay
