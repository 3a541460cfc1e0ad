"""Host-side time grid and output schedule of a fixed-step solve.

Follows torchdiffeq's FixedGridODESolver (the integrator the reference calls at
lib/VAE.py:137 -- a third-party dependency, not vendored by the reference):

* grid: ``t`` itself when no step size is given, else
  ``arange(ceil((t[-1]-t[0])/h + 1)) * h + t[0]`` with the last point set to
  ``t[-1]``, all in ``t``'s dtype (``_grid_constructor_from_step_size``);
* step n runs from grid[n] to grid[n+1] with ``dt = grid[n+1] - grid[n]``;
* after step n every not-yet-written output j with ``grid[n+1] >= t[j]`` is
  written: y(t0) if t[j] == t0, y(t1) if t[j] == t1, else the linear
  interpolation with slope ``(t[j]-t0)/(t1-t0)`` (``integrate`` /
  ``_linear_interp``).

The arithmetic is done with torch CPU tensor ops in t's dtype so every
comparison and rounding is the one torchdiffeq would make.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

MODE_T0, MODE_T1, MODE_INTERP = 0, 1, 2


@dataclass
class Schedule:
    grid: torch.Tensor           # (n_steps+1,) in t's dtype, CPU
    dt: np.ndarray               # (n_steps,) float32
    out_start: np.ndarray        # (n_steps+1,) int32 (CSR)
    out_j: np.ndarray            # (n_out,) int32, output indices 1..T-1
    out_mode: np.ndarray         # (n_out,) int32
    out_slope: np.ndarray        # (n_out,) float32
    n_times: int                 # T = len(t)

    @property
    def n_steps(self) -> int:
        return len(self.dt)

    @property
    def n_out(self) -> int:
        return len(self.out_j)

    def to_bytes(self) -> np.ndarray:
        """The packed layout documented in include/ude_rk4.h."""
        parts = [self.dt.astype("<f4").tobytes(), self.out_start.astype("<i4").tobytes(),
                 self.out_j.astype("<i4").tobytes(), self.out_mode.astype("<i4").tobytes(),
                 self.out_slope.astype("<f4").tobytes()]
        buf = b"".join(parts)
        if not buf:
            buf = b"\0\0\0\0"
        return np.frombuffer(buf, dtype=np.uint8).copy()


def fixed_grid(t: torch.Tensor, step_size=None) -> torch.Tensor:
    t = t.detach().cpu()
    if step_size is None:
        return t.clone()
    start, end = t[0], t[-1]
    if isinstance(step_size, torch.Tensor):
        step_size = step_size.detach().cpu().to(t.dtype)
    niters = torch.ceil((end - start) / step_size + 1).item()
    grid = torch.arange(0, niters, dtype=t.dtype) * step_size + start
    grid[-1] = t[-1]
    return grid


def build_schedule(t: torch.Tensor, step_size=None) -> Schedule:
    t = t.detach().cpu()
    grid = fixed_grid(t, step_size)
    if not (grid[0] == t[0] and grid[-1] == t[-1]):
        raise AssertionError("time grid must start at t[0] and end at t[-1]")
    n_steps = len(grid) - 1
    dt = (grid[1:] - grid[:-1]).to(torch.float32).numpy() if n_steps > 0 else np.zeros(0, np.float32)
    starts = [0]
    js: List[int] = []
    modes: List[int] = []
    slopes: List[float] = []
    j = 1
    T = len(t)
    for n in range(n_steps):
        t0, t1 = grid[n], grid[n + 1]
        while j < T and t1 >= t[j]:
            if t[j] == t0:
                modes.append(MODE_T0); slopes.append(0.0)
            elif t[j] == t1:
                modes.append(MODE_T1); slopes.append(1.0)
            else:
                modes.append(MODE_INTERP)
                slopes.append(float(((t[j] - t0) / (t1 - t0)).to(torch.float32)))
            js.append(j)
            j += 1
        starts.append(len(js))
    if j != T:
        raise AssertionError("not every output time is covered by the grid")
    return Schedule(grid=grid, dt=np.asarray(dt, np.float32), out_start=np.asarray(starts, np.int32),
                    out_j=np.asarray(js, np.int32), out_mode=np.asarray(modes, np.int32),
                    out_slope=np.asarray(slopes, np.float32), n_times=T)
