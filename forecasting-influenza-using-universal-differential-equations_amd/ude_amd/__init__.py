"""MI355X-native UDE influenza forecaster: the batched RK4 solve of the SIR-UDE
right-hand side (forward + backward through the solver) as gfx950 kernels,
behind the reference's own API (lib/models.py classes, torchdiffeq.odeint).
"""
from .rhs import Fp, Fa, FaFp, UDE_CLASSES
from .solvers import odeint, fusable
from .adjoint import odeint_adjoint
from . import _native, configs

__all__ = ["Fp", "Fa", "FaFp", "odeint", "odeint_adjoint", "fusable", "UDE_CLASSES"]
