"""Drop-in for ``from torchdiffeq import odeint`` (lib/VAE.py:5, run_ode.py:24,
tuning/*.py) and ``odeint_adjoint`` (torchdiffeq's adjoint API, BASELINE configs[2]): the
solver entry points, served by ude_amd."""
from ude_amd.solvers import odeint  # noqa: F401
from ude_amd.adjoint import odeint_adjoint  # noqa: F401

__all__ = ["odeint", "odeint_adjoint"]
