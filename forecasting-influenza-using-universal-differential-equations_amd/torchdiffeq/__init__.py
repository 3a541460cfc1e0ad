"""Drop-in for ``from torchdiffeq import odeint`` (lib/VAE.py:5, run_ode.py:24,
tuning/*.py): the reference's solver entry point, served by ude_amd."""
from ude_amd.solvers import odeint  # noqa: F401

__all__ = ["odeint"]
