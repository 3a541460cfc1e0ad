"""forecasting-influenza-using-universal-differential-equations_amd

The package directory itself is put on ``sys.path`` so that its drop-in
sub-packages resolve as the reference's own top-level names:
``lib.models`` / ``lib.train_functions`` / ``lib.VAE`` (the reference's host
API) and ``torchdiffeq`` (the solver API the reference imports).  The core
lives in ``ude_amd``; everything imports it under that one name.
"""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from ude_amd import *  # noqa: E402,F401,F403
import ude_amd  # noqa: E402,F401
