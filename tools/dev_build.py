"""Development build: the prebuilt library with only the configurations matching the given
substrings of their config keys (e.g. `python tools/dev_build.py FaFp_R49`).  Other shapes JIT on
first use.  Run __graft_entry__.build() for the full prebuilt set before committing."""
import importlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
importlib.import_module("forecasting-influenza-using-universal-differential-equations_amd")
from ude_amd import _native, configs  # noqa: E402

pats = sys.argv[1:]
sel = [c for c in configs.PREBUILT if any(p in configs.config_key(c) for p in pats)]
print("building", [configs.config_key(c) for c in sel])
os.makedirs(_native.BUILD, exist_ok=True)
print(_native.build_library(sel, _native.PREBUILT_LIB, "prebuilt"))
