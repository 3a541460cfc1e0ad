import glob
import importlib
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "forecasting-influenza-using-universal-differential-equations_amd"
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


def import_pkg():
    return importlib.import_module(PKG_NAME)


@pytest.fixture(scope="session")
def pkg():
    return import_pkg()


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    out = {k: d[k] for k in d.files}
    out["meta"] = json.loads(str(out.pop("meta_json")))
    return out


def solver_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "*.npz"))
                  if not os.path.basename(p).startswith(("rhs_", "e2e_", "bayes_", "loss_")))


def bayes_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "bayes_*.npz")))


def rhs_cases():
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, "rhs_*.npz")))
