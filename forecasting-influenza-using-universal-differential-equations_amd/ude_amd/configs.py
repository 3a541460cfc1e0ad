"""Model configurations compiled into the prebuilt gfx950 library.

Each entry is (kind, n_regions, latent_dim, net_sizes, aug_net_sizes).  The
list covers the configurations the reference actually runs -- ``run_ode.py``
``region_info`` (:40-68: US R=1, hhs R=10, state R=49; L=8; net_sizes
[64, 64, 32], aug_net_sizes [64, 64]) for every ODE class of ``run_ode.py:99``
-- the class defaults of ``lib/models.py`` (:110, :159, :200), the
north-star Fp [32, 32] benchmark model, and the golden-fixture shapes.  Any
other configuration is compiled on first use (see ``_native.jit_library``).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

Config = Tuple[str, int, int, Optional[Tuple[int, ...]], Optional[Tuple[int, ...]]]

# "B" prefix: the Bayesian right-hand sides of lib/in_development/models_bayes.py
# (UDE_KIND_BAYES = 4 in include/ude_rk4.h)
KIND_CODE = {"Fp": 1, "Fa": 2, "FaFp": 3, "BFp": 5, "BFa": 6, "BFaFp": 7}


def base_kind(kind: str) -> str:
    return kind[1:] if kind.startswith("B") else kind


def _c(kind: str, R: int, L: int, net: Optional[Sequence[int]], aug: Optional[Sequence[int]]) -> Config:
    b = base_kind(kind)
    return (kind, R, L, tuple(net) if net is not None and b != "Fa" else None,
            tuple(aug) if aug is not None and b != "Fp" else None)


PREBUILT: List[Config] = []
for _R in (1, 10, 49):                               # run_ode.py region_info
    PREBUILT.append(_c("FaFp", _R, 8, [64, 64, 32], [64, 64]))
    PREBUILT.append(_c("Fp", _R, 8, [64, 64, 32], None))
    PREBUILT.append(_c("Fa", _R, 8, None, [64, 64]))
PREBUILT += [
    _c("Fp", 1, 8, [32, 32], None),                  # north-star Fp "32-hidden" (BASELINE configs[0])
    _c("FaFp", 1, 8, [20, 20], [32, 32]),            # lib/models.py class defaults
    _c("Fp", 1, 8, [20, 20], None),
    _c("Fa", 1, 8, None, [32, 32]),
    _c("Fp", 1, 6, [24], None),                      # golden: fp_r1_onehidden
    _c("FaFp", 3, 5, [40, 24], [36], ),              # golden: fafp_r3_l5_ragged
    # golden single-evaluation fixtures rhs_{fp,fa,fafp}_r{1,4} (net [16, 16, 8], aug [16, 12])
    _c("Fp", 1, 8, [16, 16, 8], None), _c("Fa", 1, 8, None, [16, 12]), _c("FaFp", 1, 8, [16, 16, 8], [16, 12]),
    _c("Fp", 4, 8, [16, 16, 8], None), _c("Fa", 4, 8, None, [16, 12]), _c("FaFp", 4, 8, [16, 16, 8], [16, 12]),
    # Bayesian RHS (run_ode.py:99 'CONNb' / 'UONNb' / 'SONNb'), US model sizes
    _c("BFaFp", 1, 8, [64, 64, 32], [64, 64]),
    _c("BFp", 1, 8, [64, 64, 32], None),
    _c("BFa", 1, 8, None, [64, 64]),
    # ... and the hhs / state region sets (R = 10, 49): whole-solve kernels with the weight gradients
    # formed per evaluation by ude_gst_dw_kernel (Model::GST)
    _c("BFaFp", 10, 8, [64, 64, 32], [64, 64]),
    _c("BFp", 10, 8, [64, 64, 32], None),
    _c("BFaFp", 49, 8, [64, 64, 32], [64, 64]),
    _c("BFp", 49, 8, [64, 64, 32], None),
    _c("BFaFp", 1, 8, [20, 20], [32, 32]),           # models_bayes.py class defaults
    _c("BFp", 1, 8, [20, 20], None),
    _c("BFa", 1, 8, None, [32, 32]),
]


def config_key(cfg: Config) -> str:
    kind, R, L, net, aug = cfg
    n = "-".join(map(str, net)) if net else "x"
    a = "-".join(map(str, aug)) if aug else "x"
    return f"{kind}_R{R}_L{L}_p{n}_a{a}"


def template_args(cfg: Config) -> str:
    """Model<R, L, KIND, NPH, P0..P3, NAH, A0..A3> argument list."""
    kind, R, L, net, aug = cfg
    net = list(net or [])
    aug = list(aug or [])
    if len(net) > 4 or len(aug) > 4:
        raise ValueError("at most 4 hidden layers per MLP are supported")
    p = net + [0] * (4 - len(net))
    a = aug + [0] * (4 - len(aug))
    return ",".join(str(v) for v in [R, L, KIND_CODE[kind], len(net), *p, len(aug), *a])
