"""Deterministic, formula-defined parameter generator.

No pretrained weights exist for the reference (its checkpoints are Git-LFS pointers,
SURVEY.md Finding 6), so parity runs on *injected* weights.  Every value is a pure
function of (parameter name, element index): a splitmix64 counter hash mapped to
U(-a, a).  The golden-fixture script loads the same values into the reference model
with ``load_state_dict``, so weights are never committed.

Scale rules (by state_dict key):
  * ``*.weight`` with ndim >= 2 (conv / linear / tables): a = 1/sqrt(fan_in)
  * 1-D ``*.weight`` (BatchNorm / LayerNorm affine):    1 + U(-0.1, 0.1)
  * ``*.bias``:                                          U(-0.05, 0.05)
  * ``*.running_mean``:                                  U(-0.1, 0.1)
  * ``*.running_var``:                                   1 + U(-0.1, 0.1)
Integer buffers and any other buffer are left untouched.
"""
import hashlib
import math

import numpy as np

_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_GOLD = np.uint64(0x9E3779B97F4A7C15)


def _name_seed(name: str) -> np.uint64:
    return np.uint64(int.from_bytes(hashlib.sha256(name.encode()).digest()[:8], "little"))


def unit_uniform(name: str, n: int) -> np.ndarray:
    """n values in [-1, 1) as float64, exactly k * 2^-23 - 1 for a 24-bit k."""
    with np.errstate(over="ignore"):
        z = (np.arange(n, dtype=np.uint64) + _name_seed(name)) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    k = (z >> np.uint64(40)).astype(np.float64)
    return k * (2.0 ** -23) - 1.0


def value_for(name: str, shape) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = unit_uniform(name, n)
    if name.endswith("running_var"):
        v = 1.0 + 0.1 * u
    elif name.endswith("running_mean"):
        v = 0.1 * u
    elif name.endswith("bias"):
        v = 0.05 * u
    elif name.endswith("weight") and len(shape) == 1:
        v = 1.0 + 0.1 * u
    else:
        fan_in = n // shape[0] if len(shape) >= 2 else n
        v = u / math.sqrt(max(fan_in, 1))
    return v.astype(np.float32).reshape(shape)


def deterministic_state_dict(module, prefix: str = ""):
    """Return {key: tensor} for every float parameter and BN running stat of ``module``.

    ``prefix`` is prepended to the hashed name so that sub-modules can be generated with
    the keys they have inside the full model (e.g. ``model.pixel_level_module.``).
    """
    import torch

    out = {}
    for key, t in module.state_dict().items():
        if not t.is_floating_point():
            continue
        is_param = key in dict(module.named_parameters())
        if not (is_param or key.endswith("running_mean") or key.endswith("running_var")):
            continue
        out[key] = torch.from_numpy(value_for(prefix + key, tuple(t.shape)))
    return out


def init_deterministic(module, prefix: str = ""):
    """Overwrite ``module``'s parameters/BN stats in place with the generator's values."""
    sd = deterministic_state_dict(module, prefix)
    missing = module.load_state_dict(sd, strict=False)
    return missing
