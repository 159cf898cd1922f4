"""Counter-based splitmix64 PRNG (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py).

Every synthetic weight / volume used by the parity tests and golden fixtures is a pure
function of (seed, element index), so the GPU box regenerates exactly the tensors the
fixtures were produced from without shipping them.  numpy uint64 arithmetic wraps mod
2**64, which is exactly splitmix64's arithmetic.
"""
import zlib

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)
_SEED_MUL = np.uint64(0xD1342543DE82EF95)


def _mix(x):
    z = x + _GAMMA
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def uniform(seed, n):
    """n float32 values in [0, 1), 24-bit exact (so identical in f32/f64/bf16-free)."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) * _SEED_MUL
        x = _mix(np.arange(n, dtype=np.uint64) + base)
    return ((x >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)).astype(np.float32)


def name_seed(base_seed, name):
    return (int(base_seed) * 1000003 + zlib.crc32(name.encode())) & 0xFFFFFFFF


def mri_volume(seed, shape):
    """uniform[0,1) like the per-scan min-max normalised MRI (dataloader.py:261-270)."""
    n = int(np.prod(shape))
    return uniform(seed, n).reshape(shape)


def pet_volume(seed, shape):
    """uniform[-2,2): a bounded stand-in for z-scored PET (dataloader.py:213-215)."""
    n = int(np.prod(shape))
    return (uniform(seed, n) * 4.0 - 2.0).astype(np.float32).reshape(shape)


def labels(seed, n, n_classes):
    return np.minimum((uniform(seed, n) * n_classes).astype(np.int64), n_classes - 1)


def param_value(base_seed, name, shape):
    """Deterministic value for one state_dict entry, chosen by its key suffix.

    conv / linear weights: kaiming-uniform-like U(-b, b), b = sqrt(6 / fan_in);
    biases U(-0.1, 0.1); BN affine near (1, 0); BN running stats near (0, 1).
    """
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform(name_seed(base_seed, name), n).astype(np.float64)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "weight" and len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        b = np.sqrt(6.0 / fan_in)
        v = (2.0 * u - 1.0) * b
    elif leaf == "weight":                  # BN / BN1d affine weight
        v = 1.0 + 0.4 * (u - 0.5)
    elif leaf == "bias":
        v = 0.2 * (u - 0.5)
    elif leaf == "running_mean":
        v = 0.2 * (u - 0.5)
    elif leaf == "running_var":
        v = 0.5 + u
    else:
        raise KeyError(name)
    return v.astype(np.float32).reshape(shape)


def sample_index(name, n, k=1024):
    """Sorted distinct element indices (at most k of n) at which the full-size fixtures
    record a tensor: a pure function of the tensor's name, so the GPU tests pick the same
    elements without the fixture shipping them."""
    if n <= k:
        return np.arange(n, dtype=np.int64)
    idx = (uniform(name_seed(0x5A3B1E, name), k).astype(np.float64) * n).astype(np.int64)
    return np.unique(np.minimum(idx, n - 1))


def fill_state_dict(state_dict, base_seed):
    """Return {key: np.float32 array} for every float entry of a state_dict."""
    out = {}
    for k, t in state_dict.items():
        if not t.is_floating_point():
            continue
        if k.endswith("criterion.weight"):
            continue                        # class weights come from the hparams
        out[k] = param_value(base_seed, k, tuple(t.shape))
    return out
