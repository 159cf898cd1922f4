"""Seeded inputs of the normalisation parity cases (shared by the golden generator, the CPU
oracle tests and the GPU tests)."""
import numpy as np
import torch

# shape (B, D, H, W), quantile, intensity kind
CASES = {
    "uniform": {"shape": (3, 9, 10, 11), "q": 0.99, "kind": "uniform", "seed": 1},
    "ints_q97": {"shape": (2, 16, 12, 14), "q": 0.97, "kind": "ints", "seed": 2},
    "signed_q50": {"shape": (2, 7, 9, 11), "q": 0.5, "kind": "signed", "seed": 3},
    "q100": {"shape": (1, 8, 8, 8), "q": 1.0, "kind": "uniform", "seed": 4},
    "brain64": {"shape": (2, 64, 64, 64), "q": 0.99, "kind": "ints", "seed": 5},
}


def make_case(spec):
    rng = np.random.default_rng(spec["seed"])
    shp = spec["shape"]
    if spec["kind"] == "uniform":
        x = rng.random(shp)
    elif spec["kind"] == "ints":           # quantised scanner intensities: many duplicates
        x = rng.integers(0, 400, size=shp).astype(np.float64)
    else:
        x = rng.normal(size=shp) * 3.0
    # brain mask: a ball, plus a few in-mask voxels with intensity exactly 0
    b, d, h, w = shp
    zz, yy, xx = np.meshgrid(np.arange(d), np.arange(h), np.arange(w), indexing="ij")
    ball = ((zz - d / 2) ** 2 / (d / 2.2) ** 2 + (yy - h / 2) ** 2 / (h / 2.2) ** 2 +
            (xx - w / 2) ** 2 / (w / 2.2) ** 2) <= 1.0
    m = np.broadcast_to(ball, shp).astype(np.float64).copy()
    x.reshape(-1)[rng.integers(0, x.size, size=max(1, x.size // 50))] = 0.0
    return torch.from_numpy(x), torch.from_numpy(m)
