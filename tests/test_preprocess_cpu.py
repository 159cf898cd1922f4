"""CPU checks of the normalisation oracle (oracle/preprocess_ref.py) against torch.quantile
and the committed golden vectors (tests/golden/norm.npz)."""
import os

import numpy as np
import pytest
import torch

from oracle import preprocess_ref as P
from tests._norm_cases import CASES, make_case

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "norm.npz"))


@pytest.mark.parametrize("q", [0.0, 0.01, 0.03, 0.25, 0.5, 0.97, 0.99, 1.0])
@pytest.mark.parametrize("n", [1, 2, 7, 100, 1001])
def test_quantile_restatement_matches_torch(q, n):
    g = torch.Generator().manual_seed(n)
    v = torch.randint(0, 50, (n,), generator=g).double() + torch.rand(n, generator=g, dtype=torch.float64).round()
    assert P.quantile_linear(v.numpy(), q) == torch.quantile(v, q, interpolation="linear").item()


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_matches_golden(name):
    x, m = make_case(CASES[name])
    q = CASES[name]["q"]
    for b in range(x.shape[0]):
        y, lo, hi = P.mri_minmax_ref(x[b].clone(), m[b], q)
        assert (lo, hi) == tuple(GOLD[f"{name}_q"][b])
        v = (x[b] * m[b]).reshape(-1)
        v = v[v != 0].numpy()
        assert (P.quantile_linear(v, 1 - q), P.quantile_linear(v, q)) == (lo, hi)
        if f"{name}_minmax" in GOLD:
            assert np.array_equal(y.numpy(), GOLD[f"{name}_minmax"][b], equal_nan=True)
            z = P.mri_zscore_ref(x[b].clone(), m[b]).numpy()
            assert np.array_equal(z, GOLD[f"{name}_zscore"][b], equal_nan=True)


def test_preprocess_requires_device():
    from multimodal_alzheimer_amd import preprocess, _lib
    x = torch.zeros((1, 4, 4, 4), dtype=torch.float64)
    with pytest.raises(_lib.MMADError):
        preprocess.mri_per_scan_minmax(x, x)
