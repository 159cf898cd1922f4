"""Golden vectors for the input-pipeline normalisation (dataloader.py:244-277).

Runs the reference loader's normalisation statements (restated in oracle/preprocess_ref.py;
the module itself needs nibabel, absent here) on PRNG volumes with duplicate intensities,
negative values and in-mask zeros, and stores inputs' seeds + outputs + quantiles.

    python tests/golden/make_norm_golden.py
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import preprocess_ref as P  # noqa: E402
from tests._norm_cases import CASES, make_case  # noqa: E402


def main():
    out = {}
    for name, spec in CASES.items():
        x, m = make_case(spec)
        q = spec["q"]
        ys, qs = [], []
        for b in range(x.shape[0]):
            y, lo, hi = P.mri_minmax_ref(x[b].clone(), m[b], q)
            ys.append(y.numpy())
            qs.append((lo, hi))
        out[f"{name}_q"] = np.asarray(qs)
        if x[0].numel() > 4096:            # large case: quantiles only (outputs recomputed)
            continue
        out[f"{name}_minmax"] = np.stack(ys)
        out[f"{name}_zscore"] = np.stack([P.mri_zscore_ref(x[b].clone(), m[b]).numpy()
                                          for b in range(x.shape[0])])
    np.savez_compressed(os.path.join(HERE, "norm.npz"), **out)
    print("wrote", sorted(out))


if __name__ == "__main__":
    main()
