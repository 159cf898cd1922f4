"""CPU restatement of the reference loader's volume normalisation (TEST INFRASTRUCTURE ONLY).

Restates ``MultiModalDataset.__getitem__`` (pkg/utils/dataloader.py) in float64:

* :func:`mri_minmax_ref`  -- :244-249 (mask, flatten, drop zeros) + :262-270 (quantile
  min-max, clamp, re-mask), using the same torch calls as the reference;
* :func:`quantile_linear` -- numpy restatement of ``torch.quantile(..., 'linear')`` (sort,
  rank r = q*(n-1), torch's lerp formula), checked against torch.quantile in
  tests/test_preprocess_cpu.py so the order-statistic algorithm itself is pinned;
* :func:`mri_zscore_ref`  -- :253-260 (torch.std_mean over the masked nonzero values);
* :func:`affine_ref`      -- :213-215 / :272-277 (torchvision Normalize with scalar stats).

The reference module itself cannot be imported here (it needs nibabel, absent offline), so
these functions restate its statements line by line; tests/golden/make_norm_golden.py
records their outputs as fixtures.
"""
import numpy as np
import torch


def quantile_linear(v, q):
    """torch.quantile(v, q, interpolation='linear') for a 1-D float64 array."""
    s = np.sort(np.asarray(v, dtype=np.float64))
    r = q * (s.size - 1)
    lo = int(r)
    hi = int(np.ceil(r))
    w = r - lo
    a, b = s[lo], s[hi]
    return a + w * (b - a) if w < 0.5 else b - (b - a) * (1.0 - w)


def mri_minmax_ref(mri, mask, quantile):
    """dataloader.py:244-249, :262-270 for one scan (float64 torch tensors)."""
    data_masked = (mri * mask).reshape(-1)
    data_masked = data_masked[data_masked.nonzero()]
    qmax = torch.quantile(data_masked, quantile, interpolation="linear")
    qmin = torch.quantile(data_masked, 1 - quantile, interpolation="linear")
    out = (mri - qmin) / (qmax - qmin)
    out[out > 1] = 1
    out[out < 0] = 0
    out *= mask
    return out, float(qmin), float(qmax)


def mri_zscore_ref(mri, mask):
    """dataloader.py:244-249, :253-260 for one scan."""
    data_masked = (mri * mask).reshape(-1)
    data_masked = data_masked[data_masked.nonzero()]
    std, mean = torch.std_mean(data_masked)
    out = (mri - mean) / std
    out *= mask
    return out


def affine_ref(x, mean, std):
    """dataloader.py:213-215 / :272-277: Normalize(mean, std) with scalar statistics."""
    return (x - mean) / std
