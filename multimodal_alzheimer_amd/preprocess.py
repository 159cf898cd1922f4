"""Input-pipeline normalisation on device (float64), batched over scans.

The reference normalises every sample on the CPU inside ``MultiModalDataset.__getitem__``
(pkg/utils/dataloader.py) with 32 loader workers, in float64:

* PET (dataloader.py:213-215): ``Normalize(mean, std)`` with split statistics
  -> :func:`affine_normalize`;
* MRI ``{'all_scan_norm': {'mean', 'std'}}`` (:272-277) -> :func:`affine_normalize`;
* MRI ``{'per_scan_norm': 'min_max'}`` with ``quantile`` (:262-270): quantile min-max over the
  brain mask -> :func:`mri_per_scan_minmax` (bit-exact: exact order statistics + torch's
  lerp);
* MRI ``{'per_scan_norm': 'normalize'}`` (:253-260): per-scan z-score over the brain mask ->
  :func:`mri_per_scan_zscore` (fp64 sums in a fixed order; matches torch.std_mean to
  rounding).

Every function takes device tensors ``(B, D, H, W)`` (or any shape with the scan index
first) and calls libmmad_hip.so; there is no CPU path (a CPU tensor raises).
:class:`VolumeNormalizer` applies the reference's ``normalize_mri`` / ``normalize_pet``
dicts to a batch dict on device, so a loader built with ``normalize_*=None`` (raw volumes +
``mri_mask``) feeds ``general_step`` exactly what the reference loader would.
"""
import torch

from . import _lib as L


def _scans(x):
    L.require_device(x)
    if x.dtype != torch.float64:
        raise L.MMADError("normalisation runs in float64 (the reference loader's dtype)")
    if not x.is_contiguous():
        raise L.MMADError("volumes must be contiguous")
    b = x.shape[0]
    return b, x.numel() // b


def _workspace(b, vox, device):
    n = L.load().mmad_norm_ws_bytes(b, vox)
    return torch.empty(n, dtype=torch.uint8, device=device)


def mri_per_scan_minmax(x, mask, quantile=0.99, return_quantiles=False):
    """dataloader.py:262-270 per scan: lo, hi = quantile(v, 1-q), quantile(v, q) of
    v = nonzero(x * mask); out = clamp((x - lo) / (hi - lo), 0, 1) * mask."""
    b, vox = _scans(x)
    if mask.shape != x.shape:
        raise L.MMADError("mask must match the volume shape")
    mask = mask.to(torch.float64).contiguous()
    out = torch.empty_like(x)
    q = torch.empty((b, 2), dtype=torch.float64, device=x.device) if return_quantiles else None
    L.call("mmad_mri_minmax_norm", b, vox, L.ptr(x), L.ptr(mask), float(quantile), L.ptr(out),
           L.ptr(_workspace(b, vox, x.device)), L.ptr(q), L.stream())
    return (out, q) if return_quantiles else out


def mri_per_scan_zscore(x, mask):
    """dataloader.py:253-260 per scan: (x - mean(v)) / std(v) * mask, v = nonzero(x*mask)."""
    b, vox = _scans(x)
    if mask.shape != x.shape:
        raise L.MMADError("mask must match the volume shape")
    mask = mask.to(torch.float64).contiguous()
    out = torch.empty_like(x)
    L.call("mmad_mri_zscore_norm", b, vox, L.ptr(x), L.ptr(mask), L.ptr(out),
           L.ptr(_workspace(b, vox, x.device)), L.stream())
    return out


def affine_normalize(x, mean, std):
    """torchvision Normalize(mean, std) with scalar statistics: (x - mean) / std."""
    _scans(x)
    out = torch.empty_like(x)
    L.call("mmad_affine_norm", x.numel(), L.ptr(x), float(mean), float(std), L.ptr(out),
           L.stream())
    return out


class VolumeNormalizer:
    """Apply the reference loader's normalisation settings to a device batch.

    ``normalize_mri``: None | {'per_scan_norm': 'min_max' | 'normalize'} |
    {'all_scan_norm': {'mean': m, 'std': s}}; ``normalize_pet``: None | {'mean', 'std'};
    ``quantile`` as MultiModalDataset (dataloader.py:63-73).  ``__call__(batch)`` returns a
    new dict with 'mri' / 'pet1451' normalised (per-scan MRI modes need 'mri_mask')."""

    def __init__(self, normalize_mri=None, normalize_pet=None, quantile=0.99):
        if normalize_mri is not None:
            if not isinstance(normalize_mri, dict) or len(normalize_mri) != 1:
                raise ValueError("normalize_mri must be a dict with one key")
            key = next(iter(normalize_mri))
            if key == "per_scan_norm":
                if normalize_mri[key] not in ("min_max", "normalize"):
                    raise ValueError('If you want to normalize per scan you have to pass either '
                                     '"normalize" or "min_max"')
            elif key != "all_scan_norm":
                raise ValueError('If you use the argument "normalize_mri" only "per_scan_norm" '
                                 'or "all_scan_norm" are allowed as keys!')
        if not 0.0 <= quantile <= 1.0:
            raise ValueError("quantile must lie in [0, 1]")
        self.normalize_mri, self.normalize_pet, self.quantile = normalize_mri, normalize_pet, quantile

    def __call__(self, batch):
        out = dict(batch)
        if self.normalize_pet is not None and batch.get("pet1451") is not None:
            out["pet1451"] = affine_normalize(batch["pet1451"], self.normalize_pet["mean"],
                                              self.normalize_pet["std"])
        nm = self.normalize_mri
        if nm is not None and batch.get("mri") is not None:
            x = batch["mri"]
            if "all_scan_norm" in nm:
                out["mri"] = affine_normalize(x, nm["all_scan_norm"]["mean"],
                                              nm["all_scan_norm"]["std"])
            elif nm["per_scan_norm"] == "min_max":
                out["mri"] = mri_per_scan_minmax(x, batch["mri_mask"], self.quantile)
            else:
                out["mri"] = mri_per_scan_zscore(x, batch["mri_mask"])
        return out
