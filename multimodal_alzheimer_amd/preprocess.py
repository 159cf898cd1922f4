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

Two ways in (dataset.MultiModalDataset):

* default -- the reference's contract: ``__getitem__`` normalises each sample on the host in
  the loader worker (:func:`loader_normalize_pet` / :func:`loader_normalize_mri`, the
  reference's own float64 torch statements), so an unchanged ``train_*.py`` gets the
  reference's tensors;
* ``device_normalize=True`` (opt-in) -- ``__getitem__`` returns the raw volumes, the brain
  mask and a :data:`NORM_SPEC_KEY` string naming the settings; the model's
  ``on_after_batch_transfer`` / ``general_step`` (classifiers.Base_Model.prepare_batch ->
  :func:`apply_batch_spec`) runs the batched device kernels above on the collated batch.
  Same values (min_max and the affine forms bit-exact, z-score to rounding).
"""
import json

import torch

from . import _lib as L

NORM_SPEC_KEY = "normalize"


# ------------------------------------------------------------ loader-side (host) statements
def loader_affine(x, mean, std):
    """torchvision ``Normalize(mean, std)`` as the loader applies it to one (D, H, W) float64
    volume (dataloader.py:213-215 PET, :256-257 per-scan z-score, :276-278 all-scan): the
    statistics become 0-d tensors of the volume's dtype, then ``sub`` and ``div``."""
    if x.ndim < 3:
        raise ValueError("Normalize expects a tensor with at least 3 dimensions")
    mean = torch.as_tensor(mean, dtype=x.dtype)
    std = torch.as_tensor(std, dtype=x.dtype)
    if bool((std == 0).any()):
        raise ValueError("std evaluated to zero after conversion to float64, leading to "
                         "division by zero.")
    return x.sub(mean).div(std)


def _brain_values(mri, mask):
    """dataloader.py:244-249: the masked volume's nonzero entries, flattened."""
    v = (mri * mask).reshape(-1)
    return v[v.nonzero()]


def loader_normalize_pet(pet, normalize_pet):
    """dataloader.py:213-215."""
    return loader_affine(pet, normalize_pet["mean"], normalize_pet["std"])


def loader_normalize_mri(mri, mask, normalize_mri, quantile):
    """dataloader.py:236-281 for one scan (float64 host tensors); ``mask`` is only read by the
    per-scan modes."""
    if not isinstance(normalize_mri, dict) or len(normalize_mri) != 1:
        raise AssertionError("normalize_mri must be a dict with one key")
    if "per_scan_norm" in normalize_mri:
        mode = normalize_mri["per_scan_norm"]
        v = _brain_values(mri, mask)
        if mode == "normalize":
            std, mean = torch.std_mean(v)
            return loader_affine(mri, mean, std) * mask
        if mode == "min_max":
            if not 0 <= quantile <= 1:
                raise AssertionError("quantile must lie in [0, 1]")
            hi = torch.quantile(v, quantile, interpolation="linear")
            lo = torch.quantile(v, 1 - quantile, interpolation="linear")
            out = (mri - lo) / (hi - lo)
            out[out > 1] = 1                  # masked stores, not clamp: -0.0 and NaN kept
            out[out < 0] = 0                  # exactly as the loader leaves them
            return out.mul_(mask)
        raise ValueError('If you want to normalize per scan you have to pass either '
                         '"normalize" or "min_max"')
    if "all_scan_norm" in normalize_mri:
        st = normalize_mri["all_scan_norm"]
        return loader_affine(mri, st["mean"], st["std"])
    raise ValueError('If you use the argument "normalize_mri" only "per_scan_norm" or '
                     '"all_scan_norm" are allowed as keys!')


# ------------------------------------------------------------------ opt-in device path spec
def spec_string(normalize_mri, normalize_pet, quantile):
    """The settings a device-normalising dataset attaches to every sample (a string, so the
    DataLoader collates it into a list and the device transfer leaves it alone)."""
    def _f(d):
        return None if not d else {k: (_f(v) if isinstance(v, dict) else
                                        (v if isinstance(v, str) else float(v)))
                                    for k, v in d.items()}
    return json.dumps({"normalize_mri": _f(normalize_mri), "normalize_pet": _f(normalize_pet),
                       "quantile": float(quantile)}, sort_keys=True)


_NORMALIZERS = {}


def apply_batch_spec(batch):
    """Run the device normalisation a collated batch asks for (its :data:`NORM_SPEC_KEY`
    entry), returning the batch the reference loader would have produced: normalised
    'mri' / 'pet1451', no 'mri_mask', no spec.  Batches without a spec pass through."""
    if not isinstance(batch, dict) or NORM_SPEC_KEY not in batch:
        return batch
    spec = batch[NORM_SPEC_KEY]
    if isinstance(spec, (list, tuple)):
        if len(set(spec)) != 1:
            raise ValueError("a batch mixes samples with different normalisation settings")
        spec = spec[0]
    norm = _NORMALIZERS.get(spec)
    if norm is None:
        norm = _NORMALIZERS[spec] = VolumeNormalizer(**json.loads(spec))
    out = norm({k: v for k, v in batch.items() if k != NORM_SPEC_KEY})
    out.pop("mri_mask", None)
    return out


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
