"""Input-pipeline normalisation on the MI355X through libmmad_hip.so vs the CPU restatement
of dataloader.py:244-277 (oracle/preprocess_ref.py) and the golden quantiles
(tests/golden/norm.npz).  min_max and affine: bit-exact; zscore: within 1e-12 relative
(fixed-order fp64 sums vs torch.std_mean's own order)."""
import os

import numpy as np
import pytest
import torch

from multimodal_alzheimer_amd import preprocess
from oracle import preprocess_ref as P
from tests._norm_cases import CASES, make_case

pytestmark = pytest.mark.gpu
GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "norm.npz"))


@pytest.mark.parametrize("name", sorted(CASES))
def test_minmax_bit_exact(name):
    x, m = make_case(CASES[name])
    q = CASES[name]["q"]
    got, qs = preprocess.mri_per_scan_minmax(x.cuda(), m.cuda(), q, return_quantiles=True)
    got, qs = got.cpu(), qs.cpu()
    for b in range(x.shape[0]):
        ref, lo, hi = P.mri_minmax_ref(x[b].clone(), m[b], q)
        assert (qs[b, 0].item(), qs[b, 1].item()) == (lo, hi) == tuple(GOLD[f"{name}_q"][b])
        assert torch.equal(torch.nan_to_num(got[b], nan=-7.0), torch.nan_to_num(ref, nan=-7.0))


@pytest.mark.parametrize("q", [0.0, 0.03, 0.5, 0.9, 0.99, 1.0])
def test_minmax_quantile_sweep(q):
    x, m = make_case({"shape": (4, 13, 11, 9), "q": q, "kind": "ints", "seed": 11})
    got, qs = preprocess.mri_per_scan_minmax(x.cuda(), m.cuda(), q, return_quantiles=True)
    for b in range(4):
        ref, lo, hi = P.mri_minmax_ref(x[b].clone(), m[b], q)
        assert (qs[b, 0].item(), qs[b, 1].item()) == (lo, hi)
        assert torch.equal(torch.nan_to_num(got[b].cpu(), nan=-7.0),
                           torch.nan_to_num(ref, nan=-7.0))


def test_minmax_empty_mask_is_nan():
    x = torch.rand((2, 5, 5, 5), dtype=torch.float64)
    m = torch.ones_like(x)
    m[1] = 0
    got = preprocess.mri_per_scan_minmax(x.cuda(), m.cuda(), 0.99).cpu()
    assert torch.isnan(got[1]).all() and not torch.isnan(got[0]).any()


@pytest.mark.parametrize("name", sorted(CASES))
def test_zscore(name):
    x, m = make_case(CASES[name])
    got = preprocess.mri_per_scan_zscore(x.cuda(), m.cuda()).cpu()
    for b in range(x.shape[0]):
        ref = P.mri_zscore_ref(x[b].clone(), m[b])
        err = (got[b] - ref).abs().max().item()
        assert err <= 1e-12 * ref.abs().max().item()


def test_affine_and_normalizer():
    x, m = make_case(CASES["uniform"])
    got = preprocess.affine_normalize(x.cuda(), 0.5145, 0.5383).cpu()
    assert torch.equal(got, P.affine_ref(x, 0.5145, 0.5383))
    norm = preprocess.VolumeNormalizer({"per_scan_norm": "min_max"}, {"mean": 0.5145, "std": 0.5383},
                                       quantile=0.99)
    out = norm({"mri": x.cuda(), "mri_mask": m.cuda(), "pet1451": x.cuda(), "label": None})
    ref0, _, _ = P.mri_minmax_ref(x[0].clone(), m[0], 0.99)
    assert torch.equal(out["mri"][0].cpu(), ref0)
    assert torch.equal(out["pet1451"].cpu(), P.affine_ref(x, 0.5145, 0.5383))


@pytest.mark.parametrize("nm", [{"per_scan_norm": "min_max"}, {"per_scan_norm": "normalize"},
                                {"all_scan_norm": {"mean": 150.0, "std": 80.0}}],
                         ids=["min_max", "zscore", "all_scan"])
def test_device_normalize_opt_in_through_general_step(tmp_path, nm):
    """The drop-in dataset built as train_anat_cnn.py:180-185 builds it (default: the
    reference's normalise-on-fetch) and the same table with device_normalize=True (raw
    volumes + mask + settings, normalised on the GPU by the model's prepare_batch) give
    Anat_CNN.general_step the same inputs: identical logits and loss (z-score: to its
    1e-12 statistics)."""
    from multimodal_alzheimer_amd.dataset import MultiModalDataset
    from multimodal_alzheimer_amd.preprocess import NORM_SPEC_KEY
    from tests import _golden as G
    from tests.test_dataset_cpu import _scan_table
    import multimodal_alzheimer_amd as M
    x, m = make_case({"shape": (4, 24, 24, 24), "q": 0.99, "kind": "ints", "seed": 21})
    csv = _scan_table(tmp_path, "opt", x, m)
    host = MultiModalDataset(csv, modalities=["t1w"], normalize_mri=nm, quantile=0.98)
    dev = MultiModalDataset(csv, modalities=["t1w"], normalize_mri=nm, quantile=0.98,
                            device_normalize=True)
    bh = next(iter(torch.utils.data.DataLoader(host, batch_size=4)))
    bd = next(iter(torch.utils.data.DataLoader(dev, batch_size=4)))
    assert NORM_SPEC_KEY in bd and NORM_SPEC_KEY not in bh
    assert ("mri_mask" in bd) == ("per_scan_norm" in nm) and "mri_mask" not in bh
    torch.manual_seed(0)
    model = M.Anat_CNN(G.anat_hparams(10, n_classes=3)).to("cuda")

    def to_dev(b):
        return {k: (v.cuda() if torch.is_tensor(v) else v) for k, v in b.items()}
    # the Lightning hook and general_step's own call are the same function
    got = model.on_after_batch_transfer(to_dev(bd), 0)
    assert set(got) == {"mri", "label"}
    ref_in = to_dev(bh)["mri"]
    if "normalize" in nm.get("per_scan_norm", ""):
        assert (got["mri"] - ref_in).abs().max().item() <= 1e-12 * ref_in.abs().max().item()
    else:
        assert torch.equal(got["mri"], ref_in)
    oh = model.general_step(to_dev(bh), 0, "val")
    od = model.general_step(to_dev(bd), 0, "val")
    if nm.get("per_scan_norm") == "normalize":
        assert (oh["outputs"] - od["outputs"]).abs().max().item() <= 1e-6
    else:
        assert torch.equal(oh["outputs"], od["outputs"])
        assert torch.equal(oh["loss"], od["loss"])
