"""BASELINE configs 3/4 and 5 (build extensions): the two-backbone
PET+MRI late fusion (ResNet-10 x2 + MLP head) and the three-branch fusion (MRI ResNet-34 +
PET ResNet-18 + tabular MLP), on the MI355X through libmmad_hip.so.

  * fp32 at 32^3 against the CPU oracle's restatement of the same networks
    (oracle/models_ref.py ResNetPairFusionRef / TriResNetTabularRef): logits 1e-4, argmax,
    loss, and every gradient within the f64 bar of test_model_parity_gpu;
  * bf16 at the configs' full sizes (128^3 pairs, batch 8; 160^3, batch 2) against the
    fp32 HIP path on the same weights: finite, bounded logit drift, loss."""
import numpy as np
import pytest
import torch

import multimodal_alzheimer_amd as M
from oracle import models_ref
from tests import _golden as G
from tests.test_model_parity_gpu import _assert_f64_bar

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pair(h, product):
    if product:
        return M.PET_MRI_ResNet_Fusion(h)
    return models_ref.ResNetPairFusionRef(h, models_ref.PETResNetRef(_stage1(h, 10)),
                                          models_ref.AnatCNNRef(_stage1(h, 10)))


def _three(h, product):
    if product:
        return M.Tri_ResNet_Tabular_Fusion(h)
    return models_ref.TriResNetTabularRef(h, models_ref.AnatCNNRef(_stage1(h, 34)),
                                       models_ref.PETResNetRef(_stage1(h, 18)))


def _hp(kind):
    if kind == "pair":                    # config 3/4: ResNet-10 x2
        return G.anat_hparams(10, fl_gamma=2)
    return G.anat_hparams(10, fl_gamma=2, resnet_depth_mri=34, resnet_depth_pet=18)


def _stage1(h, depth):
    return dict(h, resnet_depth=depth, linear_out=[], conv_out=[], filter_size=[],
                batchnorm_begin=False, batchnorm_dense=False)


def _batch(n, s, seed, tab):
    b = G.batch_for((n, s, s, s), 2, seed, ("pet1451", "mri"))
    if tab:
        g = torch.Generator().manual_seed(seed)
        b["tabular"] = torch.rand((n, 9), generator=g, dtype=torch.float64)
    return b


def _live(model):
    with torch.no_grad():             # head bias: every sample keeps a positive pre-ReLU
        for m in model.modules():
            if isinstance(m, torch.nn.Linear) and m.out_features == 64:
                m.bias.add_(0.5)


@pytest.mark.parametrize("kind", ["pair", "three"])
def test_fusion_config_matches_oracle_fp32(kind):
    build = _pair if kind == "pair" else _three
    h = _hp(kind)
    ref = build(h, False)
    G.load_prng_weights(ref, 71)
    _live(ref)
    m = build(h, True)
    assert list(m.state_dict()) == list(ref.state_dict())
    m.load_state_dict(ref.state_dict())
    m = m.to(DEV)
    batch = _batch(2, 32, 72, kind == "three")
    r = ref.general_step(batch, 0, "train")
    r["loss"].backward()
    o = m.general_step({k: v.to(DEV) for k, v in batch.items()}, 0, "train")
    o["loss"].backward()
    got, exp = o["outputs"].detach().cpu().numpy(), r["outputs"].detach().numpy()
    assert np.abs(got - exp).max() <= 1e-4
    assert (got.argmax(1) == exp.argmax(1)).all()
    assert abs(o["loss"].item() - r["loss"].item()) <= 1e-4 * max(1.0, abs(r["loss"].item()))
    # gradients against an f64 evaluation of the oracle
    r64 = build(h, False)
    r64.load_state_dict(ref.state_dict())
    r64 = r64.double()
    if kind == "pair":
        y64 = r64(batch["pet1451"].unsqueeze(1).double(), batch["mri"].unsqueeze(1).double())
    else:
        y64 = r64(*r64.inputs(batch, torch.float64))
    r64.criterion(y64, batch["label"]).backward()
    exact = {k: p.grad.double().numpy().ravel() for k, p in r64.named_parameters()
             if p.grad is not None}
    gscale = max(np.abs(v).max() for v in exact.values())
    ref32 = dict(ref.named_parameters())
    n = 0
    for k, p in m.named_parameters():
        if k not in exact:
            continue
        _assert_f64_bar(k, p.grad.detach().double().cpu().numpy().ravel(),
                        ref32[k].grad.double().numpy().ravel(), exact[k], gscale, p.shape[0])
        n += 1
    assert n > 20


@pytest.mark.parametrize("kind,n,s", [("pair", 8, 128), ("three", 2, 160)],
                         ids=["config3_128", "config5_160"])
def test_fusion_config_full_size_bf16_tracks_fp32(kind, n, s):
    build = _pair if kind == "pair" else _three
    h = _hp(kind)
    torch.manual_seed(73)
    m32 = build(dict(h, precision="32"), True)
    _live(m32)
    m16 = build(dict(h, precision="bf16"), True)
    m16.load_state_dict(m32.state_dict())
    m32, m16 = m32.to(DEV), m16.to(DEV)
    g = torch.Generator(device=DEV).manual_seed(74)
    batch = {"mri": torch.rand((n, s, s, s), generator=g, device=DEV, dtype=torch.float64),
             "pet1451": torch.randn((n, s, s, s), generator=g, device=DEV, dtype=torch.float64),
             "label": torch.randint(0, 2, (n,), generator=g, device=DEV)}
    if kind == "three":
        batch["tabular"] = torch.rand((n, 9), generator=g, device=DEV, dtype=torch.float64)
    out = {}
    for key, m in (("32", m32), ("16", m16)):
        r = m.general_step(batch, 0, "train")
        r["loss"].backward()
        out[key] = (r["outputs"].detach(), r["loss"].item())
    torch.cuda.synchronize()
    l32, l16 = out["32"][0], out["16"][0]
    assert torch.isfinite(l16).all() and np.isfinite(out["16"][1])
    scale = max(1.0, l32.abs().max().item())
    assert (l16 - l32).abs().max().item() <= 3e-2 * scale
    assert abs(out["16"][1] - out["32"][1]) <= 3e-2 * max(1.0, abs(out["32"][1]))
    for (k, a), (_, b) in zip(m32.named_parameters(), m16.named_parameters()):
        if a.grad is not None:
            assert b.grad is not None and torch.isfinite(b.grad).all(), k
