"""The reference's own input geometry on the fast path: 91 x 109 x 91 MNI volumes
(pkg/utils/dataloader.py:228-229), 12 x 14 x 12 at layer3 / layer4
(pkg/utils/outdated/inspect_model.py:105).  Those grids are not 4d^3, so the residue-class
kernels run their ragged form (latticeconv.hip / lattice8.hip, RAG): a class's sub-lattice
is 3 x (3|4) x 3 (layer4) or 6 x 7 x 6 (layer3) inside the kernels' 4 x 4 / 8 x 8 planes.

* every dilated layer3 / layer4 conv at batch 8, bf16, forward + dX + dW + BN partial sums
  against the plain fp32-torch im2col reference of test_fullsize_gpu (same bounds), after
  checking the layer really takes the residue-class kernel (its stats row count);
* the whole Anat_CNN at the golden ``anat_r10_mni`` case (reference code, fp32, B=2) in bf16,
  with the residue-class kernels forced on at that batch (mode 2: at batch 2 their tiles
  would not fill the CUs, so mode 1 leaves those layers to the implicit GEMM): logits
  within 3e-2 of max(1, |logit|) of the reference's, argmax wherever the reference's
  top-2 margin exceeds twice that."""
import numpy as np
import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd import _lib
from multimodal_alzheimer_amd import volume_ops as V
from tests import _golden as G
from tests.test_fullsize_gpu import _check, _ref_conv

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d
BF = torch.bfloat16
GRID = (12, 14, 12)

# (name, Ci, Co, dilation, residue-class stats rows at batch 8 = planes per class x groups)
LAYERS = [
    ("layer3.0.conv1", 128, 256, 2, 8 * 6),
    ("layer3.0.conv2", 256, 256, 2, 8 * 6),
    ("layer4.0.conv1", 256, 512, 4, 8 * 2 * 3),
    ("layer4.0.conv2", 512, 512, 4, 8 * 2 * 3),
]


@pytest.mark.parametrize("case", LAYERS, ids=[c[0] for c in LAYERS])
def test_mni_dilated_conv_layer(case):
    name, ci, co, dl, rows = case
    n = 8
    d = V.conv_desc((n, ci) + GRID, (co, ci, 3, 3, 3), (1, 1, 1), (dl,) * 3, (dl,) * 3)
    assert _lib.load().mmad_conv3d_stats_rows(d, _lib.BF16) == rows, \
        f"{name}: not routed to the residue-class kernel"
    g = torch.Generator(device=DEV).manual_seed(300 + ci + dl)
    x = (torch.rand((n, ci) + GRID, generator=g, device=DEV) * 2 - 1).to(BF)
    w = (torch.rand((co, ci, 3, 3, 3), generator=g, device=DEV) * 2 - 1) * (3.0 / (ci * 27)) ** 0.5
    xg = x.contiguous(memory_format=CL).requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y, stats = V.conv3d(xg, wg, None, (1,) * 3, (dl,) * 3, (dl,) * 3, BF, want_stats=True)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    y.backward(gy)
    torch.cuda.synchronize()
    xr = x.float().requires_grad_(True)
    wr = w.to(BF).float().requires_grad_(True)
    yr = _ref_conv(xr, wr, 1, dl, dl)
    yr.backward(gy.float())
    _check(y, yr, 2 ** -7, 1e-3, f"{name} y")
    _check(xg.grad, xr.grad, 2 ** -7, 1e-3, f"{name} dX")
    _check(wg.grad, wr.grad, 1e-3, 1e-4, f"{name} dW")
    ysum = yr.detach().sum(dim=(0, 2, 3, 4))
    ysq = (yr.detach() ** 2).sum(dim=(0, 2, 3, 4))
    absum = yr.detach().abs().sum(dim=(0, 2, 3, 4))
    assert ((stats[:, 0].sum(0) - ysum).abs() <= 1e-4 * absum + 1e-6).all(), name
    assert ((stats[:, 1].sum(0) - ysq).abs() <= 1e-4 * ysq + 1e-6).all(), name


def test_mni_model_bf16_tracks_reference():
    g = G.load("anat_r10_mni")
    m = M.Anat_CNN(G.anat_hparams(10, precision="bf16"))
    G.load_prng_weights(m, int(g["seed"]))
    m = m.to(DEV)
    batch = {k: v.to(DEV) for k, v in G.batch_of("anat_r10_mni", g).items()}
    m.train()
    lib = _lib.load()
    prev = (lib.mmad_set_kernel_variant(b"lattice", 2), lib.mmad_set_kernel_variant(b"lattice8", 2))
    try:
        d4 = V.conv_desc((2, 512) + GRID, (512, 512, 3, 3, 3), (1,) * 3, (4,) * 3, (4,) * 3)
        d2 = V.conv_desc((2, 256) + GRID, (256, 256, 3, 3, 3), (1,) * 3, (2,) * 3, (2,) * 3)
        assert lib.mmad_conv3d_stats_rows(d4, _lib.BF16) == 2 * 2 * 3     # residue-class
        assert lib.mmad_conv3d_stats_rows(d2, _lib.BF16) == 2 * 6
        out = m.general_step(batch, 0, "train")
        out["loss"].backward()
        torch.cuda.synchronize()
    finally:
        lib.mmad_set_kernel_variant(b"lattice", prev[0])
        lib.mmad_set_kernel_variant(b"lattice8", prev[1])
    got = out["outputs"].detach().cpu().numpy()
    ref = g["train_logits"]
    bound = 3e-2 * max(1.0, np.abs(ref).max())
    err = np.abs(got - ref).max()
    assert err <= bound, f"bf16 logits {err:.3e} from the reference (bound {bound:.3e})"
    top2 = np.sort(ref, axis=1)[:, ::-1]
    decided = (top2[:, 0] - top2[:, 1]) > 2 * bound
    assert (got.argmax(1)[decided] == ref.argmax(1)[decided]).all()
    for p in m.parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all()
