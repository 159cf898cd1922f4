"""Plane-pair residue-class conv (csrc/latticezp.hip) against the one-plane form
(csrc/latticeconv.hip) it replaces for layer4 at BASELINE config 2's size.

Both accumulate every output element over the same K order (channel chunk, kz, ky, kx,
padding taps skipped), so the conv outputs must be bit-identical; the BN partial sums are
grouped into different tile rows, so their per-channel totals agree to fp32 rounding.
Covered: layer4.0.conv1 (256 -> 512) and conv2 (512 -> 512) forward (128-channel tiles) and
their input gradients (512 -> 256 runs the 64-channel-tile variant), plus the eval-mode
epilogue (residual + ReLU).  The plain fp32-torch checks of the same layers are in
tests/test_fullsize_gpu.py."""
import pytest
import torch

from multimodal_alzheimer_amd import _lib
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d
BF = torch.bfloat16


def _variant(v):
    return _lib.load().mmad_set_kernel_variant(b"lattice_zp", v)


def _conv(x, w, res=None):
    xg = x.clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y, stats = V.conv3d(xg, wg, None, (1,) * 3, (4,) * 3, (4,) * 3, BF, want_stats=True)
    g = torch.Generator(device=DEV).manual_seed(9)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    y.backward(gy)
    torch.cuda.synchronize()
    return y.detach(), stats.sum(0), xg.grad, wg.grad


@pytest.mark.parametrize("ci,co", [(256, 512), (512, 512)], ids=["l4c1", "l4c2"])
def test_plane_pair_equals_one_plane(ci, co):
    g = torch.Generator(device=DEV).manual_seed(ci + co)
    x = (torch.rand((8, ci, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    w = (torch.rand((co, ci, 3, 3, 3), generator=g, device=DEV) * 2 - 1) * (3.0 / (ci * 27)) ** 0.5
    prev = _variant(0)
    try:
        ref = _conv(x, w)
        assert _variant(1) == 0
        got = _conv(x, w)
    finally:
        _variant(prev)
    assert torch.equal(got[0], ref[0]), "forward differs"
    assert torch.equal(got[2], ref[2]), "input gradient differs"
    assert torch.equal(got[3], ref[3]), "weight gradient differs"
    # the totals of the partial sums, grouped into different tile rows: equal to fp32
    # rounding of the summed magnitudes (the per-channel sum itself may cancel to ~0)
    y = ref[0].float()
    mag = torch.stack((y.abs().sum(dim=(0, 2, 3, 4)), (y * y).sum(dim=(0, 2, 3, 4))))
    assert ((got[1] - ref[1]).abs() <= 1e-5 * mag + 1e-6).all(), "BN partial-sum totals differ"


def test_plane_pair_eval_epilogue_residual_relu():
    """conv_bn_act_eval's fused epilogue (residual + ReLU) on the plane-pair kernel equals
    the one-plane kernel's bit for bit."""
    from multimodal_alzheimer_amd import layers as Lyr
    torch.manual_seed(5)
    conv = Lyr.Conv3d(512, 512, 3, padding=4, dilation=4, bias=False).to(DEV)
    conv.compute_dtype = BF
    bn = torch.nn.BatchNorm3d(512).to(DEV).eval()
    with torch.no_grad():
        bn.running_var.uniform_(0.5, 2.0)
        bn.bias.uniform_(-0.3, 0.3)
    g = torch.Generator(device=DEV).manual_seed(6)
    x = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    res = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    prev = _variant(0)
    try:
        with torch.no_grad():
            ref = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
            _variant(1)
            got = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
        torch.cuda.synchronize()
    finally:
        _variant(prev)
    assert torch.equal(got, ref)
