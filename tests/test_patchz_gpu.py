"""Persistent z-walking layer1 conv (csrc/patchz.hip) at BASELINE config 2's layer1 shape
(8 x 64 x 32^3): it accumulates every output element in the same K order as the per-box
patch conv (csrc/patchconv.hip) it replaces (tap-major, 32-channel halves), so forward
outputs and input gradients must be bit-identical to it, and within one bf16 rounding of a
plain fp32 PyTorch conv of the same bf16 operands (|err| <= 2^-7 |ref| + 1e-3 max|ref|).
The BN partial sums are grouped into different rows (4x8x8 boxes instead of 2x8x8), so their
per-channel totals agree to fp32 rounding.  Also: the eval-mode epilogue (residual + ReLU),
and grids whose columns need several z segments (mode 2 at batch 1, a 16^3 grid).  (The
round-4 weight-stationary form measured no faster and was removed in round 5.)"""
import pytest
import torch

from multimodal_alzheimer_amd import _lib
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d
BF = torch.bfloat16


def _variant(name, v):
    return _lib.load().mmad_set_kernel_variant(name.encode(), v)


def _conv(x, w):
    xg = x.clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y, stats = V.conv3d(xg, wg, None, (1,) * 3, (1,) * 3, (1,) * 3, BF, want_stats=True)
    g = torch.Generator(device=DEV).manual_seed(19)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    y.backward(gy)
    torch.cuda.synchronize()
    return y.detach(), stats.sum(0), xg.grad, wg.grad, stats.shape[0], gy


def _ref_conv(x, w, gy):
    from tests.test_fullsize_gpu import _ref_conv as rc
    xr = x.float().requires_grad_(True)
    wr = w.to(BF).float().requires_grad_(True)
    yr = rc(xr, wr, 1, 1, 1)
    yr.backward(gy.float())
    return yr.detach(), xr.grad


def _close(got, ref, name, rel=2 ** -7, absf=1e-3):
    got, ref = got.float(), ref.float()
    err = (got - ref).abs()
    bound = rel * ref.abs() + absf * ref.abs().max()
    bad = int((err > bound).sum())
    assert bad == 0, f"{name}: {bad} beyond bound, max|err| {err.max().item():.3e}"


CASES = [(8, 32, 1), (1, 32, 2), (2, 16, 2)]
IDS = ["config2_layer1", "batch1_segments", "grid16"]


@pytest.mark.parametrize("n,size,mode", CASES, ids=IDS)
def test_patchz_matches_patch_and_fp32(n, size, mode):
    g = torch.Generator(device=DEV).manual_seed(size + n)
    x = (torch.rand((n, 64, size, size, size), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    w = (torch.rand((64, 64, 3, 3, 3), generator=g, device=DEV) * 2 - 1) * (3.0 / (64 * 27)) ** 0.5
    prev = _variant("patchz", 0)
    try:
        ref = _conv(x, w)
        _variant("patchz", mode)
        got = _conv(x, w)
    finally:
        _variant("patchz", prev)
    assert got[4] == n * (size // 4) * (size // 8) ** 2, "not routed to the z-walking kernel"
    assert torch.equal(got[3], ref[3]), "weight gradient differs (same wgrad kernel)"
    assert torch.equal(got[0], ref[0]), "forward differs"
    assert torch.equal(got[2], ref[2]), "input gradient differs"
    yr, dxr = _ref_conv(x, w, got[5])
    _close(got[0], yr, "forward vs fp32")
    _close(got[2], dxr, "input gradient vs fp32")
    y = ref[0].float()
    mag = torch.stack((y.abs().sum(dim=(0, 2, 3, 4)), (y * y).sum(dim=(0, 2, 3, 4))))
    assert ((got[1] - ref[1]).abs() <= 1e-5 * mag + 1e-6).all(), "BN partial-sum totals differ"


def test_patchz_eval_epilogue_residual_relu():
    from multimodal_alzheimer_amd import layers as Lyr
    torch.manual_seed(7)
    conv = Lyr.Conv3d(64, 64, 3, padding=1, bias=False).to(DEV)
    conv.compute_dtype = BF
    bn = torch.nn.BatchNorm3d(64).to(DEV).eval()
    with torch.no_grad():
        bn.running_var.uniform_(0.5, 2.0)
        bn.bias.uniform_(-0.3, 0.3)
    g = torch.Generator(device=DEV).manual_seed(8)
    x = (torch.rand((8, 64, 32, 32, 32), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    res = (torch.rand((8, 64, 32, 32, 32), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    prev = _variant("patchz", 0)
    try:
        with torch.no_grad():
            ref = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
            _variant("patchz", 1)
            got = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
        torch.cuda.synchronize()
    finally:
        _variant("patchz", prev)
    assert torch.equal(got, ref)
