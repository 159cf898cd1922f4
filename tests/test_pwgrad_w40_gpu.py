"""The patch-resident weight gradient on 40-wide volumes (csrc/pwgrad.hip, W40 form, round 5):
config 5's layer1 convs (64 -> 64, dense 3^3, padding 1, at 40^3 for a 160^3 input;
pet_resnet_cnn.py:12-138 / anat_cnn.py:29-31 via MedicalNet), whose rows are 5 segments of 8
voxels and whose K steps run across rows.  Weight gradient against a float64 one of the same
bf16 operands (1e-3 |ref| + 1e-4 sum |gY| |X|, the bar of every weight-gradient kernel); the
route is checked through the profiler's kernel names."""
import pytest
import torch

from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d
BF = torch.bfloat16

# (x shape, output channels): config 5's layer1 at batch 2, a shallow ragged volume, and a
# 128-output-channel case
CASES = [((2, 64, 40, 40, 40), 64), ((1, 64, 6, 16, 40), 64), ((1, 64, 8, 8, 40), 128)]


def _names(fn):
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    return names or None


@pytest.mark.parametrize("xs,co", CASES, ids=["layer1_b2", "ragged", "co128"])
def test_w40_wgrad_vs_float64(xs, co):
    g = torch.Generator(device=DEV).manual_seed(xs[2] * 7 + co)
    x = (torch.rand(xs, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    w = (torch.rand((co, xs[1], 3, 3, 3), generator=g, device=DEV) * 2 - 1) * \
        (3.0 / (xs[1] * 27)) ** 0.5
    wg = w.clone().requires_grad_(True)
    y = V.conv3d(x, wg, None, (1,) * 3, (1,) * 3, (1,) * 3, BF)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    names = _names(lambda: y.backward(gy))
    if names is not None:
        assert any("pwgrad_kernel<3>" in k for k in names), "not routed to the W40 form"
    xd, gd = x.double(), gy.double()
    ref = torch.nn.grad.conv3d_weight(xd, w.shape, gd, 1, 1, 1)
    mag = torch.nn.grad.conv3d_weight(xd.abs(), w.shape, gd.abs(), 1, 1, 1)
    err = (wg.grad.double() - ref).abs()
    assert (err <= 1e-3 * ref.abs() + 1e-4 * mag).all(), f"max err {err.max().item():.3e}"
