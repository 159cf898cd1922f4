"""The MedicalNet stem (conv1: 1 -> 64, 7^3, stride 2, pad 3; anat_cnn.py:29-31 and
pet_resnet_cnn.py:33-35 via MedicalNet) on rows wider than 64 output columns -- config 5's
160^3 volumes give 80 -- which the dedicated stem kernels (csrc/stem.hip) split into equal
column tiles, one per block (before round 5 these went to the row-gather implicit GEMM at
~9 % of peak).  Forward output within one bf16 rounding of a plain fp32 PyTorch conv of the
same bf16 operands, BN partial-sum totals within fp32 rounding of its sums, weight gradient
within 1e-3 |ref| + 1e-4 sum |gY| |U| of a float64 one; the route is checked through the
profiler's kernel names."""
import pytest
import torch

from multimodal_alzheimer_amd import _lib as L
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
BF = torch.bfloat16

# (input shape): wo 80 (2 tiles of 40, config 5's width), 100 (2 x 50), 150 (3 x 50)
CASES = [(2, 1, 20, 18, 160), (1, 1, 12, 10, 200), (1, 1, 9, 8, 300)]


def _kernel_names(fn):
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        fn()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    return names or None


@pytest.mark.parametrize("shape", CASES, ids=["w80", "w100", "w150"])
def test_stem_column_tiles_match_fp32(shape):
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    x = torch.rand(shape, generator=g, device="cuda", dtype=torch.float64)
    w = (torch.rand((64, 1, 7, 7, 7), generator=g, device="cuda") * 2 - 1) * 0.05
    d = V.conv_desc(tuple(shape), tuple(w.shape), (2,) * 3, (3,) * 3, (1,) * 3)
    dt, in_dt = L.dtype_code(BF), L.dtype_code(torch.float64)
    assert d.wo > 64
    wp = V.pack_weight(d, dt, w, BF, False)
    rows = lib.mmad_conv3d_stats_rows(d, dt)
    y = V._empty_vol(d.n, 64, d.do_, d.ho, d.wo, BF, x.device)
    st = torch.empty((rows, 2, 64), device="cuda")
    u = torch.empty(lib.mmad_conv_unfolded_elems(d), dtype=BF, device="cuda")
    gy = ((torch.rand(y.shape, generator=g, device="cuda") * 2 - 1).to(BF)
          .contiguous(memory_format=torch.channels_last_3d))
    ws = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, dt) + 3) // 4, device="cuda")
    dw = torch.empty(w.shape, device="cuda")

    def run():
        L.call("mmad_conv_unfold_input", d, in_dt, L.ptr(x), dt, L.ptr(u), L.stream())
        L.call("mmad_conv3d_fwd", d, dt, L.ptr(u), L.ptr(wp), None, L.ptr(y), L.ptr(st),
               L.stream())
        L.call("mmad_conv3d_wgrad", d, dt, L.ptr(u), L.ptr(gy), L.ptr(dw), None, L.ptr(ws),
               L.stream())
    names = _kernel_names(run)
    if names is not None:
        assert any("stem_fwdq_kernel" in k for k in names), "forward not on the stem kernel"
        assert any("stem_wgrad2_kernel" in k for k in names), "wgrad not on the stem kernel"
    xb = x.float().to(BF).float()
    wb = w.to(BF).float()
    yr = torch.nn.functional.conv3d(xb, wb, None, 2, 3)
    err = (y.float() - yr).abs()
    assert (err <= 2 ** -7 * yr.abs() + 1e-3 * yr.abs().max()).all(), err.max().item()
    yd = yr.double()
    tot = st.sum(0).double()
    ref = torch.stack((yd.sum(dim=(0, 2, 3, 4)), (yd * yd).sum(dim=(0, 2, 3, 4))))
    mag = torch.stack((yd.abs().sum(dim=(0, 2, 3, 4)), (yd * yd).sum(dim=(0, 2, 3, 4))))
    assert ((tot - ref).abs() <= 1e-3 * mag + 1e-6).all(), "BN partial sums"
    xd, gd = xb.double(), gy.double()
    wr = torch.nn.grad.conv3d_weight(xd, w.shape, gd, 2, 3)
    mg = torch.nn.grad.conv3d_weight(xd.abs(), w.shape, gd.abs(), 2, 3)
    e = (dw.double() - wr).abs()
    assert (e <= 1e-3 * wr.abs() + 1e-4 * mg).all(), e.max().item()
