"""BN-backward partial sums from the consumer's dgrad epilogue (volume_ops BNSUM,
mmad_conv3d_dgrad_bnsum; csrc/bnsum.h): a MedicalNet BasicBlock's bn1 -> relu -> conv2 in
bf16, backward with the fused epilogue against the column-sum pass it replaces
(mmad_bn_relu_bwd_reduce, MMAD_BNSUM=0 path):

  * the fused route actually runs (mmad_conv3d_dgrad_bnsum called, no bn_relu_bwd_reduce);
  * forward outputs and conv2's input gradient are bit-identical (the same dgrad kernel);
  * bn1's dgamma / dbeta (the sums themselves, summed over tiles instead of row ranges)
    within fp32 reduction-order rounding, and everything downstream of them (bn1's input
    gradient, conv1's weight gradient, the block input gradient) within one bf16 rounding;
  * the partial rows themselves against a float64 evaluation of the same masked sums.
"""
import pytest
import torch

from multimodal_alzheimer_amd import _lib as L
from multimodal_alzheimer_amd import layers as Lyr
from multimodal_alzheimer_amd import medicalnet
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d

# (planes, grid, dilation, batch, kernel-variant overrides): the routes with the epilogue
CASES = {
    "layer4_lattice_zp": (512, 16, 4, 2, {"lattice": 2, "lattice_zp": 2}),
    "layer3_lattice8": (256, 16, 2, 2, {"lattice8": 2}),
    "layer2_patch": (128, 16, 1, 2, {}),
}


def _run(block, x, gy, bnsum, calls):
    prev = V.BNSUM
    V.BNSUM = bnsum
    V.clear_twins()
    for p in block.parameters():
        p.grad = None
    xg = x.clone().requires_grad_(True)
    real = L.call

    def spy(name, *a):
        calls.append(name)
        return real(name, *a)

    L.call = spy
    try:
        out = block(xg)
        out.backward(gy)
    finally:
        L.call = real
        V.BNSUM = prev
    torch.cuda.synchronize()
    return out.detach().clone(), xg.grad.clone(), {k: p.grad.clone()
                                                   for k, p in block.named_parameters()}


@pytest.mark.parametrize("name", list(CASES))
def test_fused_bn_sums_match_column_sum_pass(name):
    planes, s, dil, n, variants = CASES[name]
    lib = L.load()
    prev = {k: lib.mmad_set_kernel_variant(k.encode(), v) for k, v in variants.items()}
    try:
        torch.manual_seed(1)
        block = medicalnet.BasicBlock(planes, planes, dilation=dil).to(DEV)
        Lyr.set_compute_dtype(block, torch.bfloat16)
        block.train()
        g = torch.Generator(device=DEV).manual_seed(2)
        x = (torch.randn((n, planes, s, s, s), generator=g, device=DEV)).to(torch.bfloat16) \
            .contiguous(memory_format=CL)
        gy = (torch.randn((n, planes, s, s, s), generator=g, device=DEV)).to(torch.bfloat16) \
            .contiguous(memory_format=CL)
        sd = {k: v.clone() for k, v in block.state_dict().items()}
        c_ref, c_new = [], []
        o_ref, dx_ref, g_ref = _run(block, x, gy, False, c_ref)
        block.load_state_dict(sd)
        o_new, dx_new, g_new = _run(block, x, gy, True, c_new)
    finally:
        for k, v in prev.items():
            lib.mmad_set_kernel_variant(k.encode(), v)
    assert "mmad_conv3d_dgrad_bnsum" in c_new and "mmad_bn_relu_bwd_reduce" not in c_new
    assert "mmad_bn_relu_bwd_reduce" in c_ref
    assert torch.equal(o_new, o_ref)
    for k in ("bn1.weight", "bn1.bias"):
        ref = g_ref[k].double()
        err = (g_new[k].double() - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item() + 1e-6, (k, err)
    for k, ref in list(g_ref.items()) + [("x", dx_ref)]:
        got = dx_new if k == "x" else g_new[k]
        ref = ref.double()
        err = (got.double() - ref).abs()
        tol = 2 ** -7 * ref.abs() + 2e-3 * ref.abs().max()
        assert (err <= tol).all(), (k, err.max().item(), ref.abs().max().item())


@pytest.mark.parametrize("name", list(CASES))
def test_bnsum_partial_rows_vs_float64(name):
    """the partial rows of one dgrad launch, summed, against float64 masked sums over the
    same bf16 gradient and BN input; dX bit-identical to the plain dgrad"""
    planes, s, dil, n, variants = CASES[name]
    lib = L.load()
    prev = {k: lib.mmad_set_kernel_variant(k.encode(), v) for k, v in variants.items()}
    try:
        g = torch.Generator(device=DEV).manual_seed(3)
        mk = lambda: torch.randn((n, planes, s, s, s), generator=g, device=DEV).to(  # noqa
            torch.bfloat16).contiguous(memory_format=CL)
        gy, y = mk(), mk()
        w = torch.randn((planes, planes, 3, 3, 3), generator=g, device=DEV) * 0.02
        sc = torch.rand(planes, generator=g, device=DEV) + 0.5
        sh = torch.randn(planes, generator=g, device=DEV) * 0.3
        mu = torch.randn(planes, generator=g, device=DEV) * 0.1
        ist = torch.rand(planes, generator=g, device=DEV) + 0.5
        d = V.conv_desc((n, planes, s, s, s), tuple(w.shape), (1,) * 3, (dil,) * 3, (dil,) * 3)
        dt = L.dtype_code(torch.bfloat16)
        wpt = V.pack_weight(d, dt, w, torch.bfloat16, True)
        rows = lib.mmad_conv3d_dgrad_bnsum_rows(d, dt)
        assert rows > 0
        dx = torch.empty_like(y)
        parts = torch.empty((rows, 2, planes), device=DEV)
        L.call("mmad_conv3d_dgrad_bnsum", d, dt, L.ptr(gy), L.ptr(wpt), L.ptr(dx), L.ptr(y),
               L.ptr(sc), L.ptr(sh), L.ptr(mu), L.ptr(ist), L.ptr(parts), L.stream())
        dx2 = torch.empty_like(y)
        L.call("mmad_conv3d_dgrad", d, dt, L.ptr(gy), L.ptr(wpt), L.ptr(dx2), L.stream())
        torch.cuda.synchronize()
    finally:
        for k, v in prev.items():
            lib.mmad_set_kernel_variant(k.encode(), v)
    assert torch.equal(dx, dx2)
    gd = dx.double().permute(0, 2, 3, 4, 1).reshape(-1, planes)
    yd = y.double().permute(0, 2, 3, 4, 1).reshape(-1, planes)
    mask = torch.addcmul(sh.double(), yd, sc.double()) > 0
    gm = torch.where(mask, gd, torch.zeros_like(gd))
    S = gm.sum(0)
    Q = (gm * ((yd - mu.double()) * ist.double())).sum(0)
    got = parts.double().sum(0)
    for ref, row in ((S, got[0]), (Q, got[1])):
        mag = gm.abs().sum(0) * (1 + (yd - mu.double()).abs().max() * ist.double())
        assert ((row - ref).abs() <= 1e-5 * mag + 1e-6).all()
