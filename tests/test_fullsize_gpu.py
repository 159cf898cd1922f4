"""BASELINE-size correctness: the exact kernel variants the bench launches.

Kernel variants are chosen by problem size (tile shape by grid fill, the patch-resident
kernel by channel count, split-K counts by voxel count, the stem's row layout by output
width), so the small per-op cases of test_kernels_gpu.py do not reach the ones config 2
(ResNet-10, 1x128^3, batch 8, bf16) runs.  Every conv layer of that step runs here at its
real shape through ``volume_ops.conv3d`` (the model's own dispatch), forward + dX + dW,
against a plain PyTorch fp32 reference of the same conv on the GPU (im2col + matmul, on the
bf16-rounded operands, so the only differences are accumulation order and the kernel's
final bf16 rounding).  Tolerances, per element:
  bf16 outputs (y, dX): |err| <= 2^-7 |ref| + 1e-3 max|ref|   (one bf16 rounding + fp32 sums)
  fp32 weight gradients: |err| <= 1e-3 |ref| + 1e-4 max|ref|
Plus the whole config-2 step in bf16 against the golden-pinned fp32 HIP path on the same
weights and volumes, and config 5's 160^3 stem (output width 80: the wide-row stem path)."""
import pytest
import torch
import torch.nn.functional as F

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last_3d
BF = torch.bfloat16


def _ref_conv(x, w, s, p, d):
    """fp32 conv3d as im2col + matmul (autograd gives dX and dW)."""
    n, c = x.shape[:2]
    co, k = w.shape[0], w.shape[2]
    span = (k - 1) * d + 1
    u = F.pad(x, (p,) * 6)
    for dim in (2, 3, 4):
        u = u.unfold(dim, span, s)
    u = u[..., ::d, ::d, ::d]                             # N,C,Do,Ho,Wo,k,k,k
    do, ho, wo = u.shape[2:5]
    cols = u.permute(0, 2, 3, 4, 1, 5, 6, 7).reshape(n * do * ho * wo, c * k ** 3)
    y = cols @ w.reshape(co, -1).t()
    return y.view(n, do, ho, wo, co).permute(0, 4, 1, 2, 3)


def _check(got, ref, rel, absf, name):
    got = got.detach().float()
    ref = ref.detach().float()
    scale = ref.abs().max().item()
    err = (got - ref).abs()
    bound = rel * ref.abs() + absf * scale
    bad = (err > bound).sum().item()
    assert bad == 0, (f"{name}: {bad} elements out of bound; max|err| {err.max().item():.3e}, "
                      f"max|ref| {scale:.3e}")


def _gen(seed):
    return torch.Generator(device=DEV).manual_seed(seed)


# (name, N, Ci, S_in, Co, k, stride, pad, dil): ResNet-10 at 1x128^3, batch 8
LAYERS = [
    ("layer1.convX", 8, 64, 32, 64, 3, 1, 1, 1),
    ("layer2.0.conv1", 8, 64, 32, 128, 3, 2, 1, 1),
    ("layer2.0.downsample", 8, 64, 32, 128, 1, 2, 0, 1),
    ("layer2.0.conv2", 8, 128, 16, 128, 3, 1, 1, 1),
    ("layer3.0.conv1", 8, 128, 16, 256, 3, 1, 2, 2),
    ("layer3.0.downsample", 8, 128, 16, 256, 1, 1, 0, 1),
    ("layer3.0.conv2", 8, 256, 16, 256, 3, 1, 2, 2),
    ("layer4.0.conv1", 8, 256, 16, 512, 3, 1, 4, 4),
    ("layer4.0.downsample", 8, 256, 16, 512, 1, 1, 0, 1),
    ("layer4.0.conv2", 8, 512, 16, 512, 3, 1, 4, 4),
]


# BASELINE config 5's 20^3 layers (160^3 input, batch 8): the implicit-GEMM route and, from
# M = 49152 output voxels on, the 256 x 256 weight-gradient tiles
LAYERS5 = [
    ("c5.layer3.conv2", 8, 256, 20, 256, 3, 1, 2, 2),
    ("c5.layer4.conv2", 8, 512, 20, 512, 3, 1, 4, 4),
]


@pytest.mark.parametrize("case", LAYERS + LAYERS5, ids=[c[0] for c in LAYERS + LAYERS5])
def test_config2_conv_layer_full_size(case):
    name, n, ci, s_in, co, k, st, p, dl = case
    g = _gen(100 + (LAYERS + LAYERS5).index(case))
    x = (torch.rand((n, ci, s_in, s_in, s_in), generator=g, device=DEV) * 2 - 1).to(BF)
    w = (torch.rand((co, ci, k, k, k), generator=g, device=DEV) * 2 - 1) * (3.0 / (ci * k ** 3)) ** 0.5
    xg = x.contiguous(memory_format=CL).requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    y, stats = V.conv3d(xg, wg, None, (st,) * 3, (p,) * 3, (dl,) * 3, BF, want_stats=True)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    y.backward(gy)
    torch.cuda.synchronize()

    xr = x.float().requires_grad_(True)
    wr = w.to(BF).float().requires_grad_(True)
    yr = _ref_conv(xr, wr, st, p, dl)
    yr.backward(gy.float())
    _check(y, yr, 2 ** -7, 1e-3, f"{name} y")
    _check(xg.grad, xr.grad, 2 ** -7, 1e-3, f"{name} dX")
    _check(wg.grad, wr.grad, 1e-3, 1e-4, f"{name} dW")
    # BN partial sums from the conv epilogue (fp32 accumulators, before the bf16 rounding)
    ysum = yr.detach().sum(dim=(0, 2, 3, 4))
    ysq = (yr.detach() ** 2).sum(dim=(0, 2, 3, 4))
    absum = yr.detach().abs().sum(dim=(0, 2, 3, 4))
    assert ((stats[:, 0].sum(0) - ysum).abs() <= 1e-4 * absum + 1e-6).all(), name
    assert ((stats[:, 1].sum(0) - ysq).abs() <= 1e-4 * ysq + 1e-6).all(), name


@pytest.mark.parametrize("n,size", [(8, 128), (2, 160)], ids=["config2_128", "config5_160"])
def test_stem_full_size(n, size):
    """conv1 7^3 / s2 / p3 on the raw f64 volume (unfold + cast on device, then the stem
    kernels): forward and dW at the bench's size (output width 64) and config 5's 160^3
    (output width 80, the stem's other row layout)."""
    g = _gen(size)
    vol = torch.rand((n, 1, size, size, size), generator=g, device=DEV, dtype=torch.float64)
    w = (torch.rand((64, 1, 7, 7, 7), generator=g, device=DEV) * 2 - 1) * (3.0 / 343) ** 0.5
    wg = w.clone().requires_grad_(True)
    y = V.conv3d(vol, wg, None, (2,) * 3, (3,) * 3, (1,) * 3, BF)
    gy = (torch.rand(y.shape, generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
    y.backward(gy)
    torch.cuda.synchronize()
    xr = vol.float().to(BF).float()
    wr = w.to(BF).float().requires_grad_(True)
    yr = _ref_conv(xr, wr, 2, 3, 1)
    yr.backward(gy.float())
    _check(y, yr, 2 ** -7, 1e-3, "stem y")
    _check(wg.grad, wr.grad, 1e-3, 1e-4, "stem dW")


def test_stem_bn_relu_pool_full_size():
    """The fused stem tail (BN(train) + ReLU + max-pool 3/2/1) at (8,64,64^3) bf16: forward
    bit-identical to the unfused batchnorm_act -> max_pool3d chain, gradients to rounding,
    running statistics equal."""
    g = _gen(77)
    y0 = ((torch.rand((8, 64, 64, 64, 64), generator=g, device=DEV) * 4 - 1.5)
          .to(BF).contiguous(memory_format=CL))

    class _BN:
        def __init__(self):
            self.weight = torch.linspace(0.5, 1.5, 64, device=DEV).requires_grad_(True)
            self.bias = torch.linspace(-0.2, 0.2, 64, device=DEV).requires_grad_(True)
            self.running_mean = torch.zeros(64, device=DEV)
            self.running_var = torch.ones(64, device=DEV)
            self.num_batches_tracked = torch.zeros((), dtype=torch.long, device=DEV)
            self.momentum, self.eps = 0.1, 1e-5
            self.training, self.track_running_stats = True, True

    a, b = _BN(), _BN()
    ya = y0.clone().requires_grad_(True)
    pa = V.max_pool3d(V.batchnorm_act(ya, a, relu=True), 3, 2, 1)
    yb = y0.clone().requires_grad_(True)
    pb = V.batchnorm_relu_maxpool(yb, b, None, 3, 2, 1)
    gp = (torch.rand(pa.shape, generator=g, device=DEV) - 0.5).to(BF).contiguous(memory_format=CL)
    pa.backward(gp)
    pb.backward(gp)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb)
    _check(yb.grad, ya.grad, 2 ** -7, 1e-3, "dy")
    # dgamma = sum g_bn * xhat, dbeta = sum g_bn over the ~2M voxels of a channel: the
    # unfused chain rounds g_bn (the scattered pool gradient) to bf16 before summing, the
    # fused backward does not, so they differ by up to 2^-9 of the summed magnitude
    yf = y0.float()
    xh = ((yf - yf.mean(dim=(0, 2, 3, 4), keepdim=True)) /
          (yf.var(dim=(0, 2, 3, 4), unbiased=False, keepdim=True) + 1e-5).sqrt())
    gabs = gp.float().abs().sum(dim=(0, 2, 3, 4))
    xmax = xh.abs().amax(dim=(0, 2, 3, 4))
    assert ((b.weight.grad - a.weight.grad).abs() <= 2 ** -8 * gabs * xmax + 1e-3).all()
    assert ((b.bias.grad - a.bias.grad).abs() <= 2 ** -8 * gabs + 1e-3).all()
    assert torch.allclose(b.running_mean, a.running_mean, rtol=1e-5, atol=1e-7)
    assert torch.allclose(b.running_var, a.running_var, rtol=1e-5, atol=1e-7)


def test_config2_step_bf16_tracks_fp32_hip_path():
    """The benched step itself (Anat_CNN ResNet-10, 8x1x128^3, weighted CE) in bf16 against
    the same model in fp32 (the path pinned to the reference's golden vectors at <= 64^3):
    logits drift, argmax wherever the fp32 top-2 margin exceeds that drift, loss, BN running
    statistics, and the direction of every weight gradient."""
    h = {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
         "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
         "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
         "reduce_factor_lr_schedule": None,
         "loss_class_weights": torch.tensor([0.2031496, 0.7968504], dtype=torch.float64)}
    torch.manual_seed(15)
    m32 = M.Anat_CNN(dict(h, precision="32"))
    m16 = M.Anat_CNN(dict(h, precision="bf16"))
    with torch.no_grad():            # live logits: the head's final ReLU passes gradient
        m32.model.conv_seg[-2].bias.fill_(1.0)
    m16.load_state_dict(m32.state_dict())
    m32, m16 = m32.to(DEV), m16.to(DEV)
    g = _gen(1000)
    batch = {"mri": torch.rand((8, 128, 128, 128), generator=g, device=DEV, dtype=torch.float64),
             "label": torch.randint(0, 2, (8,), generator=g, device=DEV)}
    outs = {}
    for key, m in (("32", m32), ("16", m16)):
        r = m.general_step(batch, 0, "train")
        r["loss"].backward()
        outs[key] = (r["outputs"].detach(), r["loss"].detach())
    torch.cuda.synchronize()
    l32, l16 = outs["32"][0], outs["16"][0]
    assert torch.isfinite(l16).all()
    scale = max(1.0, l32.abs().max().item())
    drift = (l16 - l32).abs().max().item()
    assert drift <= 3e-2 * scale, f"bf16 logits drift {drift:.3e} (scale {scale:.3e})"
    top2 = l32.topk(2, dim=1).values
    decided = (top2[:, 0] - top2[:, 1]) > 2 * drift
    assert torch.equal(l16.argmax(1)[decided], l32.argmax(1)[decided])
    assert abs(outs["16"][1].item() - outs["32"][1].item()) <= 3e-2 * max(1.0, abs(outs["32"][1].item()))
    b32, b16 = dict(m32.named_buffers()), dict(m16.named_buffers())
    for k, v in b32.items():
        if "running" in k:
            err = (b16[k] - v).abs().max().item()
            assert err <= 2e-2 * max(1e-3, v.abs().max().item()), (k, err)
    # gradient direction per tensor.  bf16 rounding noise compounds along the backward
    # chain (measured on MI355X: cosine 0.998 at layer4, 0.99 at layer3, 0.97-0.985 at
    # layer1/2, 0.95 at the stem conv), and the stem sits in front of the 3^3 max-pool,
    # where rounding its output to bf16 reorders near-equal window values and routes a few
    # % of the pooled gradients to other voxels.  A wrong kernel shows as a break in that
    # smooth decay, not as a slightly lower cosine.
    p16 = dict(m16.named_parameters())
    cosines = {}
    for k, p in m32.named_parameters():
        if p.grad is None or not p.grad.any():
            continue
        a, b = p.grad.flatten().double(), p16[k].grad.flatten().double()
        cosines[k] = (a @ b / (a.norm() * b.norm())).item()
    assert len(cosines) > 20
    for k, cos in cosines.items():
        print(f"cos {k} {cos:.5f}")
    floor = {"model.conv1": 0.9, "model.bn1": 0.9, "model.layer1": 0.95, "model.layer2": 0.95}
    for k, cos in cosines.items():
        lim = next((v for pre, v in floor.items() if k.startswith(pre + ".")), 0.98)
        assert cos > lim, (k, cos)


def test_layer4_eval_fused_conv_bn_res_relu_full_size():
    """Eval-mode fused layer4 conv (BN folded into the weights, residual + ReLU in the
    epilogue: the residue-class kernel's eval epilogue at 8 x 512 x 16^3) against the
    unfused conv -> BN(running stats) + residual + ReLU on the same bf16 operands."""
    from multimodal_alzheimer_amd import layers as Lyr
    torch.manual_seed(21)
    conv = Lyr.Conv3d(512, 512, 3, padding=4, dilation=4, bias=False).to(DEV)
    conv.compute_dtype = BF
    bn = torch.nn.BatchNorm3d(512).to(DEV)
    with torch.no_grad():
        bn.running_mean.uniform_(-0.2, 0.2)
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.3, 0.3)
    bn.eval()
    g = _gen(22)
    x = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    res = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF) \
        .contiguous(memory_format=CL)
    with torch.no_grad():
        y = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
        assert y is not None
        # the fold as mmad_bn_fold computes it (1/sqrt in f64, products in fp32)
        inv = (1.0 / (bn.running_var.double() + bn.eps).sqrt()).float()
        scale = bn.weight * inv
        shift = bn.bias - bn.running_mean * bn.weight * inv
        wf = (conv.weight * scale.view(-1, 1, 1, 1, 1)).to(BF).float()
        pre = _ref_conv(x.float(), wf, 1, 4, 4) + shift.view(1, -1, 1, 1, 1)
        ref = torch.relu(pre + res.float())
    # the epilogue rounds conv + BN shift to bf16, adds the bf16 residual and rounds the sum
    # again: two roundings, each up to 2^-8 of its own value (bf16 unit roundoff)
    err = (y.float() - ref).abs()
    bound = 2 ** -8 * (pre.abs() + (pre + res.float()).abs()) + 1e-3 * ref.abs().max()
    assert (err <= bound).all(), f"fused eval conv: max|err| {err.max().item():.3e}"
