"""Per-kernel parity on the MI355X: every HIP op against a torch-CPU float64 reference of
the same op on the same seeded inputs (fp32 mode to ~1e-5, bf16 mode to bf16 rounding).
All calls go through libmmad_hip.so (no torch fallback exists)."""
import pytest
import torch
import torch.nn.functional as F

from multimodal_alzheimer_amd import _lib, head_ops, volume_ops as V

pytestmark = pytest.mark.gpu
CL = torch.channels_last_3d
DEV = "cuda"


def rnd(*shape, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1) * scale


def to_vol(x, dtype):
    return x.to(DEV, dtype).contiguous(memory_format=CL)


def close(got, ref, rtol, name=""):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item() + 1e-12
    assert err <= rtol * scale, f"{name}: max|err| {err:.3e} > {rtol:.1e} * {scale:.3e}"


# (N, Ci, D, H, W, Co, k, stride, pad, dil, bias)
CONV_CASES = [
    (2, 1, 20, 18, 22, 64, 7, 2, 3, 1, False),     # MedicalNet stem (unfolded path)
    (2, 64, 8, 10, 6, 64, 3, 1, 1, 1, False),      # layer1
    (2, 64, 9, 8, 10, 128, 3, 2, 1, 1, False),     # layer2.0.conv1 (stride 2)
    (2, 64, 16, 16, 16, 128, 3, 2, 1, 1, False),   # stride 2: sub-patch fwd and all-class dgrad
    (1, 64, 8, 16, 16, 64, 3, 2, 1, 1, True),      # stride 2, sub-patch fwd (64 co), bias
    (1, 64, 4, 32, 16, 256, 3, 2, 1, 1, True),     # stride 2, sub-patch fwd: 2 co tiles, bias
    (2, 128, 6, 9, 10, 128, 3, 1, 1, 1, False),    # layer2 conv2 (patch kernel, 2 ci chunks)
    (1, 64, 13, 17, 9, 128, 3, 1, 1, 1, True),     # ragged boxes + bias (patch kernel)
    (2, 128, 6, 7, 5, 256, 3, 1, 2, 2, False),     # layer3 (dilation 2)
    (1, 128, 16, 16, 16, 256, 3, 1, 2, 2, False),  # layer3 at 16^3: residue-class patch wgrad
    (2, 64, 16, 16, 16, 64, 3, 1, 2, 2, True),     # same, 2 ci chunks, one co tile, bias
    (1, 256, 6, 6, 6, 512, 3, 1, 4, 4, False),     # layer4 (dilation 4)
    (2, 64, 9, 8, 10, 128, 1, 2, 0, 1, False),     # shortcut B, stride 2
    (2, 64, 16, 16, 16, 128, 1, 2, 0, 1, False),   # stride 2, pointwise GEMM fwd / cell dgrad
    (1, 64, 15, 16, 31, 128, 1, 2, 0, 1, True),    # same, odd input extents (clipped cells)
    (2, 128, 5, 6, 7, 256, 1, 1, 0, 1, False),     # shortcut B, stride 1
    (2, 128, 8, 8, 8, 256, 1, 1, 0, 1, False),     # shortcut B, stride 1: pointwise GEMM fwd
    (1, 256, 8, 4, 8, 512, 1, 1, 0, 1, True),      # pointwise GEMM fwd: 2 column tiles, bias
    (2, 1, 12, 11, 13, 8, 5, 1, 2, 1, True),       # Small_PET_CNN conv 1 (k5 'same')
    (2, 1, 9, 10, 8, 16, 7, 1, 3, 1, True),        # Small_PET_CNN conv 1 (k7 'same')
    (2, 8, 10, 9, 11, 16, 5, 1, 2, 1, True),       # Small_PET_CNN conv 2
    (2, 32, 6, 5, 7, 64, 3, 1, 1, 1, True),        # Small_PET_CNN conv 4
    (1, 32, 4, 8, 32, 64, 3, 1, 1, 1, False),      # 32-wide: patch wgrad, one split
    (2, 128, 8, 16, 16, 128, 3, 1, 1, 1, False),   # 16-wide: patch wgrad (2-row K steps)
    (1, 64, 6, 16, 16, 64, 3, 1, 1, 1, True),      # 16-wide: one z split of 6 planes, bias
    (2, 64, 6, 16, 32, 128, 3, 1, 1, 1, True),     # 32-wide: patch wgrad, 2 co tiles, bias
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES, ids=lambda c: f"ci{c[1]}co{c[5]}k{c[6]}s{c[7]}d{c[9]}")
def test_conv3d_fwd_bwd(case, dtype):
    n, ci, d, h, w, co, k, s, p, dl, has_bias = case
    x = rnd(n, ci, d, h, w, seed=1)
    wt = rnd(co, ci, k, k, k, seed=2, scale=(3.0 / (ci * k ** 3)) ** 0.5)
    b = rnd(co, seed=3) if has_bias else None
    if dtype == torch.bfloat16:          # reference on the bf16-rounded operands
        x = x.to(torch.bfloat16).double()
        wt = wt.float().to(torch.bfloat16).double()
    xr = x.clone().requires_grad_(ci > 1)
    wr = wt.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True) if has_bias else None
    yr = F.conv3d(xr, wr, br, s, p, dl)
    gy = rnd(*yr.shape, seed=4)
    if dtype == torch.bfloat16:
        gy = gy.to(torch.bfloat16).double()
    yr.backward(gy)

    xg = (x.to(DEV, torch.float32) if ci == 1 else to_vol(x, dtype)).requires_grad_(ci > 1)
    wg = wt.float().to(DEV).requires_grad_(True)
    bg = b.float().to(DEV).requires_grad_(True) if has_bias else None
    y, stats = V.conv3d(xg, wg, bg, (s,) * 3, (p,) * 3, (dl,) * 3, dtype, want_stats=True)
    assert y.is_contiguous(memory_format=CL) and y.dtype == dtype
    y.backward(to_vol(gy, dtype))
    tol = 2e-5 if dtype == torch.float32 else 1.2e-2
    close(y, yr, tol, "y")
    ysum = yr.detach().sum(dim=(0, 2, 3, 4))
    ysq = (yr.detach() ** 2).sum(dim=(0, 2, 3, 4))
    close(stats[:, 0].sum(0), ysum, 1e-4 if dtype == torch.float32 else 2e-2, "stats.sum")
    close(stats[:, 1].sum(0), ysq, 1e-4 if dtype == torch.float32 else 2e-2, "stats.sumsq")
    gtol = 3e-5 if dtype == torch.float32 else 2e-2
    close(wg.grad, wr.grad, gtol, "dw")
    if has_bias:
        close(bg.grad, br.grad, gtol, "db")
    if ci > 1:
        close(xg.grad, xr.grad, gtol, "dx")


def test_conv_large_k_split():
    """wgrad split-K path with many voxels (M >> tile) and Co = 64."""
    n, ci, co = 2, 64, 64
    x = rnd(n, ci, 16, 16, 16, seed=5)
    wt = rnd(co, ci, 3, 3, 3, seed=6, scale=0.05)
    xr = x.clone().requires_grad_(True)
    wr = wt.clone().requires_grad_(True)
    yr = F.conv3d(xr, wr, None, 1, 1, 1)
    gy = rnd(*yr.shape, seed=7)
    yr.backward(gy)
    xg = to_vol(x, torch.float32).requires_grad_(True)
    wg = wt.float().to(DEV).requires_grad_(True)
    y = V.conv3d(xg, wg, None, (1,) * 3, (1,) * 3, (1,) * 3, torch.float32)
    y.backward(to_vol(gy, torch.float32))
    close(y, yr, 2e-5, "y")
    close(wg.grad, wr.grad, 3e-5, "dw")
    close(xg.grad, xr.grad, 3e-5, "dx")


class _BN:
    def __init__(self, c, seed):
        self.weight = (1 + 0.3 * rnd(c, seed=seed)).float().to(DEV).requires_grad_(True)
        self.bias = (0.2 * rnd(c, seed=seed + 1)).float().to(DEV).requires_grad_(True)
        self.running_mean = (0.1 * rnd(c, seed=seed + 2)).float().to(DEV)
        self.running_var = (1 + 0.5 * rnd(c, seed=seed + 3).abs()).float().to(DEV)
        self.num_batches_tracked = torch.zeros((), dtype=torch.long, device=DEV)
        self.momentum, self.eps = 0.1, 1e-5
        self.training, self.track_running_stats = True, True


def _ref_bn(x, bn, training):
    rm = bn.running_mean.double().cpu().clone()
    rv = bn.running_var.double().cpu().clone()
    w = bn.weight.detach().double().cpu().requires_grad_(True)
    b = bn.bias.detach().double().cpu().requires_grad_(True)
    y = F.batch_norm(x, rm, rv, w, b, training, bn.momentum, bn.eps)
    return y, w, b, rm, rv


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("mode", ["plain", "relu", "identity_res", "bn_res", "eval"])
def test_batchnorm_act(mode, dtype):
    n, c, d, h, w = 2, 64, 5, 6, 7
    y0 = rnd(n, c, d, h, w, seed=10, scale=2.0) + 0.5
    r0 = rnd(n, c, d, h, w, seed=11)
    if dtype == torch.bfloat16:
        y0, r0 = y0.to(dtype).double(), r0.to(dtype).double()
    training = mode != "eval"
    bn, rbn = _BN(c, 20), _BN(c, 30)
    bn.training = rbn.training = training
    yr = y0.clone().requires_grad_(True)
    rr = r0.clone().requires_grad_(True)
    out_r, w1, b1, rm1, rv1 = _ref_bn(yr, bn, training)
    if mode == "identity_res":
        out_r = out_r + rr
    if mode == "bn_res":
        o2, w2, b2, rm2, rv2 = _ref_bn(rr, rbn, training)
        out_r = out_r + o2
    if mode in ("relu", "identity_res", "bn_res"):
        out_r = torch.relu(out_r)
    g = rnd(*out_r.shape, seed=12)
    if dtype == torch.bfloat16:
        g = g.to(dtype).double()
    out_r.backward(g)

    yg = to_vol(y0, dtype).requires_grad_(True)
    rg = to_vol(r0, dtype).requires_grad_(True)
    out = V.batchnorm_act(yg, bn, relu=mode in ("relu", "identity_res", "bn_res"),
                          res=rg if mode in ("identity_res", "bn_res") else None,
                          res_bn=rbn if mode == "bn_res" else None)
    out.backward(to_vol(g, dtype))
    tol = 2e-5 if dtype == torch.float32 else 1.5e-2
    close(out, out_r, tol, "out")
    close(yg.grad, yr.grad, 5 * tol, "dy")
    close(bn.weight.grad, w1.grad, 5 * tol, "dgamma")
    close(bn.bias.grad, b1.grad, 5 * tol, "dbeta")
    close(bn.running_mean, rm1, 1e-5, "running_mean")
    close(bn.running_var, rv1, 1e-5, "running_var")
    if mode in ("identity_res", "bn_res"):
        close(rg.grad, rr.grad, 5 * tol, "dres")
    if mode == "bn_res":
        close(rbn.weight.grad, w2.grad, 5 * tol, "dgamma_res")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("training", [True, False])
@pytest.mark.parametrize("c", [64, 512])
def test_bn_residual_pair_dual_bitexact(dtype, training, c):
    """relu(bn(y) + bn_r(res)) forward statistics (mmad_bn_finalize2) and backward through
    the one-pass pair kernels (mmad_bn_bwd_reduce2 / _finalize2 / _apply2) == the per-BN
    calls, bit for bit (outputs, gradients, running statistics)."""
    n, d, h, w = 2, 4, 6, 5
    y0 = rnd(n, c, d, h, w, seed=80, scale=2.0) + 0.5
    r0 = rnd(n, c, d, h, w, seed=81)
    g0 = rnd(n, c, d, h, w, seed=82)
    res = {}
    for dual in (False, True):
        bn, rbn = _BN(c, 83), _BN(c, 84)
        bn.training = rbn.training = training
        yg = to_vol(y0, dtype).requires_grad_(True)
        rg = to_vol(r0, dtype).requires_grad_(True)
        old = V._BN_DUAL
        V._BN_DUAL = dual
        try:
            out = V.batchnorm_act(yg, bn, relu=True, res=rg, res_bn=rbn)
            out.backward(to_vol(g0, dtype))
        finally:
            V._BN_DUAL = old
        torch.cuda.synchronize()
        res[dual] = (out, yg.grad, rg.grad, bn.weight.grad, bn.bias.grad, rbn.weight.grad,
                     rbn.bias.grad, bn.running_mean, bn.running_var, rbn.running_mean,
                     rbn.running_var, bn.num_batches_tracked, rbn.num_batches_tracked)
    names = ("out", "dy", "dres", "dgamma", "dbeta", "dgamma_res", "dbeta_res", "running_mean",
             "running_var", "running_mean_res", "running_var_res", "nbt", "nbt_res")
    for nm, a, b in zip(names, res[False], res[True]):
        assert torch.equal(a, b), nm


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("training", [True, False])
def test_bn_relu_maxpool_fused(dtype, training):
    """Fused stem tail maxpool(relu(bn(y))) == the unfused batchnorm_act -> max_pool3d chain
    (forward bit-exact incl. ties on ReLU zeros; backward to rounding), and both against
    torch float64."""
    n, c, d, h, w = 2, 64, 9, 10, 11
    y0 = rnd(n, c, d, h, w, seed=70, scale=2.0)
    if dtype == torch.bfloat16:
        y0 = y0.to(dtype).double()
    bn_a, bn_b, bn_r = _BN(c, 71), _BN(c, 71), _BN(c, 71)
    for b_ in (bn_a, bn_b, bn_r):
        b_.training = training
    yr = y0.clone().requires_grad_(True)
    out_r, w_r, b_r, rm_r, rv_r = _ref_bn(yr, bn_r, training)
    pr = F.max_pool3d(torch.relu(out_r), 3, 2, 1)
    g = rnd(*pr.shape, seed=72)
    if dtype == torch.bfloat16:
        g = g.to(dtype).double()
    pr.backward(g)

    ya = to_vol(y0, dtype).requires_grad_(True)
    pa = V.max_pool3d(V.batchnorm_act(ya, bn_a, relu=True), 3, 2, 1)
    pa.backward(to_vol(g, dtype))
    yb = to_vol(y0, dtype).requires_grad_(True)
    pb = V.batchnorm_relu_maxpool(yb, bn_b, None, 3, 2, 1)
    pb.backward(to_vol(g, dtype))

    assert torch.equal(pa, pb), "fused forward differs from the unfused chain"
    tol = 2e-5 if dtype == torch.float32 else 1.5e-2
    close(pb, pr, tol, "out")
    close(yb.grad, ya.grad, tol, "dy fused vs unfused")
    close(bn_b.weight.grad, bn_a.weight.grad, tol, "dgamma fused vs unfused")
    close(bn_b.bias.grad, bn_a.bias.grad, tol, "dbeta fused vs unfused")
    if dtype == torch.float32:
        # (bf16: rounding the BN output before the max moves argmaxes between near-equal
        # values, which routes gradient elsewhere -- compared against the unfused chain only)
        close(yb.grad, yr.grad, 5 * tol, "dy")
        close(bn_b.weight.grad, w_r.grad, 5 * tol, "dgamma")
        close(bn_b.bias.grad, b_r.grad, 5 * tol, "dbeta")
    close(bn_b.running_mean, rm_r, 1e-5, "running_mean")
    close(bn_b.running_var, rv_r, 1e-5, "running_var")


@pytest.mark.parametrize("shape", [(2, 64, 9, 10, 11), (2, 64, 64, 64, 64), (1, 128, 8, 6, 4)],
                         ids=["odd", "stem", "c128"])
def test_bnpool_zwalk_kernel_matches_rows_kernel(shape):
    """The z-walking stem pool kernel of pool.hip (pool_run 2, the default) against the
    per-output rows kernel (0): pooled output, argmax-routed input gradient and BN parameter
    gradients bit-identical (ties on ReLU zeros everywhere)."""
    n, c = shape[:2]
    lib = _lib.load()
    res = {}
    for mode in (0, 2):
        bn = _BN(c, 75)
        bn.training = True
        y = to_vol(rnd(*shape, seed=74, scale=2.0), torch.bfloat16).requires_grad_(True)
        prev = lib.mmad_set_kernel_variant(b"pool_run", mode)
        try:
            p = V.batchnorm_relu_maxpool(y, bn, None, 3, 2, 1)
            p.backward(to_vol(rnd(*p.shape, seed=76), torch.bfloat16))
            torch.cuda.synchronize()
        finally:
            lib.mmad_set_kernel_variant(b"pool_run", prev)
        res[mode] = (p, y.grad, bn.weight.grad, bn.bias.grad)
    for nm, a, b in zip(("out", "dy", "dgamma", "dbeta"), res[0], res[2]):
        assert torch.equal(a, b), nm


@pytest.mark.parametrize("shape,dil", [((2, 512, 4, 4, 4), 4), ((2, 256, 4, 4, 4), 2),
                                       ((2, 64, 8, 8, 8), 1)])
def test_conv_bn_relu_chain(shape, dil):
    """conv (epilogue BN partial sums) -> BN(train) + ReLU -> conv, forward and backward,
    fp32, against torch float64 -- the fused block structure of MedicalNet's BasicBlock."""
    n, c, d, h, w = shape
    x = rnd(*shape, seed=80)
    w1 = rnd(c, c, 3, 3, 3, seed=81, scale=(3.0 / (27 * c)) ** 0.5)
    w2 = rnd(c, c, 3, 3, 3, seed=82, scale=(3.0 / (27 * c)) ** 0.5)
    bn = _BN(c, 83)
    xr = x.clone().requires_grad_(True)
    w1r, w2r = w1.clone().requires_grad_(True), w2.clone().requires_grad_(True)
    c1 = F.conv3d(xr, w1r, None, 1, dil, dil)
    a1, gw, gb, rm, rv = _ref_bn(c1, bn, True)
    a1 = torch.relu(a1)
    out = F.conv3d(a1, w2r, None, 1, dil, dil)
    gy = rnd(*out.shape, seed=84)
    out.backward(gy)

    xg = to_vol(x, torch.float32).requires_grad_(True)
    w1g = w1.float().to(DEV).requires_grad_(True)
    w2g = w2.float().to(DEV).requires_grad_(True)
    y1, parts = V.conv3d(xg, w1g, None, (1,) * 3, (dil,) * 3, (dil,) * 3, torch.float32, True)
    h1 = V.batchnorm_act(y1, bn, parts, relu=True)
    o = V.conv3d(h1, w2g, None, (1,) * 3, (dil,) * 3, (dil,) * 3, torch.float32)
    o.backward(to_vol(gy, torch.float32))
    close(o, out, 2e-5, "out")
    close(bn.bias.grad, gb.grad, 1e-4, "dbeta")
    close(bn.weight.grad, gw.grad, 1e-4, "dgamma")
    close(w1g.grad, w1r.grad, 1e-4, "dw1")
    close(w2g.grad, w2r.grad, 1e-4, "dw2")
    close(xg.grad, xr.grad, 1e-4, "dx")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("k,s,p,shape", [(3, 2, 1, (2, 64, 9, 10, 11)), (2, 2, 0, (2, 16, 9, 8, 7))])
def test_maxpool(k, s, p, shape, dtype):
    x = rnd(*shape, seed=40)
    x = torch.relu(x)                          # exact zeros -> ties everywhere
    x = x.to(dtype).double()
    xr = x.clone().requires_grad_(True)
    yr = F.max_pool3d(xr.float(), k, s, p).double()   # torch CPU kernel = the tie rule
    g = rnd(*yr.shape, seed=41).to(dtype).double()
    yr.backward(g)
    xg = to_vol(x, dtype).requires_grad_(True)
    y = V.max_pool3d(xg, k, s, p)
    y.backward(to_vol(g, dtype))
    assert torch.equal(y.double().cpu(), yr.detach())
    close(xg.grad, xr.grad, 1e-6 if dtype == torch.float32 else 1e-2, "dx")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_global_avg_pool(dtype):
    x = rnd(3, 512, 4, 5, 6, seed=50).to(dtype).double()
    xr = x.clone().requires_grad_(True)
    yr = F.adaptive_avg_pool3d(xr, 1)
    g = rnd(3, 512, 1, 1, 1, seed=51)
    yr.backward(g)
    xg = to_vol(x, dtype).requires_grad_(True)
    y = V.global_avg_pool(xg)
    y.backward(g.float().to(DEV))
    close(y, yr, 1e-6, "gap")
    close(xg.grad, xr.grad, 1e-6 if dtype == torch.float32 else 5e-3, "dgap")


def test_linear_concat_relu():
    x1, x2 = rnd(8, 64, seed=60), rnd(8, 64, seed=61)
    w, b = rnd(64, 128, seed=62, scale=0.1), rnd(64, seed=63)
    refs = [t.clone().requires_grad_(True) for t in (x1, x2, w, b)]
    yr = torch.relu(F.linear(torch.cat(refs[:2], 1), refs[2], refs[3]))
    g = rnd(8, 64, seed=64)
    yr.backward(g)
    gs = [t.float().to(DEV).requires_grad_(True) for t in (x1, x2, w, b)]
    y = V.relu(head_ops.linear(head_ops.concat_features(gs[0], gs[1]), gs[2], gs[3]))
    y.backward(g.float().to(DEV))
    close(y, yr, 1e-5, "linear")
    for a, r, nm in zip(gs, refs, ("dx1", "dx2", "dw", "db")):
        close(a.grad, r.grad, 1e-5, nm)


@pytest.mark.parametrize("C", [2, 3])
@pytest.mark.parametrize("gamma", [None, 1, 2, 5])
def test_losses_vs_golden(C, gamma):
    from tests import _golden as G
    g = G.load("losses")
    x = torch.tensor(g[f"x_C{C}"], device=DEV, requires_grad=True)
    y = torch.from_numpy(g[f"y_C{C}"]).to(DEV)
    if gamma is None:
        wts = torch.tensor(G.W2 if C == 2 else G.W3, dtype=torch.float64, device=DEV)
        loss = head_ops.weighted_cross_entropy(x, y, wts)
        key = f"ce_C{C}"
    else:
        loss = head_ops.focal_loss(x, y, gamma)
        key = f"focal_g{gamma}_C{C}"
    loss.backward()
    assert abs(loss.item() - float(g[key + "_loss"])) <= 1e-12 * max(1, abs(float(g[key + "_loss"])))
    close(x.grad, torch.from_numpy(g[key + "_grad"]), 1e-12, "dlogits")


def test_cast_roundtrip():
    x = rnd(1000, seed=70).to(DEV)
    y = V.cast(x, torch.bfloat16)
    assert torch.equal(y.cpu(), x.cpu().float().to(torch.bfloat16))
    z = V.cast(V.cast(x, torch.float32), torch.float64)
    assert torch.equal(z.cpu(), x.cpu().float().double())


def test_library_loaded_is_ours():
    import os
    lib = _lib.load()
    assert os.path.samefile(lib._name, _lib.LIB_PATH)


# ------------------------------------------------------------ voxel-level fusion (fusion.hip)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_stacked_input_conv_matches_stack_then_conv(dtype):
    """early_fusion.py:77-80 + :35: conv over torch.stack((pet, mri), 1).to(float32); the
    HIP path gathers the two f64 planes into a channel-padded NDHWC operand (odd extents,
    'same' k=5 with bias) -- forward, weight and bias gradients."""
    pet, mri = rnd(2, 11, 9, 13, seed=40), rnd(2, 11, 9, 13, seed=41)
    w = rnd(8, 2, 5, 5, 5, seed=42, scale=0.2).float()
    b = rnd(8, seed=43, scale=0.1).float()
    x = torch.stack((pet, mri), 1)
    xr = x.float().double() if dtype == torch.float32 else x.to(torch.bfloat16).double()
    wr = w.double().requires_grad_()
    br = b.double().requires_grad_()
    ref = F.conv3d(xr, wr if dtype == torch.float32 else wr.to(torch.bfloat16).double(), br,
                   padding=2)
    g = rnd(*ref.shape, seed=44)
    ref.backward(g)
    wd, bd = w.to(DEV).requires_grad_(), b.to(DEV).requires_grad_()
    sv = V.StackedVolumes([pet.to(DEV), mri.to(DEV)])
    y = V.conv3d(sv, wd, bd, padding=(2, 2, 2), cdtype=dtype)
    y.backward(to_vol(g, dtype))
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    close(y, ref, tol, "fwd")
    close(wd.grad, wr.grad, tol if dtype == torch.float32 else 3e-2, "dw")
    close(bd.grad, br.grad, tol if dtype == torch.float32 else 3e-2, "db")
    # same result from one stacked 5-D NCDHW tensor
    y2 = V.conv3d(x.to(DEV), wd.detach(), bd.detach(), padding=(2, 2, 2), cdtype=dtype)
    assert torch.equal(y.detach(), y2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_maxout_ties_nan_and_gradient_routing(dtype):
    a = rnd(2, 16, 3, 5, 4, seed=45)
    b = rnd(2, 16, 3, 5, 4, seed=46)
    b[:, :4] = a[:, :4]                    # exact ties -> first operand (index 0)
    a[0, 5, 1, 1, 1] = float("nan")
    b[1, 6, 2, 2, 2] = float("nan")
    ad, bd = to_vol(a, dtype).requires_grad_(), to_vol(b, dtype).requires_grad_()
    y = V.maxout(ad, bd)
    ar, br = ad.detach().cpu().double(), bd.detach().cpu().double()
    ref, idx = torch.max(torch.stack((ar, br), 0), 0)          # torch's tie / NaN rules
    assert torch.equal(y.detach().cpu().double().isnan(), ref.isnan())
    assert torch.equal(y.detach().cpu().double().nan_to_num(), ref.nan_to_num())
    g = to_vol(rnd(*a.shape, seed=47), dtype)
    y.backward(g)
    gq = g.cpu().double()
    assert torch.equal(ad.grad.cpu().double(), torch.where(idx == 0, gq, 0.0))
    assert torch.equal(bd.grad.cpu().double(), torch.where(idx == 1, gq, 0.0))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_channel_concat_and_split(dtype):
    a = to_vol(rnd(2, 16, 3, 4, 5, seed=48), dtype).requires_grad_()
    b = to_vol(rnd(2, 32, 3, 4, 5, seed=49), dtype).requires_grad_()
    y = V.cat_channels(a, b)
    assert torch.equal(y, torch.cat((a.detach(), b.detach()), 1))
    g = to_vol(rnd(2, 48, 3, 4, 5, seed=50), dtype)
    y.backward(g)
    assert torch.equal(a.grad, g[:, :16]) and torch.equal(b.grad, g[:, 16:])


def test_pad_rows_roundtrip():
    w = torch.randn(6, 54, device=DEV)
    p = torch.empty(6, 216, device=DEV)
    _lib.call("mmad_pad_rows", 6, 54, 216, _lib.ptr(w), _lib.ptr(p), _lib.stream())
    assert torch.equal(p[:, :54], w) and not p[:, 54:].any()
    back = torch.empty_like(w)
    _lib.call("mmad_pad_rows", 6, 216, 54, _lib.ptr(p), _lib.ptr(back), _lib.stream())
    assert torch.equal(back, w)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_batched_weight_pack_equals_per_call_pack(dtype):
    """PackPlan (one launch for every conv: 64x64 LDS-tile jobs for the dgrad layout, one
    (co*ci) x taps job per forward layout, 128x32 tiles when taps <= 32) ==
    mmad_conv_pack_weight per conv, bit for bit."""
    from multimodal_alzheimer_amd import layers as Lyr
    specs = [(64, 64, 3, 1, 1, 1), (64, 128, 3, 2, 1, 1), (128, 256, 3, 1, 2, 2),
             (64, 128, 1, 2, 0, 1), (256, 512, 1, 1, 0, 1), (32, 64, 5, 1, 2, 1)]
    torch.manual_seed(5)
    convs = []
    for ci, co, k, st, p, dl in specs:
        c = Lyr.Conv3d(ci, co, k, stride=st, padding=p, dilation=dl, bias=False).to(DEV)
        c.compute_dtype = dtype
        convs.append(c)
    plan = V.PackPlan(convs, dtype, True)
    plan.run()
    code = _lib.dtype_code(dtype)
    iv = torch.int16 if dtype == torch.bfloat16 else torch.int32
    batched = 0
    for c in convs:
        wp, wpt = c._prepacked if c._prepacked is not None else (None, None)
        d = V._weight_desc(c.weight, c._stride3(), c._pads(), c._dilation3())
        # (a layout whose K needs padding rows keeps the per-call packer: None here)
        if wp is not None:
            assert torch.equal(wp.view(iv), V.pack_weight(d, code, c.weight, dtype, False).view(iv))
            batched += 1
        if wpt is not None:
            assert torch.equal(wpt.view(iv), V.pack_weight(d, code, c.weight, dtype, True).view(iv))
    assert batched >= 5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape,k,s,p", [((2, 1, 5, 6, 22), 7, 2, 3), ((1, 1, 3, 4, 131), 7, 2, 3),
                                         ((1, 1, 2, 3, 300), 5, 1, 2)],
                         ids=["w22", "w131_rows_ragged", "w300_unstaged"])
def test_unfold_input_f64(shape, k, s, p, dtype):
    """W-unfold of an f64 volume for the Cin = 1 convs (LDS-staged rows for W <= 256, the
    per-output form above): out[row][wo][j] = x[row][wo*s - p + j] (0 outside / j >= k),
    f64 -> fp32 -> dtype, exactly."""
    x = rnd(*shape, seed=90).to(DEV)
    d = V.conv_desc(shape, (8, 1, k, k, k), (s, s, s), (p, p, p), (1, 1, 1))
    out = torch.empty(_lib.load().mmad_conv_unfolded_elems(d), dtype=dtype, device=DEV)
    _lib.call("mmad_conv_unfold_input", d, _lib.dtype_code(torch.float64), _lib.ptr(x),
              _lib.dtype_code(dtype), _lib.ptr(out), _lib.stream())
    torch.cuda.synchronize()
    n, _, di, hi, wi = shape
    wo = d.wo
    rows = x.reshape(-1, wi).float().cpu()
    ref = torch.zeros(rows.shape[0], wo, 8)
    for j in range(k):
        xi = torch.arange(wo) * s - p + j
        ok = (xi >= 0) & (xi < wi)
        ref[:, ok, j] = rows[:, xi[ok]]
    assert torch.equal(out.view(rows.shape[0], wo, 8).cpu(), ref.to(dtype))


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("p", [0.2, 0.5])
def test_dropout_keep_rate_scaling_routing(dtype, p):
    """nn.Dropout(p) semantics (pet_cnn.py:27-29, :38-39): train mode zeroes ~p of the
    elements and scales the rest by 1/(1-p); backward routes the gradient through the same
    mask with the same scale; eval mode is the identity; two calls draw different masks."""
    n = 1 << 18
    x = (torch.rand(n, device=DEV) + 0.5).to(dtype).requires_grad_(True)
    y = head_ops.dropout(x, p, True)
    keep = y.detach() != 0
    rate = keep.float().mean().item()
    assert abs(rate - (1 - p)) < 4 * ((p * (1 - p) / n) ** 0.5) + 1e-3
    sc = 1.0 / (1.0 - p)
    exp = (x.detach().float() * sc).to(dtype)
    assert torch.equal(y.detach()[keep], exp[keep])
    g = (torch.rand(n, device=DEV) - 0.5).to(dtype)
    y.backward(g)
    assert torch.equal(x.grad[~keep], torch.zeros_like(x.grad[~keep]))
    assert torch.equal(x.grad[keep], (g.float() * sc).to(dtype)[keep])
    y2 = head_ops.dropout(x.detach(), p, True)
    assert not torch.equal(y2 != 0, keep)
    assert head_ops.dropout(x.detach(), p, False) is not None
    assert torch.equal(head_ops.dropout(x.detach(), p, False), x.detach())
    # 5-D channels-last volumes keep their layout
    v = to_vol(rnd(2, 8, 3, 4, 5, seed=91), dtype)
    yv = head_ops.dropout(v, p, True)
    assert yv.is_contiguous(memory_format=CL)
