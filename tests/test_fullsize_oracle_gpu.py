"""BASELINE configs 2 and 3 at their FULL size (batch 8 of 1 x 128^3) against the reference.

Fixtures (tests/golden/make_golden.py, cases ``anat_r10_128`` and ``pair_r10_128``): the
reference's own code run in fp32 on CPU -- Anat_CNN (anat_cnn.py:13-109) for config 2; for
config 3 the reference's PET_CNN_ResNet and Anat_CNN branches under the build's two-backbone
head (a build extension, so that head is unpinned) -- plus the same train step evaluated in
float64 on the oracle restatement.  Weights and volumes come from oracle.prng, so this box
regenerates them; gradients are recorded at the elements ``prng.sample_index`` picks.

Config 5's PET branch (``pet_r18_160``: the reference's PET_CNN_ResNet, depth 18, 2 x 1 x
160^3) pins the 20^3 layer3 / layer4 route.  Config 5's MRI branch (``anat_r34_160``: Anat_CNN
on ResNet-34, 4 x 1 x 160^3) pins the 34-layer wiring against the oracle restatement only:
the reference's Anat_CNN rejects depth 34 (anat_cnn.py:37-46), so its "reference" logits are
the restatement's fp32 run and its bf16 yardstick the restatement under CPU autocast.  Each fixture's final Linear bias is chosen by the
generator (``mixed_head``: the leading principal direction of the batch's pooled features)
so the train argmax is split across the batch and no eval row is ReLU'd to all zeros; the
tests load it after the prng weights.

Bars:
  * fp32 HIP path: logits within 1e-4 (the north star's bar), argmax bit-exact (mixed
    classes, train and eval), loss within 1e-4, running
    statistics within 2e-3 of each tensor's max, every sampled gradient element within
    max(4 x the reference fp32 error, 1e-2 of the tensor's max) of float64 (one output
    channel may exceed it, up to 25 %: a ReLU mask flip, see _assert_f64_bar), and the
    full-tensor |g| sums and norms within 2e-3 of the reference's.
  * bf16 HIP path (the kernels the bench launches: stem, patch, lattice, lattice8, pwgrad,
    fused pool) against float64, with the REFERENCE's own bf16 path as the yardstick: the
    fixture also holds the reference's train step under CPU autocast bf16 (Lightning's
    precision "bf16"), whose error against float64 is what bf16 storage costs.  Logits within
    3e-2 of max(1, |logit|) and within 2x the reference's bf16 logit error (+5e-3), argmax
    exact wherever the float64 top-2 margin exceeds twice the bound, loss within 3e-2
    relative; running statistics within 2e-2 of each tensor's max; per gradient tensor, the
    normwise relative error of the sampled elements, the relative error of every LARGE
    sampled element (|g| >= half the tensor's max) and the |g|-sum error each within 2x the
    reference's bf16 error of the same quantity + 0.02 (+0.05 for the large elements, + a
    quarter of the reference's normwise error for the sum), and the median over tensors of
    our normwise error / the reference's at most 1.25 (measured 0.95-1.01).
    bf16 rounding noise compounds along the backward chain (each dgrad re-rounds to bf16) and
    through BN's cancelling sums and the stem's max-pool argmax moves, so both paths' errors
    grow towards the input (ResNet-18 at 160^3: ~0.4 normwise at layer1 for both); the
    strict per-kernel bar is test_full_size_bf16_every_conv_in_situ below.
"""
import numpy as np
import pytest
import torch

import multimodal_alzheimer_amd as M
from oracle import prng
from tests import _golden as G

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_ATOL = 1e-4

# bf16 bars relative to the reference's own bf16 error (module docstring)
REF16_X, REF16_ABS, REF16_LRG_ABS = 2.0, 0.02, 0.05


def _errs(got, ex, full_abs_sum, exact_abs_sum):
    """normwise, large-element and |g|-sum relative errors of sampled gradient elements"""
    nrm = np.linalg.norm(got - ex) / max(np.linalg.norm(ex), 1e-30)
    big = np.abs(ex) >= 0.5 * np.abs(ex).max()
    lrg = float((np.abs(got - ex)[big] / np.abs(ex)[big]).max()) if big.any() else 0.0
    return nrm, lrg, abs(full_abs_sum - exact_abs_sum) / max(exact_abs_sum, 1e-30)


# fixture -> (model builder, batch keys, batch seed)
BUILD = {
    "anat_r10_128": (lambda p: M.Anat_CNN(G.anat_hparams(10, precision=p)), ("mri",), 1301),
    "pair_r10_128": (lambda p: M.PET_MRI_ResNet_Fusion(G.anat_hparams(10, fl_gamma=2, precision=p)),
                     ("pet1451", "mri"), 1401),
    "pet_r18_160": (lambda p: M.PET_CNN_ResNet(G.anat_hparams(18, fl_gamma=2, precision=p)),
                    ("pet1451",), 1501),
    "anat_r34_160": (lambda p: M.Anat_CNN(G.anat_hparams(34, fl_gamma=2, precision=p)),
                     ("mri",), 1601),
    # config 5's whole network (build extension) against the oracle restatement at 2 x 160^3
    "tri_160": (lambda p: M.Tri_ResNet_Tabular_Fusion(G.anat_hparams(
        10, fl_gamma=2, resnet_depth_mri=34, resnet_depth_pet=18, precision=p)),
        ("pet1451", "mri"), 1701),
}
CASES = ["anat_r10_128", "pair_r10_128", "pet_r18_160", "anat_r34_160", "tri_160"]
IDS = ["config2", "config3", "config5_pet", "config5_mri", "config5_tri"]
# cases whose gradient sums may fall back to the float64 bar (the 36-layer ResNet-34 chain)
DEEP = ("anat_r34_160", "tri_160")


@pytest.fixture(autouse=True)
def _bench_routes():
    """The config-5 fixtures run at batch 2, where the 20^3 layer4 convs have too few
    residue-class blocks (128) for lattice5.hip's default rule; the bench runs them at batch
    8 through that kernel, so it is forced on here (it only matches 5d^3 grids)."""
    from multimodal_alzheimer_amd import _lib
    lib = _lib.load()
    prev = lib.mmad_set_kernel_variant(b"lattice5", 2)
    yield
    lib.mmad_set_kernel_variant(b"lattice5", prev)


def _build(name, precision):
    g = G.load(name)
    fn, keys, bseed = BUILD[name]
    m = fn(precision)
    assert list(m.state_dict()) == [str(k) for k in g["state_dict_keys"]]
    G.load_fixture_weights(m, g)
    shape = tuple(int(v) for v in g["shape"])
    batch = G.batch_for(shape, 2, bseed, keys)
    if name == "tri_160":                 # make_golden.tri_160: 9 tabular features
        from oracle import tabpfn_standin
        batch["tabular"] = tabpfn_standin.training_table(bseed + 50, shape[0])[0]
    batch = {k: v.to(DEV) for k, v in batch.items()}
    return g, m.to(DEV), batch


def _run(name, precision):
    g, m, batch = _build(name, precision)
    m.eval()
    with torch.no_grad():
        ev = m.general_step(batch, 0, "val")["outputs"].cpu().numpy()
    m.train()
    res = m.general_step(batch, 0, "train")
    res["loss"].backward()
    torch.cuda.synchronize()
    return g, m, ev, res["outputs"].detach().cpu().numpy(), res["loss"].item()


@pytest.mark.parametrize("name", CASES, ids=IDS)
def test_full_size_fp32_matches_reference(name):
    g, m, ev, tr, loss = _run(name, "32")
    for got, key in ((ev, "eval_logits"), (tr, "train_logits")):
        err = np.abs(got - g[key]).max()
        assert err <= LOGIT_ATOL, f"{key}: max|err| {err:.3e}"
        assert (got.argmax(1) == g[key].argmax(1)).all(), key
    assert abs(loss - float(g["train_loss"])) <= 1e-4 * max(1.0, abs(float(g["train_loss"])))
    bufs = dict(m.named_buffers())
    for key in g:
        if key.startswith("buf/"):
            pname = key.split("/", 2)[2]
            ref = g[key]
            err = np.abs(bufs[pname].double().cpu().numpy().ravel()[: ref.size] - ref).max()
            assert err <= 2e-3 * max(np.abs(ref).max(), 1e-30), (key, err)
    params = dict(m.named_parameters())
    gscale = max(np.abs(g[k]).max() for k in g if k.startswith("grad64/samp/"))
    n = 0
    for key in g:
        if not key.startswith("grad/samp/"):
            continue
        pname = key[len("grad/samp/"):]
        p = params[pname]
        full = p.grad.detach().double().cpu().numpy().ravel()
        idx = prng.sample_index(pname, full.size)
        ours, ref32, exact = full[idx], g[key], g["grad64/samp/" + pname]
        e_ref = np.abs(ref32 - exact).max()
        bound = max(4 * e_ref, 1e-2 * np.abs(exact).max()) + 1e-6 * gscale
        err = np.abs(ours - exact)
        rows = p.shape[0] if full.size % p.shape[0] == 0 else full.size
        bad_rows = np.unique((idx // (full.size // rows))[err > bound])
        assert bad_rows.size <= 1, f"{pname}: {bad_rows.size} channels beyond {bound:.3e}"
        assert err.max() <= max(bound, 0.25 * np.abs(exact).max()), \
            f"{pname}: max err {err.max():.3e} vs bound {bound:.3e} (reference fp32 {e_ref:.3e})"
        st = g["grad/stats/" + pname]
        got = np.array([np.abs(full).sum(), np.sqrt((full * full).sum())])
        # within 2e-3 of the reference's fp32 sums.  Only for the 36-layer ResNet-34 chain
        # (anat_r34_160 / tri_160, whose "reference" is the oracle's fp32 run), where fp32 noise
        # compounds (ReLU masks flipped by pre-activations within fp32 rounding of 0), the
        # float64 sums may stand in: within 2e-3 + the larger of twice the fp32 reference's
        # own deviation from them and a fixed 2e-2 -- a bound that does not depend on this
        # implementation's error, so a regression cannot widen it
        st64 = g["grad64/stats/" + pname][1:]
        ok32 = np.all(np.abs(got - st[1:]) <= 2e-3 * np.abs(st[1:]) + 1e-6 * gscale)
        ok64 = False
        if name in DEEP:
            ref_dev = np.abs(st[1:] - st64) / np.abs(st64)
            ok64 = np.all(np.abs(got - st64) <=
                          (2e-3 + np.maximum(2 * ref_dev, 2e-2)) * np.abs(st64) + 1e-6 * gscale)
        assert ok32 or ok64, (pname, got, st[1:], st64, np.abs(got - st64) / np.abs(st64))
        n += 1
    assert n >= 20


@pytest.mark.parametrize("name", CASES, ids=IDS)
def test_full_size_bf16_matches_reference(name):
    """The benched bf16 kernels at the benched size against the same reference fixture."""
    g, m, ev, tr, loss = _run(name, "bf16")
    exact = g["train_logits64"]
    e16 = np.abs(g["train_logits16"] - exact).max()
    bound = min(3e-2 * max(1.0, np.abs(exact).max()), REF16_X * e16 + 5e-3)
    err = np.abs(tr - exact).max()
    print(f"{name} bf16 logits max|err| vs f64 {err:.3e} (reference bf16 {e16:.3e}, "
          f"bound {bound:.3e})")
    assert err <= bound
    top2 = np.sort(exact, axis=1)[:, ::-1]
    decided = (top2[:, 0] - top2[:, 1]) > 2 * bound
    assert decided.any()
    assert (tr.argmax(1)[decided] == exact.argmax(1)[decided]).all()
    err_ev = np.abs(ev - g["eval_logits"]).max()
    assert err_ev <= 3e-2 * max(1.0, np.abs(g["eval_logits"]).max()), err_ev
    l64 = float(g["train_loss64"])
    assert abs(loss - l64) <= 3e-2 * max(1.0, abs(l64)), (loss, l64)
    bufs = dict(m.named_buffers())
    for key in g:
        if key.startswith("buf/"):
            pname = key.split("/", 2)[2]
            ref = g[key]
            e = np.abs(bufs[pname].double().cpu().numpy().ravel()[: ref.size] - ref).max()
            assert e <= 2e-2 * max(np.abs(ref).max(), 1e-3), (key, e)
    params = dict(m.named_parameters())
    rows, bad, ratios = [], [], []
    for key in g:
        if not key.startswith("grad64/samp/"):
            continue
        pname = key[len("grad64/samp/"):]
        full = params[pname].grad.detach().double().cpu().numpy().ravel()
        ex, st = g[key], g["grad64/stats/" + pname]
        ours = _errs(full[prng.sample_index(pname, full.size)], ex, np.abs(full).sum(), st[1])
        ref = _errs(g["grad16/samp/" + pname], ex, g["grad16/stats/" + pname][1], st[1])
        # (a |g| sum over 64..512 BN channels fluctuates with the per-element noise: the
        # reference's own sum error can be small by chance, so a quarter of its normwise
        # error is allowed on top)
        lim = (REF16_X * ref[0] + REF16_ABS, REF16_X * ref[1] + REF16_LRG_ABS,
               REF16_X * ref[2] + 0.25 * ref[0] + REF16_ABS)
        rows.append((pname, ours, ref))
        ratios.append(ours[0] / max(ref[0], 1e-12))
        if any(o > b for o, b in zip(ours, lim)):
            bad.append(pname)
    for pname, ours, ref in rows:
        print(f"  {pname}: normwise {ours[0]:.3e} (ref bf16 {ref[0]:.3e})  large-element "
              f"{ours[1]:.3e} ({ref[1]:.3e})  |g| sum {ours[2]:.3e} ({ref[2]:.3e})")
    print(f"  median normwise ratio ours / reference bf16: {np.median(ratios):.3f}")
    assert len(rows) >= 20
    assert not bad, f"bf16 gradients beyond 2x the reference's bf16 error: {bad}"
    assert np.median(ratios) <= 1.25, np.median(ratios)


def _ref_conv(x, w, s, p, d):
    """fp32 conv3d as im2col + matmul (autograd gives dX and dW)."""
    from tests.test_fullsize_gpu import _ref_conv as rc
    return rc(x, w, s, p, d)


def _ref_dw(x, gy, k, s, p, d, planes=2):
    """dW = sum over output voxels of gY x im2col(X), as fp32 GEMMs over chunks of output
    z-planes (K <= a few 10^4 voxels each) summed in float64: a weight-gradient reference
    whose own summation error is far below the kernel's (one fp32 GEMM over all 2^21
    voxels of the stem is not)."""
    import torch.nn.functional as F
    n, c = x.shape[:2]
    co = gy.shape[1]
    span = (k - 1) * d + 1
    u = F.pad(x.float(), (p,) * 6)
    out = torch.zeros((co, c * k ** 3), dtype=torch.float64, device=x.device)
    do = gy.shape[2]
    for z0 in range(0, do, planes):
        z1 = min(do, z0 + planes)
        ub = u[:, :, z0 * s:(z1 - 1) * s + span]
        for dim in (2, 3, 4):
            ub = ub.unfold(dim, span, s)
        ub = ub[..., ::d, ::d, ::d]
        cols = ub.permute(0, 2, 3, 4, 1, 5, 6, 7).reshape(-1, c * k ** 3)
        g = gy[:, :, z0:z1].float().permute(0, 2, 3, 4, 1).reshape(-1, co)
        out += (g.t() @ cols).double()
    return out.view(co, c, k, k, k)


@pytest.mark.parametrize("name", ["anat_r10_128", "pet_r18_160", "anat_r34_160"],
                         ids=["config2", "config5_pet", "config5_mri"])
def test_full_size_bf16_every_conv_in_situ(name):
    """The per-kernel bar at the benched size on the step's REAL operands: the bf16 step of
    the fixture's model runs with every conv's input, output, output gradient and input
    gradient recorded, and each conv (stem, patchz / patch, s2conv / s2dgrad, pointwise,
    lattice8, lattice_zp, pwgrad, lattice wgrad: whatever the dispatch picked) is checked
    against a plain PyTorch conv (fp32 im2col + matmul; the weight gradient as fp32 GEMMs over
    two output planes at a time summed in float64) of the SAME bf16 operands -- its own
    error only, not the chain's compounded bf16 drift the model-level test bounds:
      y, dX (bf16): |err| <= 2^-7 |ref| + 1e-3 max|ref|   (one bf16 rounding + fp32 sums)
      dW (fp32):    |err| <= 1e-3 |ref| + 1e-4 (|X|.|gY|) + 1e-6 max|ref|
    (|X|.|gY| = the same contraction over absolute values: the scale of a weight gradient's
    fp32 summation error, since dW cancels heavily -- BN's backward makes gY zero-mean per
    channel -- over 2^15 .. 2^21 voxels)."""
    from multimodal_alzheimer_amd import layers as Lyr
    g, m, batch = _build(name, "bf16")
    recs = {}
    for cname, conv in m.named_modules():
        if not isinstance(conv, Lyr.Conv3d):
            continue

        def run(x, want_stats, _orig=conv._run, _name=cname):
            out = _orig(x, want_stats)
            y = out[0] if want_stats else out
            rec = recs[_name] = {"x": x.detach(), "y": y.detach()}
            if x.requires_grad:
                x.register_hook(lambda gx: rec.__setitem__("dx", gx.detach()))
            y.register_hook(lambda gy: rec.__setitem__("gy", gy.detach()))
            return out
        conv._run = run
    m.train()
    res = m.general_step(batch, 0, "train")
    res["loss"].backward()
    torch.cuda.synchronize()
    convs = dict(m.named_modules())
    checked, bad = [], []
    D = torch.float64
    for cname, rec in recs.items():
        conv = convs[cname]
        st, p, d = conv._stride3()[0], conv._pads()[0], conv._dilation3()[0]
        k = conv.kernel_size[0]
        x = rec["x"]
        xr = (x.float().to(torch.bfloat16) if x.dtype != torch.bfloat16 else x).float()
        xr = xr.detach().requires_grad_(x.requires_grad)
        wr = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
        yr = _ref_conv(xr, wr, st, p, d)
        assert "gy" in rec, cname
        gy = rec["gy"].float()
        yr.backward(gy)
        dwr = _ref_dw(xr.detach(), gy, k, st, p, d)
        absdw = _ref_dw(xr.detach().abs(), gy.abs(), k, st, p, d)
        line = [cname]
        for got, ref, what in ((rec["y"], yr, "y"), (rec.get("dx"), xr.grad, "dX")):
            if got is None or ref is None:
                continue
            got, ref = got.to(D), ref.detach()
            err = (got - ref).abs()
            nbad = int((err > 2 ** -7 * ref.abs() + 1e-3 * ref.abs().max()).sum())
            line.append(f"{what} err/max {err.max().item() / ref.abs().max().item():.2e}"
                        f"{' BAD ' + str(nbad) if nbad else ''}")
            if nbad:
                bad.append((cname, what))
        dw = conv.weight.grad.to(D)
        err = (dw - dwr).abs()
        nbad = int((err > 1e-3 * dwr.abs() + 1e-4 * absdw + 1e-6 * dwr.abs().max()).sum())
        line.append(f"dW err/max {err.max().item() / dwr.abs().max().item():.2e} "
                    f"err/abs {(err / absdw.clamp_min(1e-30)).max().item():.2e}"
                    f"{' BAD ' + str(nbad) if nbad else ''}")
        if nbad:
            bad.append((cname, "dW"))
        print("  ".join(line))
        checked.append(cname)
        del yr, xr, wr, dwr, absdw
        torch.cuda.empty_cache()
    print(f"{name}: {len(checked)} convs checked in situ")
    assert len(checked) >= (12 if name == "anat_r10_128" else 20)
    assert not bad, bad
