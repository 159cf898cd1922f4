"""Module-level parity on the MI355X: the drop-in pkg.models classes running on
libmmad_hip.so against golden vectors produced by the real reference code
(tests/golden/make_golden.py).  Bar (BASELINE.json north star): fp32 logits within 1e-4,
argmax bit-exact (ties on ReLU-zeroed logits included); loss, gradients and BN running
statistics within fp32 reduction-order tolerance."""
import numpy as np
import pytest
import torch

import multimodal_alzheimer_amd as M
from oracle import models_ref
from tests import _golden as G

pytestmark = pytest.mark.gpu
DEV = "cuda"
LOGIT_ATOL = 1e-4


def build_product(name):
    hp_fn, kind, _, _ = G.CASES[name]
    h = hp_fn()
    if kind == "anat":
        return M.Anat_CNN(h)
    if kind == "petres":
        return M.PET_CNN_ResNet(h)
    if kind == "smallpet":
        return M.Small_PET_CNN(h)
    if kind == "ef":
        return M.PET_MRI_EF(h)
    if kind == "fmf":
        return M.PET_MRI_FMF(h)
    if kind == "amf":                      # stage 1 -> 2 -> 3 through checkpoint files
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            return G.amf_checkpoint_chain(d)
    pet = M.Small_PET_CNN(G.pet_hparams())
    mri = M.Anat_CNN(G.anat_hparams(10))
    return M.Anat_PET_CNN(h, pet_model=pet, mri_model=mri)


def run_product(name, precision=None):
    g = G.load(name)
    m = build_product(name)
    G.load_prng_weights(m, int(g["seed"]))
    if precision is not None:
        M.layers.set_compute_dtype(m, precision)
    m = m.to(DEV)
    batch = {k: v.to(DEV) for k, v in G.batch_of(name, g).items()}
    out = {}
    m.eval()
    with torch.no_grad():
        out["eval_logits"] = m.general_step(batch, 0, "val")["outputs"].cpu().numpy()
    m.train()
    res = m.general_step(batch, 0, "train")
    res["loss"].backward()
    torch.cuda.synchronize()
    out["train_logits"] = res["outputs"].detach().cpu().numpy()
    out["train_loss"] = res["loss"].item()
    return g, m, out


@pytest.mark.parametrize("name", list(G.CASES))
def test_model_matches_reference(name):
    g, m, out = run_product(name)
    for key in ("eval_logits", "train_logits"):
        err = np.abs(out[key] - g[key]).max()
        assert err <= LOGIT_ATOL, f"{key}: max|err| {err:.3e}"
        assert (out[key].argmax(1) == g[key].argmax(1)).all(), f"{key}: argmax differs"
    assert abs(out["train_loss"] - float(g["train_loss"])) <= 1e-4 * max(1.0, abs(float(g["train_loss"])))
    params = dict(m.named_parameters())
    buffers = dict(m.named_buffers())
    # gradients that are analytically ~0 (e.g. a BN bias feeding GAP -> Linear -> BN1d:
    # the batch-normalised downstream makes sum_n dL/dfeat_n vanish) are pure rounding
    # noise in both implementations; compare against the largest gradient of the model.
    gscale = max(np.abs(g[k]).max() for k in g if k.startswith("grad/") and "/stats/" not in k)
    checked = 0
    beyond = []          # gradients outside the golden tolerance: judged against f64 below
    for key in g:
        kind, _, rest = key.partition("/")
        if kind not in ("grad", "buf"):
            continue
        sub, _, pname = rest.partition("/")
        t = params[pname].grad if kind == "grad" else buffers[pname]
        assert t is not None, key
        a = t.detach().double().cpu().numpy().ravel()
        ref = g[key]
        if sub in ("full", "head"):
            a = a[: ref.size]
            scale = max(np.abs(ref).max(), 1e-30)
            err = np.abs(a - ref).max()
            # grads: 1e-2 of the tensor's max -- an isolated ReLU mask flip (a pre-activation
            # within ~1e-5 of 0, which the reference's own fp32 path also produces against
            # f64, see test_fp32_gradient_*) moves gradients at the 1e-3 level
            tol = (1e-2 * scale + 1e-6 * gscale) if kind == "grad" else 2e-3 * scale
            if kind == "grad" and err > tol:
                beyond.append(key)
            else:
                assert err <= tol, f"{key}: err {err:.3e} (ref max {scale:.3e})"
        else:
            got = np.array([a.sum(), np.abs(a).sum(), np.sqrt((a * a).sum())])
            np.testing.assert_allclose(got[1:], ref[1:], rtol=2e-3, err_msg=key)
        checked += 1
    assert checked > 3
    if beyond:
        # The reference's own fp32 gradients are not exact either: where a ReLU / max-pool
        # decision sits within fp32 rounding of a tie the two fp32 paths route differently.
        # Such tensors must be as close to an f64 evaluation of the same network as the
        # reference's fp32 result is (the bar of the test below).
        _, f64 = _f64_oracle_grads(name)
        for key in beyond:
            pname = key.split("/", 2)[2]
            ref32 = g[key]
            exact = f64[pname][: ref32.size]
            ours = params[pname].grad.detach().double().cpu().numpy().ravel()[: ref32.size]
            _assert_f64_bar(key, ours, ref32, exact, gscale, params[pname].shape[0])


def _assert_f64_bar(key, ours, ref32, exact, gscale, rows=None):
    """ours within max(4x the reference-fp32 error, 1e-2 of the tensor's max) of the f64
    evaluation, except in at most one output channel (row ``rows`` of the tensor seen as
    [rows][-1]; default: one element): a single ReLU mask flip -- a pre-activation within
    fp32 rounding of 0 (tools/diag_maskflip.py finds channel 503 of layer4.1.bn2 at
    |x| = 2.9e-5 in anat_r50's 50-layer forward) -- routes that voxel's gradient
    differently, which moves that channel's BN gradients and its conv filter's gradient
    (dW[c] = sum dY[v, c] X[v + tap]) and nothing else measurably (the flipped activation is
    ~0 on either side, so the next layer's dW barely sees it).  The reference's own fp32 path
    can flip just as well; that channel must still stay within 25 % of the tensor's max."""
    e_ref = np.abs(ref32 - exact).max()
    n = exact.size
    rows = n if rows is None or n % rows else rows
    err = np.abs(ours - exact).reshape(rows, -1).max(axis=1)
    err = np.sort(err)[::-1]
    bound = max(4 * e_ref, 1e-2 * np.abs(exact).max()) + 1e-6 * gscale
    second = err[1] if err.size > 1 else 0.0
    assert second <= bound and err[0] <= max(bound, 0.25 * np.abs(exact).max()), \
        f"{key}: ours {err[0]:.3e} / {second:.3e} vs f64, reference fp32 {e_ref:.3e}"


def _f64_oracle_grads(name):
    """The oracle evaluated in float64 (all weights, activations and the loss in f64)."""
    g = G.load(name)
    ref = G.build_oracle(name)
    G.load_prng_weights(ref, int(g["seed"]))
    ref = ref.double()
    batch = G.batch_of(name, g)
    ref.train()
    if hasattr(ref, "inputs"):
        y_hat = ref(*ref.inputs(batch, torch.float64))
    elif hasattr(ref, "batch_key"):
        y_hat = ref(batch[ref.batch_key].unsqueeze(1).double())
    else:
        y_hat = ref(batch["pet1451"].unsqueeze(1).double(), batch["mri"].unsqueeze(1).double())
    ref.criterion(y_hat, batch["label"]).backward()
    return g, {k: p.grad.double().numpy().ravel() for k, p in ref.named_parameters()
               if p.grad is not None}


@pytest.mark.parametrize("name", [n for n in G.CASES if n not in ("anat_r10_32", "anat_r10_64")])
def test_fp32_gradient_error_no_worse_than_reference_cpu(name):
    """Against a float64 evaluation of the same network, the HIP fp32 gradients are as
    accurate as the reference's own fp32 CPU gradients (golden): per parameter, our error
    <= 4x the reference's error, or <= 1e-2 of the tensor's max when a ReLU mask flip
    (pre-activation within fp32 rounding of 0 -- tools/diag_forward.py shows the reference
    fp32 path flipping too) moves it, + 1e-6 of the model's gradient scale.
    (anat_r10_32 / anat_r10_64 have all-zero gradients: every logit is ReLU'd to 0.)"""
    g, f64 = _f64_oracle_grads(name)
    _, m, _ = run_product(name)
    params = dict(m.named_parameters())
    gscale = max(np.abs(v).max() for v in f64.values())
    worst = 0.0
    for key in g:
        if not key.startswith("grad/") or "/stats/" in key:
            continue
        pname = key.split("/", 2)[2]
        ref32 = g[key]
        exact = f64[pname][: ref32.size]
        ours = params[pname].grad.detach().double().cpu().numpy().ravel()[: ref32.size]
        e_ref = np.abs(ref32 - exact).max()
        e_ours = np.abs(ours - exact).max()
        _assert_f64_bar(pname, ours, ref32, exact, gscale, params[pname].shape[0])
        worst = max(worst, e_ours / (e_ref + 1e-6 * gscale))
    assert worst > 0


def test_bf16_mode_tracks_fp32():
    """bf16 throughput mode: same model, activations/weights in bf16, f32 accumulation."""
    g, m, out = run_product("anat_r10_32", precision=torch.bfloat16)
    assert np.isfinite(out["train_logits"]).all()
    err = np.abs(out["train_logits"] - g["train_logits"]).max()
    assert err <= 5e-2 * max(1.0, np.abs(g["train_logits"]).max()), f"bf16 drift {err:.3e}"
    for p in m.parameters():
        if p.grad is not None:
            assert torch.isfinite(p.grad).all()


def test_oracle_live_vs_product_r10_64():
    """BASELINE config 1 shape (64^3, B=2): product on GPU vs the CPU oracle run live."""
    g = G.load("anat_r10_64")
    ref = models_ref.AnatCNNRef(G.anat_hparams(10))
    G.load_prng_weights(ref, int(g["seed"]))
    batch = G.batch_of("anat_r10_64", g)
    r = ref.general_step(batch, 0, "train")
    m = M.Anat_CNN(G.anat_hparams(10))
    m.load_state_dict(ref.state_dict())
    m = m.to(DEV)
    o = m.general_step({k: v.to(DEV) for k, v in batch.items()}, 0, "train")
    err = (o["outputs"].detach().cpu() - r["outputs"].detach()).abs().max().item()
    assert err <= LOGIT_ATOL
    assert torch.equal(o["outputs"].argmax(1).cpu(), r["outputs"].argmax(1))


def test_two_backbone_fusion_and_three_branch_run():
    """Build extensions (configs 3 and 5): shapes, finiteness, gradients reach every branch."""
    h = G.anat_hparams(10, fl_gamma=2)
    m = M.PET_MRI_ResNet_Fusion(h).to(DEV)
    b = {k: v.to(DEV) for k, v in G.batch_for((2, 32, 32, 32), 2, 3, ("pet1451", "mri")).items()}
    o = m.general_step(b, 0, "train")
    o["loss"].backward()
    assert o["outputs"].shape == (2, 2)
    assert m.model_pet.model.conv1.weight.grad is not None
    assert m.model_mri.model.conv1.weight.grad is not None
    h5 = G.anat_hparams(10, precision="bf16", resnet_depth_mri=34, resnet_depth_pet=18)
    m5 = M.Tri_ResNet_Tabular_Fusion(h5).to(DEV)
    b["tabular"] = torch.rand(2, 9, dtype=torch.float64, device=DEV)
    o5 = m5.general_step(b, 0, "train")
    o5["loss"].backward()
    assert torch.isfinite(o5["loss"])


@pytest.mark.parametrize("size", [32, 64])
def test_eval_fused_blocks_match_unfused(size):
    """Eval-mode BasicBlocks (BN folded into the conv, residual + ReLU in the epilogue) vs
    the training-style op sequence on the same trained weights and running statistics.
    At 64^3 layer2.0.conv1 (16^3 -> 8^3) runs the stride-2 sub-patch kernel's epilogue."""
    from multimodal_alzheimer_amd import medicalnet
    for precision, tol in ((torch.float32, 2e-5), (torch.bfloat16, 3e-2)):
        torch.manual_seed(3)
        h = G.anat_hparams(10)
        m = M.Anat_CNN(h)
        M.layers.set_compute_dtype(m, precision)
        m = m.to(DEV)
        batch = {"mri": torch.rand((2, size, size, size), dtype=torch.float64, device=DEV),
                 "label": torch.tensor([0, 1], device=DEV)}
        opt = m.configure_optimizers()
        for _ in range(3):                       # non-trivial running statistics
            opt.zero_grad()
            m.general_step(batch, 0, "train")["loss"].backward()
            opt.step()
        m.eval()
        with torch.no_grad():
            medicalnet.EVAL_FUSED = True
            fused = m.general_step(batch, 0, "val")["outputs"].float()
            medicalnet.EVAL_FUSED = False
            ref = m.general_step(batch, 0, "val")["outputs"].float()
            medicalnet.EVAL_FUSED = True
        err = (fused - ref).abs().max().item()
        assert err <= tol * max(1.0, ref.abs().max().item()), (precision, err)


@pytest.mark.parametrize("n,c", [(37, 2), (120, 3), (7, 3)])
def test_bootstrap_metrics_on_device_match_reference_loop(n, c):
    """Base_Model.bootstrap_metric (base_model.py:219-239) on device vs the oracle's
    restatement of the reference loop, same global RNG state: the drawn index sets are
    identical, so mean and CI agree to f32 rounding (ties in the logits included)."""
    from multimodal_alzheimer_amd.lightning_compat import (MulticlassF1Score,
                                                          MulticlassMatthewsCorrCoef)
    from oracle import metrics_ref
    g = torch.Generator().manual_seed(n)
    y_hat = torch.randn(n, c, generator=g, dtype=torch.float64).round(decimals=1)
    y_hat[: n // 4] = torch.relu(y_hat[: n // 4]) * 0       # all-zero rows: argmax ties
    y = torch.randint(0, c, (n,), generator=g)
    m = M.Anat_CNN(G.anat_hparams(10, n_classes=c)).to(DEV)
    for kind, metric in (("f1", MulticlassF1Score(num_classes=c, average="macro")),
                         ("mcc", MulticlassMatthewsCorrCoef(num_classes=c))):
        torch.manual_seed(123)
        mean_ref, ci_ref, _ = metrics_ref.bootstrap(kind, y_hat, y, 1000)
        torch.manual_seed(123)
        mean, ci = m.bootstrap_metric(metric, y_hat.to(DEV), y.to(DEV), 1000)
        assert abs(mean.item() - mean_ref.item()) <= 2e-6, (kind, mean, mean_ref)
        assert abs(ci.item() - ci_ref.item()) <= 2e-6 * max(1.0, ci_ref.item()), (kind, ci, ci_ref)


def test_grad_allreduce_rccl_bucket_views_single_rank():
    """GradAllReduce over RCCL (world 1, so the mean is the local gradient): conv weight
    gradients written straight into the bucket slices, BN / head gradients copied in and
    out; two steps with set_to_none=True and one accumulating step (set_to_none=False)
    all equal the plain single-process gradients."""
    import torch.distributed as dist
    from multimodal_alzheimer_amd.data_parallel import GradAllReduce
    batch = {k: v.to(DEV) for k, v in G.batch_for((2, 32, 32, 32), 2, 41).items()}
    ref = M.Anat_CNN(G.anat_hparams(10, linear_out=[32]))
    G.load_prng_weights(ref, 40)
    ref = ref.to(DEV)
    mdl = M.Anat_CNN(G.anat_hparams(10, linear_out=[32]))
    mdl.load_state_dict(ref.state_dict())
    mdl = mdl.to(DEV)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29561", rank=0, world_size=1,
                            device_id=torch.device(DEV, torch.cuda.current_device()))
    try:
        red = GradAllReduce(mdl.parameters(), bucket_mb=8.0)
        assert len(red.buckets) > 1
        for step, none in enumerate((True, True, False)):
            for m in (ref, mdl):
                m.zero_grad(set_to_none=none)
                m.general_step(batch, 0, "train")["loss"].backward()
            red.finish()
            torch.cuda.synchronize()
            conv = mdl.model.layer4[0].conv2.weight
            if none:
                assert conv.grad.data_ptr() == conv._mmad_grad_view.data_ptr(), step
            for (k, a), (_, b) in zip(ref.named_parameters(), mdl.named_parameters()):
                assert torch.allclose(a.grad, b.grad, rtol=1e-5, atol=1e-7), (step, k)
    finally:
        dist.destroy_process_group()


def test_fusion_from_stage1_checkpoints_matches_golden(tmp_path):
    """§8(f) row 1: stage-1 checkpoints -> Anat_PET_CNN(path_pet=, path_anat=) -> golden
    `anat_pet_fusion` logits (fp32, 1e-4) and loss."""
    g = G.load("anat_pet_fusion")
    fus, _ = G.fusion_via_stage1_checkpoints(str(tmp_path))
    fus = fus.to(DEV)
    batch = {k: v.to(DEV) for k, v in G.batch_of("anat_pet_fusion", g).items()}
    fus.eval()
    with torch.no_grad():
        ev = fus.general_step(batch, 0, "val")["outputs"].cpu().numpy()
    fus.train()
    res = fus.general_step(batch, 0, "train")
    tr = res["outputs"].detach().cpu().numpy()
    for got, key in ((ev, "eval_logits"), (tr, "train_logits")):
        assert np.abs(got - g[key]).max() <= LOGIT_ATOL, key
        assert (got.argmax(1) == g[key].argmax(1)).all(), key
    assert abs(res["loss"].item() - float(g["train_loss"])) <= 1e-4


def test_adam_step_matches_reference_adam():
    """One optimizer step of the product (fused Adam on merged groups, on the GPU) equals the
    reference's per-tensor torch.optim.Adam (anat_cnn.py:111-128, CPU) on the same gradients,
    to fp32 rounding of the fused vs single-tensor update."""
    h = G.anat_hparams(10, linear_out=[32], l2_reg=1e-4)
    ref = models_ref.AnatCNNRef(h)
    G.load_prng_weights(ref, 9)
    m = M.Anat_CNN(h)
    m.load_state_dict(ref.state_dict())
    m = m.to(DEV)
    opt = m.configure_optimizers()
    ref_opt = torch.optim.Adam(models_ref.adam_param_groups(ref, h), weight_decay=h["l2_reg"])
    gen = torch.Generator().manual_seed(4)
    for step in range(3):
        for (k, p), (_, q) in zip(ref.named_parameters(), m.named_parameters()):
            gr = torch.randn(p.shape, generator=gen) * 1e-2
            p.grad = gr.clone()
            q.grad = gr.to(DEV)
        ref_opt.step()
        opt.step()
    for (k, p), (_, q) in zip(ref.named_parameters(), m.named_parameters()):
        err = (q.detach().cpu() - p.detach()).abs().max().item()
        assert err <= 1e-6 * max(1.0, p.abs().max().item()), (k, err)
    # resume from the reference optimizer's checkpoint state (torch Adam groups: fused
    # unset): the product keeps its fused multi-tensor Adam and steps on identically
    import copy
    opt.load_state_dict(copy.deepcopy(ref_opt.state_dict()))
    assert all(g["fused"] for g in opt.param_groups)
    for (k, p), (_, q) in zip(ref.named_parameters(), m.named_parameters()):
        gr = torch.randn(p.shape, generator=gen) * 1e-2
        p.grad = gr.clone()
        q.grad = gr.to(DEV)
    ref_opt.step()
    opt.step()
    for (k, p), (_, q) in zip(ref.named_parameters(), m.named_parameters()):
        err = (q.detach().cpu() - p.detach()).abs().max().item()
        assert err <= 1e-6 * max(1.0, p.abs().max().item()), (k, err)
