"""Twin outputs (volume_ops "twin outputs"): a residual block's input gradient from conv1
and from the shortcut meet inside the producer's BN backward kernels (g2 of
mmad_bn_bwd_* / mmad_bnpool_bwd_*) instead of in torch's gradient-accumulation add.  Also
the broadcast global-average-pool gradient (volume_ops.GAP_BCAST: the last BN pair reads
the pooled gradient's per-sample rows in place instead of a materialised broadcast).

The kernels add g2 as torch adds two gradients of one tensor (fp32 sum, then one rounding to
the storage dtype), so the whole training step must be BIT-identical with and without twins:
logits, loss, every parameter gradient, every running statistic.  Covered: ResNet-10 (one
block per stage: stem pool -> layer1 identity residual, shortcut-B pairs after), ResNet-18
(block-to-block identity residuals inside the dilated stages) and ResNet-50 (Bottleneck), in
fp32 and bf16, plus the config-2 size itself (1x128^3, batch 8, bf16)."""
import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hp(depth, precision):
    return {"n_classes": 2, "resnet_depth": depth, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": precision,
            "loss_class_weights": torch.tensor([0.2031496, 0.7968504], dtype=torch.float64)}


def _step(model, batch):
    r = model.general_step(batch, 0, "train")
    r["loss"].backward()
    torch.cuda.synchronize()
    return r["outputs"].detach().clone(), r["loss"].detach().clone()


@pytest.mark.parametrize("depth,precision,n,size", [
    (10, "bf16", 2, 48), (10, "32", 2, 40), (18, "bf16", 2, 48), (50, "bf16", 1, 32),
    (10, "bf16", 8, 128)], ids=["r10-bf16", "r10-fp32", "r18-bf16", "r50-bf16", "r10-config2"])
def test_twin_step_bit_identical(depth, precision, n, size, monkeypatch):
    torch.manual_seed(3)
    ma = M.Anat_CNN(_hp(depth, precision))
    with torch.no_grad():            # live logits: the head's final ReLU passes gradient
        ma.model.conv_seg[-2].bias.fill_(1.0)
    mb = M.Anat_CNN(_hp(depth, precision))
    mb.load_state_dict(ma.state_dict())
    ma, mb = ma.to(DEV), mb.to(DEV)
    g = torch.Generator(device=DEV).manual_seed(11)
    batch = {"mri": torch.rand((n, size, size, size), generator=g, device=DEV,
                               dtype=torch.float64),
             "label": torch.randint(0, 2, (n,), generator=g, device=DEV)}
    monkeypatch.setattr(V, "TWIN", True)
    monkeypatch.setattr(V, "GAP_BCAST", True)
    la, lossa = _step(ma, batch)
    assert not V._TWINS, "every twin made in the step was taken by its block"
    monkeypatch.setattr(V, "TWIN", False)
    monkeypatch.setattr(V, "GAP_BCAST", False)     # and the materialised GAP gradient
    lb, lossb = _step(mb, batch)
    assert torch.equal(la, lb) and torch.equal(lossa, lossb)
    pb = dict(mb.named_parameters())
    checked = 0
    for k, p in ma.named_parameters():
        if p.grad is None:
            assert pb[k].grad is None, k
            continue
        assert torch.equal(p.grad, pb[k].grad), k
        checked += 1
    assert checked > 20
    bb = dict(mb.named_buffers())
    for k, v in ma.named_buffers():
        assert torch.equal(v, bb[k]), k


def test_twin_kernels_match_summed_gradient():
    """The g2 entry points directly, fixed-channel (fused) and generic (caller-added) BN
    layouts: dy / gmask / dgamma / dbeta with (g, g2) == with g + g2 rounded to bf16."""
    torch.manual_seed(5)
    for c in (64, 24):
        y = torch.randn(2, c, 6, 7, 5, device=DEV).to(memory_format=torch.channels_last_3d)
        bn = torch.nn.BatchNorm3d(c).to(DEV)
        yb = y.to(torch.bfloat16)
        res = torch.randn_like(yb)
        ga = torch.randn_like(yb)
        gb = torch.randn_like(yb)
        outs = []
        for twin in (True, False):
            yy = yb.clone().requires_grad_(True)
            rr = res.clone().requires_grad_(True)
            o = V.batchnorm_act(yy, bn, relu=True, res=rr, twin=twin)
            if twin:
                o2 = V.take_twin(o)
                assert o2 is not o and o2.data_ptr() == o.data_ptr()
            else:
                o2 = o
            (o.float() * ga.float()).sum().add((o2.float() * gb.float()).sum()).backward()
            torch.cuda.synchronize()
            outs.append((yy.grad.clone(), rr.grad.clone(), bn.weight.grad.clone(),
                         bn.bias.grad.clone()))
            bn.weight.grad = bn.bias.grad = None
        for a, b in zip(*outs):
            assert torch.equal(a, b), c


@pytest.mark.parametrize("c", [64, 12])
def test_twin_bn_relu_maxpool_matches_summed_gradient(c):
    """The fused stem BN+ReLU+max-pool with a twin (g2 in mmad_bnpool_bwd_reduce / _apply:
    the k3 s2 cell kernels for 64 channels, the caller-added sum for 12)."""
    torch.manual_seed(6)
    y = torch.randn(2, c, 10, 9, 8, device=DEV).to(memory_format=torch.channels_last_3d)
    yb = y.to(torch.bfloat16)
    bn = torch.nn.BatchNorm3d(c).to(DEV)
    outs = []
    ga = gb = None
    for twin in (True, False):
        yy = yb.clone().requires_grad_(True)
        o = V.batchnorm_relu_maxpool(yy, bn, None, 3, 2, 1, twin=twin)
        o2 = V.take_twin(o) if twin else o
        assert (o2 is not o) == twin
        if ga is None:
            ga, gb = torch.randn_like(o), torch.randn_like(o)
        (o.float() * ga.float()).sum().add((o2.float() * gb.float()).sum()).backward()
        torch.cuda.synchronize()
        outs.append((yy.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()))
        bn.weight.grad = bn.bias.grad = None
    for a, b in zip(*outs):
        assert torch.equal(a, b), c


@pytest.mark.parametrize("shape", [
    # (N, Ci, S, Co, k, pad, dil): the igemm wgrad (layer2-like), the lattice wgrad (layer4
    # dilation 4 on 16^3), the 1^3 shortcut
    (2, 64, 16, 128, 3, 1, 1), (2, 256, 16, 128, 3, 4, 4), (2, 128, 16, 64, 1, 0, 1)],
    ids=["igemm", "lattice", "pointwise"])
def test_wgrad_split_stream_matches(shape, monkeypatch):
    """mmad_conv3d_wgrad_split (split-K reduction on the side stream, REDUCE_STREAM) writes
    the same dW bits as mmad_conv3d_wgrad; the step joins the side stream before reading."""
    n, ci, s, co, k, p, d = shape
    torch.manual_seed(9)
    x = torch.randn(n, ci, s, s, s, device=DEV).to(torch.bfloat16).to(
        memory_format=torch.channels_last_3d)
    gy = torch.randn(n, co, s, s, s, device=DEV).to(torch.bfloat16).to(
        memory_format=torch.channels_last_3d)
    w0 = torch.randn(co, ci, k, k, k, device=DEV) * 0.05
    grads = []
    for split in (False, True):
        monkeypatch.setattr(V, "REDUCE_STREAM", split)
        w = w0.clone().requires_grad_(True)
        y = V.conv3d(x, w, None, (1, 1, 1), (p, p, p), (d, d, d), torch.bfloat16)
        y.backward(gy)
        torch.cuda.synchronize()
        grads.append(w.grad.clone())
    assert torch.equal(grads[0], grads[1])
