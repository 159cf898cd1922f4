"""conv_seg's AdaptiveAvgPool3d(1) -> Flatten -> Linear (-> ReLU) (anat_cnn.py:66-76) as the
fused head_ops.gap_linear (mmad_gap_partial + mmad_gap_linear_fwd, mmad_linear_gap_bwd)
against the same modules run one by one (global_avg_pool, flatten, linear): the fold order,
the dot products and the row rounding are the same, so logits, dW, dbias and the input
gradient must be bit-identical."""
import pytest
import torch

from multimodal_alzheimer_amd import head_ops, layers
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
CL = torch.channels_last_3d


def _run(x0, w0, b0, relu, fused):
    x = x0.clone().requires_grad_(True)
    w = w0.clone().requires_grad_(True)
    b = b0.clone().requires_grad_(True)
    if fused:
        y = head_ops.gap_linear(x, w, b, relu=relu)
    else:
        y = head_ops.linear(torch.flatten(V.global_avg_pool(x), 1), w, b, relu=relu)
    g = torch.Generator(device="cuda").manual_seed(7)
    gy = torch.randn(y.shape, device="cuda", generator=g)
    y.backward(gy)
    torch.cuda.synchronize()
    return y.detach(), x.grad, w.grad, b.grad


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "f32"])
@pytest.mark.parametrize("relu", [True, False], ids=["relu", "plain"])
@pytest.mark.parametrize("shape,n_out", [((8, 512, 16, 16, 16), 2), ((2, 64, 2, 2, 2), 3),
                                         ((3, 256, 5, 7, 6), 10)],
                         ids=["config2_head", "one_part", "ragged"])
def test_gap_linear_bit_identical_to_modules(dtype, relu, shape, n_out):
    g = torch.Generator(device="cuda").manual_seed(sum(shape))
    x = torch.randn(shape, device="cuda", generator=g).to(dtype).contiguous(memory_format=CL)
    w = torch.randn((n_out, shape[1]), device="cuda", generator=g) * 0.05
    b = torch.randn(n_out, device="cuda", generator=g) * 0.1
    ref = _run(x, w, b, relu, False)
    got = _run(x, w, b, relu, True)
    for a, r, what in zip(got, ref, ("y", "dx", "dW", "dbias")):
        assert a.shape == r.shape, what
        assert torch.equal(a, r), (what, (a.float() - r.float()).abs().max().item())
    assert ref[0].abs().sum() > 0


def test_conv_seg_uses_the_fused_head_and_matches(monkeypatch):
    """Anat_CNN's conv_seg (the Sequential pattern match in layers.Sequential): loss and every
    gradient identical with the fused head on and off."""
    import multimodal_alzheimer_amd as M
    from tests import _golden as G
    calls = []
    real = head_ops.gap_linear
    monkeypatch.setattr(head_ops, "gap_linear", lambda *a, **k: calls.append(1) or real(*a, **k))
    res = []
    for on in (False, True):
        monkeypatch.setattr(layers, "GAP_LINEAR", on)
        torch.manual_seed(3)
        m = M.Anat_CNN(G.anat_hparams(10, precision="bf16")).cuda()
        g = torch.Generator(device="cuda").manual_seed(5)
        batch = {"mri": torch.rand((2, 32, 32, 32), generator=g, device="cuda",
                                   dtype=torch.float64),
                 "label": torch.tensor([0, 1], device="cuda")}
        o = m.general_step(batch, 0, "train")
        o["loss"].backward()
        torch.cuda.synchronize()
        res.append((o["loss"].detach(), {k: p.grad.detach().clone()
                                         for k, p in m.named_parameters()}))
    assert calls, "the fused head did not run"
    assert torch.equal(res[0][0], res[1][0])
    for k in res[0][1]:
        assert torch.equal(res[0][1][k], res[1][1][k]), k
