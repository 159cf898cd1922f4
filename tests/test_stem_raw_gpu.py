"""The MedicalNet stem (conv1: Cin 1 -> 64, 7^3, stride 2, pad 3; anat_cnn.py:29-31 via
MedicalNet's ResNet) read straight from the raw volume (mmad_conv3d_fwd_raw /
mmad_conv3d_wgrad_raw: the kernels unfold each input row in registers) against the
unfold-then-convolve path (mmad_conv_unfold_input + mmad_conv3d_fwd / _wgrad) on the same
inputs: the LDS images are the same bf16 values in the same places, so the output, the BN
partial sums and the weight gradient must be BIT-identical.  Shapes: BASELINE config 2
(8 x 128^3, f64 as the DataLoader delivers it), batch 2 at 64^3, ragged depth / height with a
narrower width, and a tiny volume (fewer z-steps than the pipeline depth)."""
import pytest
import torch

from multimodal_alzheimer_amd import _lib as L
from multimodal_alzheimer_amd import volume_ops as V

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _run(shape, dtype, seed):
    lib = L.load()
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.rand(shape, generator=g, device="cuda", dtype=torch.float64).to(dtype)
    w = (torch.rand((64, 1, 7, 7, 7), generator=g, device="cuda") * 2 - 1) * 0.05
    d = V.conv_desc(tuple(shape), tuple(w.shape), (2,) * 3, (3,) * 3, (1,) * 3)
    dt, in_dt = L.dtype_code(BF), L.dtype_code(dtype)
    assert lib.mmad_stem_raw_ok(d, in_dt, dt) == 1, shape
    wp = V.pack_weight(d, dt, w, BF, False)
    rows = lib.mmad_conv3d_stats_rows(d, dt)
    out = {}
    for raw in (False, True):
        y = V._empty_vol(d.n, 64, d.do_, d.ho, d.wo, BF, x.device)
        st = torch.empty((rows, 2, 64), device="cuda")
        if raw:
            L.call("mmad_conv3d_fwd_raw", d, in_dt, L.ptr(x), dt, L.ptr(wp), None, L.ptr(y),
                   L.ptr(st), L.stream())
        else:
            u = torch.empty(lib.mmad_conv_unfolded_elems(d), dtype=BF, device="cuda")
            L.call("mmad_conv_unfold_input", d, in_dt, L.ptr(x), dt, L.ptr(u), L.stream())
            L.call("mmad_conv3d_fwd", d, dt, L.ptr(u), L.ptr(wp), None, L.ptr(y), L.ptr(st),
                   L.stream())
        gy = ((torch.rand(y.shape, generator=torch.Generator(device="cuda").manual_seed(seed + 1),
                          device="cuda") * 2 - 1).to(BF)
              .contiguous(memory_format=torch.channels_last_3d))
        ws = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, dt) + 3) // 4, device="cuda")
        dw = torch.empty(w.shape, device="cuda")
        if raw:
            L.call("mmad_conv3d_wgrad_raw", d, in_dt, L.ptr(x), dt, L.ptr(gy), L.ptr(dw), None,
                   L.ptr(ws), L.stream(), None)
        else:
            L.call("mmad_conv3d_wgrad", d, dt, L.ptr(u), L.ptr(gy), L.ptr(dw), None, L.ptr(ws),
                   L.stream())
        torch.cuda.synchronize()
        out[raw] = (y, st, dw)
    return out


CASES = [((8, 1, 128, 128, 128), torch.float64), ((2, 1, 64, 64, 64), torch.float64),
         ((1, 1, 37, 50, 64), torch.float64), ((1, 1, 9, 11, 16), torch.float64)]
IDS = ["config2_f64", "batch2_64", "ragged_w64", "tiny"]


def test_stem_raw_not_offered_off_its_geometry():
    """W > 128 (config 5's 160^3), odd W (MNI 91 x 109 x 91) and f32 input keep the unfold
    path: mmad_stem_raw_ok says no."""
    lib = L.load()
    dt = L.dtype_code(BF)
    for shape, dtype in (((2, 1, 160, 160, 160), torch.float64),
                         ((2, 1, 91, 109, 91), torch.float64),
                         ((2, 1, 64, 64, 64), torch.float32)):
        d = V.conv_desc(shape, (64, 1, 7, 7, 7), (2,) * 3, (3,) * 3, (1,) * 3)
        assert lib.mmad_stem_raw_ok(d, L.dtype_code(dtype), dt) == 0, shape


@pytest.mark.parametrize("shape,dtype", CASES, ids=IDS)
def test_stem_raw_bit_identical_to_unfolded(shape, dtype):
    out = _run(shape, dtype, 31)
    for a, b, what in zip(out[False], out[True], ("output", "BN partial sums", "dW")):
        assert torch.equal(a, b), f"{what}: max|diff| {(a.float() - b.float()).abs().max()}"
    assert out[True][0].float().abs().sum() > 0


def test_stem_raw_in_the_model_matches_unfolded(monkeypatch):
    """The model-level route (volume_ops._Conv3dFn on a f64 (B,1,D,H,W) input): the same
    loss and stem weight gradient with MMAD_STEM_RAW on and off."""
    import multimodal_alzheimer_amd as M
    from tests import _golden as G
    res = []
    for raw in (False, True):
        monkeypatch.setattr(V, "STEM_RAW", raw)
        torch.manual_seed(3)
        m = M.Anat_CNN(G.anat_hparams(10, precision="bf16")).cuda()
        g = torch.Generator(device="cuda").manual_seed(5)
        batch = {"mri": torch.rand((2, 64, 64, 64), generator=g, device="cuda",
                                   dtype=torch.float64),
                 "label": torch.tensor([0, 1], device="cuda")}
        o = m.general_step(batch, 0, "train")
        o["loss"].backward()
        torch.cuda.synchronize()
        res.append((o["loss"].detach(), m.model.conv1.weight.grad.detach().clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
