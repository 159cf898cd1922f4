"""mmad_adam_repack (csrc/adam.hip, fused_optim.AdamRepack): the captured step's Adam fused
with the bf16 weight repack.  Its update must be torch's fused Adam bit for bit (the
reference's optimizer, anat_cnn.py:111-126, as torch.optim.Adam(fused=True) runs it: param,
exp_avg, exp_avg_sq and the device step counter), and the packed layouts it writes must be
exactly what mmad_conv_pack_dual_batch makes of the updated weights."""
import copy

import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd import fused_optim as F
from multimodal_alzheimer_amd import layers as Lyr
from multimodal_alzheimer_amd import volume_ops as V
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep

pytestmark = pytest.mark.gpu

SHAPES = [(64, 64, 3, 3, 3), (128, 64, 1, 1, 1), (32, 16, 3, 3, 3), (64,), (2, 512), (2,),
          (7, 5), (1000,)]


def _opt(params, lrs=(1e-3, 3e-4), wd=(0.0, 0.01)):
    groups = [{"params": params[0::2], "lr": torch.tensor(lrs[0], device="cuda"),
               "weight_decay": wd[0]},
              {"params": params[1::2], "lr": torch.tensor(lrs[1], device="cuda"),
               "weight_decay": wd[1], "betas": (0.8, 0.99), "eps": 1e-6}]
    return torch.optim.Adam(groups, fused=True, capturable=True)


def _params(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(s, device="cuda", generator=g) * 0.1) for s in SHAPES]


def _grads(params, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    for p in params:
        p.grad = torch.randn(p.shape, device="cuda", generator=g) * 1e-2


def test_adam_update_bit_identical_to_torch_fused():
    pa, pb = _params(1), _params(1)
    oa, ob = _opt(pa), _opt(pb)
    _grads(pa, 2)
    _grads(pb, 2)
    oa.step()                                   # state initialised by torch in both
    ob.step()
    fused = F.AdamRepack(ob)
    for it in range(4):
        _grads(pa, 10 + it)
        _grads(pb, 10 + it)
        oa.step()
        fused.step()
        torch.cuda.synchronize()
        for a, b in zip(pa, pb):
            sa, sb = oa.state[a], ob.state[b]
            assert torch.equal(a, b), (it, tuple(a.shape), (a - b).abs().max().item())
            assert torch.equal(sa["exp_avg"], sb["exp_avg"])
            assert torch.equal(sa["exp_avg_sq"], sb["exp_avg_sq"])
            assert torch.equal(sa["step"], sb["step"])
    assert float(ob.state[pb[0]]["step"]) == 5.0
    assert int(fused.arrivals.abs().sum()) == 0          # re-armed for the next launch


def test_adam_repack_writes_both_packed_layouts():
    torch.manual_seed(3)
    convs = torch.nn.Sequential(
        Lyr.Conv3d(1, 64, 7, stride=2, padding=3, bias=False),       # the unfolded stem
        Lyr.Conv3d(64, 64, 3, padding=1, bias=False), Lyr.Conv3d(64, 128, 3, stride=2, padding=1,
                                                                bias=False),
        Lyr.Conv3d(128, 128, 3, padding=2, dilation=2, bias=False),
        Lyr.Conv3d(128, 256, 1, stride=2, bias=False)).cuda()
    for c in convs:
        c.compute_dtype = torch.bfloat16
    V.prepack(convs)
    plan = convs._mmad_pack_plan
    assert plan.nduals >= 2 and len(plan.unfolds) == 1
    params = list(convs.parameters())
    opt = torch.optim.Adam([{"params": params, "lr": torch.tensor(1e-2, device="cuda")}],
                           fused=True, capturable=True)
    _grads(params, 5)
    opt.step()
    fused = F.AdamRepack(opt, [plan])
    _grads(params, 6)
    fused.step()
    torch.cuda.synchronize()
    def bufs():
        return [tuple(None if b is None else b.clone() for b in e[2:4]) for e in plan.entries]
    got = bufs()
    plan.run_duals()                                     # the same weights, packed separately
    torch.cuda.synchronize()
    for g, r in zip(got, bufs()):
        for a, b in zip(g, r):
            assert (a is None) == (b is None)
            assert a is None or torch.equal(a, b)


def _hparams():
    return {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": "bf16",
            "loss_class_weights": torch.tensor([0.3, 0.7], dtype=torch.float64)}


def _batch(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {"mri": torch.rand((2, 32, 32, 32), device="cuda", dtype=torch.float64, generator=g),
            "label": torch.randint(0, 2, (2,), device="cuda", generator=g)}


def test_captured_step_repacks_weights_changed_outside_the_graph():
    """GraphedTrainStep with the fused optimizer: replays take their packed weights from the
    previous replay's Adam; a load_state_dict between replays (new fp32 weights, versions
    bumped) must be seen -- the next replay equals the eager step from the same weights."""
    torch.manual_seed(9)
    a = M.Anat_CNN(_hparams()).cuda()
    b = copy.deepcopy(a)
    other = {k: v.clone() for k, v in M.Anat_CNN(_hparams()).cuda().state_dict().items()}
    batches = [_batch(30 + i) for i in range(4)]
    warm = 1

    opt_a = a.configure_optimizers()
    for grp in opt_a.param_groups:
        grp["capturable"] = True
        grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")

    def eager(i):
        opt_a.zero_grad(set_to_none=True)
        out = a.general_step(batches[i], 0, "train")
        out["loss"].backward()
        opt_a.step()
        return out["loss"].detach().clone()

    for _ in range(warm):
        eager(0)
    la = [eager(0), eager(1)]
    a.load_state_dict(other)
    la += [eager(2), eager(3)]

    opt_b = b.configure_optimizers()
    gs = GraphedTrainStep(b, opt_b, batches[0], warmup=warm)
    assert gs.fused is not None and gs.fused.plans
    lb = [gs(batches[0])["loss"].clone(), gs(batches[1])["loss"].clone()]
    b.load_state_dict(other)
    lb += [gs(batches[2])["loss"].clone(), gs(batches[3])["loss"].clone()]
    torch.cuda.synchronize()
    for x, y in zip(la, lb):
        assert torch.equal(x, y)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(pa, pb), na
    sa, sb = opt_a.state_dict()["state"], opt_b.state_dict()["state"]
    for k in sa:
        for f in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(sa[k][f], sb[k][f]), (k, f)
