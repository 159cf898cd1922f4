"""A training step replayed from a captured HIP graph (graph_step.GraphedTrainStep) equals the
eager step: same kernels in the same order, so parameters, BN running statistics and the
loss after the same number of steps are bit-identical."""
import copy

import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep

pytestmark = pytest.mark.gpu


def _hparams(precision):
    return {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": precision,
            "loss_class_weights": torch.tensor([0.3, 0.7], dtype=torch.float64)}


@pytest.mark.parametrize("precision", ["bf16", "32"])
def test_graph_replay_equals_eager_steps(precision):
    torch.manual_seed(3)
    a = M.Anat_CNN(_hparams(precision)).cuda()
    b = copy.deepcopy(a)
    g = torch.Generator(device="cuda").manual_seed(4)
    batches = [{"mri": torch.rand((2, 32, 32, 32), device="cuda", dtype=torch.float64,
                                  generator=g),
                "label": torch.randint(0, 2, (2,), device="cuda", generator=g)}
               for _ in range(3)]
    warm, steps = 2, 3

    opt_a = a.configure_optimizers()
    for grp in opt_a.param_groups:             # as GraphedTrainStep configures it: the
        grp["capturable"] = True               # captured Adam reads lr from the device
        grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
    for _ in range(warm):                      # GraphedTrainStep's eager warm-up steps
        opt_a.zero_grad(set_to_none=True)
        a.general_step(batches[0], 0, "train")["loss"].backward()
        opt_a.step()
    losses_a = []
    for i in range(steps):
        opt_a.zero_grad(set_to_none=True)
        out = a.general_step(batches[i], 0, "train")
        out["loss"].backward()
        opt_a.step()
        losses_a.append(out["loss"].detach().clone())

    opt_b = b.configure_optimizers()
    gs = GraphedTrainStep(b, opt_b, batches[0], warmup=warm)
    losses_b = [gs(batches[i])["loss"].detach().clone() for i in range(steps)]
    torch.cuda.synchronize()

    for la, lb in zip(losses_a, losses_b):
        assert torch.equal(la, lb)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb
        assert torch.equal(pa, pb), na


def _batch(seed, n=2, s=32):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {"mri": torch.rand((n, s, s, s), device="cuda", dtype=torch.float64, generator=g),
            "label": torch.randint(0, 2, (n,), device="cuda", generator=g)}


def _eval_fused_vs_unfused(m, batch):
    from multimodal_alzheimer_amd import medicalnet
    m.eval()
    with torch.no_grad():
        medicalnet.EVAL_FUSED = True
        fused = m.general_step(batch, 0, "val")["outputs"].clone()
        medicalnet.EVAL_FUSED = False
        ref = m.general_step(batch, 0, "val")["outputs"].clone()
        medicalnet.EVAL_FUSED = True
    m.train()
    return fused, ref


def test_graph_replays_then_eval_refolds_weights():
    """train (graph replays) -> eval -> more replays -> eval: the eval-mode folded-weight
    cache must see the weights and running statistics the replays changed on the device
    (a replay runs no Python, so no tensor version moves)."""
    torch.manual_seed(5)
    m = M.Anat_CNN(_hparams("32")).cuda()
    opt = m.configure_optimizers()
    batch = _batch(6)
    gs = GraphedTrainStep(m, opt, batch, warmup=1)
    outs = []
    for _ in range(2):
        for _ in range(2):
            gs()
        fused, ref = _eval_fused_vs_unfused(m, batch)
        assert (fused - ref).abs().max().item() <= 2e-5 * max(1.0, ref.abs().max().item())
        outs.append(ref)
    assert not torch.equal(outs[0], outs[1]), "weights did not change between evaluations"


def test_graph_replay_draws_fresh_dropout_masks():
    """head_ops.dropout inside a captured graph: every replay draws a new mask (device-side
    seed), keep rate ~ 1 - p, kept values scaled by 1 / (1 - p)."""
    from multimodal_alzheimer_amd import head_ops
    p = 0.4
    x = torch.rand(1 << 16, device="cuda") + 0.5
    head_ops.dropout(x, p, True)                    # warm up outside the capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = head_ops.dropout(x, p, True)
    masks = []
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        keep = y != 0
        masks.append(keep.clone())
        assert abs(keep.float().mean().item() - (1 - p)) < 0.01
        assert torch.allclose(y[keep], x[keep] / (1 - p), rtol=1e-6)
    assert not torch.equal(masks[0], masks[1]) and not torch.equal(masks[1], masks[2])


def test_graph_replay_follows_lr_scheduler():
    """ReduceLROnPlateau (configure_optimizers with reduce_factor_lr_schedule) updates the
    device-resident lr in place; the next replay uses it: at lr ~1e-33 Adam moves nothing."""
    torch.manual_seed(7)
    h = dict(_hparams("32"), reduce_factor_lr_schedule=1e-30)
    m = M.Anat_CNN(h).cuda()
    cfg = m.configure_optimizers()
    opt, sched = cfg["optimizer"], cfg["lr_scheduler"]
    sched.patience = 0
    gs = GraphedTrainStep(m, opt, _batch(8), warmup=1)
    gs()
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    gs()
    moved = [k for k, v in m.named_parameters() if not torch.equal(v, before[k])]
    assert moved, "a replay at the configured lr must update the weights"
    sched.step(1.0)
    sched.step(2.0)                                # no improvement -> lr *= 1e-30
    assert all(float(g["lr"]) < 1e-30 for g in opt.param_groups)
    before = {k: v.detach().clone() for k, v in m.named_parameters()}
    gs()
    torch.cuda.synchronize()
    for k, v in m.named_parameters():
        assert torch.equal(v, before[k]), k


def test_capture_after_eager_default_stream_steps():
    """Eager steps on the default stream, then GraphedTrainStep (its warm-up on a side
    stream, the capture on torch's capture stream), then replays: bit-identical to the same
    sequence run eagerly.  This once faulted at capture_end: the logged loss kept each step's
    autograd graph -- and the parameters' AccumulateGrad nodes, bound to the stream they were
    created on -- alive into the next step, so the captured backward synchronised with the
    default stream.  Now nothing holds a finished step's graph."""
    torch.manual_seed(11)
    a = M.Anat_CNN(_hparams("bf16")).cuda()
    b = copy.deepcopy(a)
    batches = [_batch(20 + i) for i in range(3)]
    n_eager, warm = 2, 1

    def eager(m, opt, batch):
        opt.zero_grad(set_to_none=True)
        out = m.general_step(batch, 0, "train")
        out["loss"].backward()
        opt.step()
        return out["loss"].detach().clone()

    opt_a = a.configure_optimizers()
    for _ in range(n_eager):
        eager(a, opt_a, batches[0])
    for grp in opt_a.param_groups:
        grp["capturable"] = True
        grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
    for _ in range(warm):
        eager(a, opt_a, batches[0])
    losses_a = [eager(a, opt_a, batches[i]) for i in range(3)]

    opt_b = b.configure_optimizers()
    for _ in range(n_eager):
        eager(b, opt_b, batches[0])          # default stream
    assert b.logged["train_loss"].grad_fn is None
    gs = GraphedTrainStep(b, opt_b, batches[0], warmup=warm)
    assert gs.out["loss"].grad_fn is None
    losses_b = [gs(batches[i])["loss"].clone() for i in range(3)]
    torch.cuda.synchronize()
    for la, lb in zip(losses_a, losses_b):
        assert torch.equal(la, lb)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(pa, pb), na


@pytest.mark.parametrize("mode", ["staged", "after"])
def test_graph_with_allreduce_replay_equals_eager(mode):
    """bench.py's N > 1 launch modes at one RCCL rank: "staged" (the default: the backward
    replayed as four stage graphs, each stage's bucket all-reduced on the side stream while
    the next replays) and "after" (forward + backward in one graph, the bucketed all-reduces
    issued after it), then the captured Adam -- bit-identical to plain eager steps of an
    identical model (at world 1 the average is the gradient itself)."""
    import torch.distributed as dist
    from multimodal_alzheimer_amd.data_parallel import GradAllReduce
    from multimodal_alzheimer_amd.graph_step import backward_stages
    torch.manual_seed(13)
    a = M.Anat_CNN(_hparams("bf16")).cuda()
    b = copy.deepcopy(a)
    batches = [_batch(40 + i) for i in range(3)]
    warm = 2
    port = 29563 + (mode == "after")
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", torch.cuda.current_device()))
    try:
        opt_a = a.configure_optimizers()
        for grp in opt_a.param_groups:
            grp["capturable"] = True
            grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
        for _ in range(warm):
            opt_a.zero_grad(set_to_none=True)
            a.general_step(batches[0], 0, "train")["loss"].backward()
            opt_a.step()
        losses_a = []
        for i in range(3):
            opt_a.zero_grad(set_to_none=True)
            out = a.general_step(batches[i], 0, "train")
            out["loss"].backward()
            opt_a.step()
            losses_a.append(out["loss"].detach().clone())
        opt_b = b.configure_optimizers()
        if mode == "staged":
            red = GradAllReduce(b.parameters(), bucket_mb=None, stages=backward_stages(b)[1])
        else:
            red = GradAllReduce(b.parameters(), bucket_mb=4.0)
        gs = GraphedTrainStep(b, opt_b, batches[0], warmup=warm, reducer=red, collectives=mode)
        assert gs.opt_graph is not None
        assert len(gs.graphs) == (4 if mode == "staged" else 1)
        losses_b = [gs(batches[i])["loss"].clone() for i in range(3)]
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()
    for la, lb in zip(losses_a, losses_b):
        assert torch.equal(la, lb)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(pa, pb), na
