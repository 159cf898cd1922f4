"""Staged backward (graph_step.StagedBackward / backward_stages) and per-stage gradient
buckets (GradAllReduce(stages=...), launch_stage) on CPU.

bench.py's N > 1 launch mode replays the backward as consecutive captured graphs split at
backbone stage boundaries and starts each stage's all-reduce while the next stage runs.
Checked here without a GPU:
  * backward_stages partitions a MedicalNet ResNet (and the two-backbone fusion model) by
    stage -- head + layer4 | layer3 | layer2 | layer1 + stem -- covering every trainable
    parameter once;
  * the staged backward through a two-output "twin alias" producer (the residual blocks'
    volume_ops twin outputs) gives bit-identical gradients to one loss.backward(), and each
    producer node runs exactly once;
  * world 2 (gloo): per-stage launches + finish() == the mean of the per-rank gradients.
"""
import os
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from multimodal_alzheimer_amd import volume_ops
from multimodal_alzheimer_amd.data_parallel import GradAllReduce
from multimodal_alzheimer_amd.graph_step import StagedBackward, backward_stages

CALLS = {"n": 0}


class _Twin(torch.autograd.Function):
    """relu(x) returned twice, the second output an alias of the first (as volume_ops'
    producers return their twin); the backward sums both gradients."""

    @staticmethod
    def forward(ctx, x):
        out = x.relu()
        ctx.save_for_backward(out)
        return out, out.view_as(out)

    @staticmethod
    def backward(ctx, g1, g2):
        CALLS["n"] += 1
        (out,) = ctx.saved_tensors
        g = g1 if g2 is None else (g2 if g1 is None else g1 + g2)
        return g * (out > 0)


class _Block(nn.Module):
    """residual block reading its input through the twin alias for the shortcut"""

    def __init__(self, w, twin_out=True):
        super().__init__()
        self.f = nn.Linear(w, w)
        self.sc = nn.Linear(w, w)
        self.twin_out = twin_out

    def forward(self, x):
        xr = volume_ops.take_twin(x)
        y = self.f(x) + self.sc(xr)
        if not self.twin_out:
            return y.relu()
        out, alias = _Twin.apply(y)
        volume_ops._register_twin(out, alias)
        return out


class _Net(nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.stem = nn.Linear(8, 16)
        self.s1 = nn.Sequential(_Block(16))
        self.s2 = nn.Sequential(_Block(16))
        self.s3 = nn.Sequential(_Block(16, twin_out=False))
        self.head = nn.Linear(16, 3)

    def forward(self, x):
        volume_ops.clear_twins()
        out, alias = _Twin.apply(self.stem(x))
        volume_ops._register_twin(out, alias)
        return self.head(self.s3(self.s2(self.s1(out))))

    def stages(self):
        return ([[self.s3], [self.s2], [self.s1]],
                [list(self.s3.parameters()) + list(self.head.parameters()),
                 list(self.s2.parameters()), list(self.s1.parameters()),
                 list(self.stem.parameters())])


def _data(seed=1, n=6):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(n, 8, generator=g), torch.randint(0, 3, (n,), generator=g)


def test_staged_backward_equals_backward():
    x, y = _data()
    a, b = _Net(), _Net()
    nn.functional.cross_entropy(a(x), y).backward()
    CALLS["n"] = 0
    nn.functional.cross_entropy(a(x), y)         # forward only: count the nodes of one step
    sb = StagedBackward(*b.stages())
    sb.arm()
    loss = nn.functional.cross_entropy(b(x), y)
    sb.disarm()
    assert [len(r) for r in sb._rec] == [2, 2, 2]  # each boundary: the tensor + its twin
    CALLS["n"] = 0
    sb.run_all(loss)
    assert CALLS["n"] == 3                       # stem, s1, s2 producers: once each
    for (k, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        assert pb.grad is not None, k
        assert torch.equal(pa.grad, pb.grad), k


def test_backward_stages_partitions_resnet():
    import multimodal_alzheimer_amd as M
    from tests import _golden as G
    m = M.Anat_CNN(G.anat_hparams(10))
    bounds, params = backward_stages(m)
    net = m.model
    assert bounds == [[net.layer4], [net.layer3], [net.layer2]]
    names = {p: n for n, p in m.named_parameters()}
    got = [sorted(names[p] for p in st) for st in params]
    assert all(n.startswith(("model.layer4.", "model.conv_seg.")) for n in got[0])
    assert all(n.startswith("model.layer3.") for n in got[1])
    assert all(n.startswith("model.layer2.") for n in got[2])
    assert all(n.startswith(("model.layer1.", "model.conv1.", "model.bn1.")) for n in got[3])
    flat = [p for st in params for p in st]
    assert len(flat) == len(set(flat)) == sum(1 for p in m.parameters() if p.requires_grad)
    # layer4 holds most of the gradient bytes: the bucket overlapped longest
    sizes = [sum(p.numel() for p in st) for st in params]
    assert sizes[0] > 0.7 * sum(sizes) and sizes[3] < 0.02 * sum(sizes)


def test_backward_stages_two_backbones():
    import multimodal_alzheimer_amd as M
    from tests import _golden as G
    m = M.PET_MRI_ResNet_Fusion(G.anat_hparams(10, fl_gamma=2))
    bounds, params = backward_stages(m)
    assert [len(b) for b in bounds] == [2, 2, 2]
    names = {p: n for n, p in m.named_parameters()}
    head = [names[p] for p in params[0] if not names[p].startswith(("model_pet", "model_mri"))]
    assert any(n.startswith("stage2out") for n in head)
    assert any(n.startswith("reduce_dim_pet") for n in head)
    last = [names[p] for p in params[3]]
    assert any(n.startswith("model_pet.model.conv1") for n in last)
    assert any(n.startswith("model_mri.model.layer1") for n in last)


def _worker(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank,
                            world_size=world)
    m = _Net()
    bounds, params = m.stages()
    red = GradAllReduce(m.parameters(), bucket_mb=None, stages=params)
    assert len(red.buckets) == 4 and red.stage_buckets == [[0], [1], [2], [3]]
    x, y = _data()
    sl = slice(3 * rank, 3 * rank + 3)
    sb = StagedBackward(bounds, params)
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        sb.arm()
        loss = nn.functional.cross_entropy(m(x[sl]), y[sl])
        sb.disarm()
        red.defer = True                  # as in a capture: hooks (if any ran) only count
        for k in range(sb.n):
            sb.run(k, loss)
            red.launch_stage(k)
        red.defer = False
        red.finish()
    torch.save({k: p.grad.clone() for k, p in m.named_parameters()}, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_staged_allreduce_world2_equals_mean_of_ranks():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_worker, args=(world, os.path.join(td, "init"), os.path.join(td, "g")),
                 nprocs=world, join=True)
        got = [torch.load(os.path.join(td, f"g.{r}"), weights_only=True) for r in range(world)]
    x, y = _data()
    per = []
    for r in range(world):
        m = _Net()
        sl = slice(3 * r, 3 * r + 3)
        nn.functional.cross_entropy(m(x[sl]), y[sl]).backward()
        per.append({k: p.grad for k, p in m.named_parameters()})
    for k in per[0]:
        mean = (per[0][k] + per[1][k]) / 2
        for r in range(world):
            torch.testing.assert_close(got[r][k], mean, rtol=1e-6, atol=1e-7)
