"""bench.py's N > 1 launch modes at world size 2 on BASELINE config 3/4's model
(PET_MRI_ResNet_Fusion: PET + MRI ResNet-10 x2 + MLP head, focal loss) and on config 5's
(Tri_ResNet_Tabular_Fusion: MRI ResNet-34 + PET ResNet-18 + tabular MLP), SURVEY.md §8(e).

Two processes share the test box's one GPU (RCCL refuses two ranks on one device, so the
collective is gloo over the same CUDA tensors); everything else is the benched path:
``GraphedTrainStep(reducer=GradAllReduce(...), collectives=mode)`` for
  * "staged" (one of the modes bench.py's "auto" default probes at N > 1): the backward replayed as four captured graphs
    (head + layer4 | layer3 | layer2 | layer1 + stem of both backbones), each stage's bucket
    all-reduced on the side stream while the next graph replays;
  * "after": forward + backward in one graph, every bucket all-reduced after it.
Each rank trains on its own shard (fp32, 32^3, 2 pairs per rank) for 3 replays.  Checked:
  * every rank's averaged gradient of replay 3 == the mean of the two per-replica
    gradients computed in one process from the same pre-replay weights (1e-5 relative);
  * each replica's replay-3 logits == the CPU oracle (oracle ResNetPairFusionRef / TriResNetTabularRef) on that
    replica's shard at the same weights (1e-4, argmax exact);
  * replays 1-3 are bit-identical (losses, parameters, BN running statistics) to eager
    steps of an identical model with the eager hook-driven all-reduce.
"""
import copy
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"
N_PER_RANK, SIZE, STEPS, WARM = 2, 32, 3, 2


def _build(kind, product):
    from tests.test_fusion_configs_gpu import _hp, _pair, _three
    return (_pair if kind == "pair" else _three)(_hp(kind), product)


def _model(kind):
    from tests import _golden as G
    from tests.test_fusion_configs_gpu import _live
    ref = _build(kind, False)
    G.load_prng_weights(ref, 81)
    _live(ref)
    m = _build(kind, True)
    m.load_state_dict(ref.state_dict())
    return m


def _batches(rank, kind):
    from tests.test_fusion_configs_gpu import _batch
    out = []
    for i in range(STEPS):
        b = _batch(2 * N_PER_RANK, SIZE, 90 + 3 * i, kind == "three")
        sl = slice(N_PER_RANK * rank, N_PER_RANK * (rank + 1))
        out.append({k: v[sl] for k, v in b.items()})
    return out


def _worker(rank, world, port, out_dir, mode, kind):
    import torch.distributed as dist
    from multimodal_alzheimer_amd.data_parallel import GradAllReduce
    from multimodal_alzheimer_amd.graph_step import GraphedTrainStep, backward_stages
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        a = _model(kind).to(DEV)
        b = copy.deepcopy(a)
        batches = [{k: v.to(DEV) for k, v in bt.items()} for bt in _batches(rank, kind)]

        # graph-replayed (the benched mode)
        opt_a = a.configure_optimizers()
        if mode == "staged":
            red_a = GradAllReduce(a.parameters(), bucket_mb=None,
                                  stages=backward_stages(a)[1])
        else:
            red_a = GradAllReduce(a.parameters(), bucket_mb=4.0)
        gs = GraphedTrainStep(a, opt_a, batches[0], warmup=WARM, reducer=red_a,
                              collectives=mode)
        losses_a = []
        for i in range(STEPS):
            if i == STEPS - 1:
                torch.cuda.synchronize()
                pre = {k: v.detach().cpu().clone() for k, v in a.state_dict().items()}
            out = gs(batches[i])
            losses_a.append(out["loss"].clone())
        torch.cuda.synchronize()
        grads = {k: p.grad.detach().cpu().clone() for k, p in a.named_parameters()}
        logits = out["outputs"].detach().cpu().clone()

        # eager twin: hook-driven all-reduce, same optimizer configuration
        opt_b = b.configure_optimizers()
        for grp in opt_b.param_groups:
            grp["capturable"] = True
            grp["lr"] = torch.tensor(float(grp["lr"]), device=DEV)
        red_b = GradAllReduce(b.parameters(), bucket_mb=4.0)

        def eager(batch):
            opt_b.zero_grad(set_to_none=True)
            o = b.general_step(batch, 0, "train")
            o["loss"].backward()
            red_b.finish()
            opt_b.step()
            return o["loss"].detach().clone()

        for _ in range(WARM):
            eager(batches[0])
        losses_b = [eager(batches[i]) for i in range(STEPS)]
        torch.cuda.synchronize()
        same_loss = [bool(torch.equal(x, y)) for x, y in zip(losses_a, losses_b)]
        diff = [k for (k, x), (_, y) in zip(a.state_dict().items(), b.state_dict().items())
                if not torch.equal(x, y)]
        torch.save({"pre": pre, "grads": grads, "logits": logits, "same_loss": same_loss,
                    "diff": diff, "final": {k: v.detach().cpu() for k, v in a.state_dict().items()}},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["pair", "three"])
@pytest.mark.parametrize("mode", ["staged", "after"])
def test_graphed_dp_world2_fusion(tmp_path, mode, kind):
    from oracle import models_ref  # noqa: F401  (the checker only)
    ctx = mp.get_context("spawn")
    port = (29100 + os.getpid() % 400 + (0 if mode == "staged" else 450) +
            (0 if kind == "pair" else 900))
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), mode, kind))
             for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=150)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    for r in range(2):
        assert all(res[r]["same_loss"]), (r, res[r]["same_loss"])
        assert not res[r]["diff"], (r, res[r]["diff"][:5])
    for k in res[0]["pre"]:
        if "running" in k or "num_batches" in k:
            continue                              # BN statistics are per replica
        # the parameters stay identical across replicas (averaged gradients, same Adam)
        assert torch.equal(res[0]["pre"][k], res[1]["pre"][k]), k
        assert torch.equal(res[0]["final"][k], res[1]["final"][k]), k

    per = []
    for r in range(2):
        batch = _batches(r, kind)[STEPS - 1]
        m = _build(kind, True)
        m.load_state_dict(res[0]["pre"])
        m = m.to(DEV)
        o = m.general_step({k: v.to(DEV) for k, v in batch.items()}, 0, "train")
        o["loss"].backward()
        torch.cuda.synchronize()
        per.append({k: p.grad.detach().cpu() for k, p in m.named_parameters()})
        ref = _build(kind, False)
        ref.load_state_dict(res[0]["pre"])
        rr = ref.general_step(batch, 0, "train")
        got, exp = res[r]["logits"].numpy(), rr["outputs"].detach().numpy()
        assert np.abs(got - exp).max() <= 1e-4, (r, np.abs(got - exp).max())
        assert (got.argmax(1) == exp.argmax(1)).all()
    n = 0
    for k in per[0]:
        mean = (per[0][k] + per[1][k]) / 2
        scale = max(mean.abs().max().item(), 1e-12)
        for r in range(2):
            err = (res[r]["grads"][k] - mean).abs().max().item()
            assert err <= 1e-5 * scale + 1e-9, (mode, r, k, err, scale)
        n += 1
    assert n > 50
    assert any(not torch.equal(per[0][k], per[1][k]) for k in per[0]), "shards identical"
