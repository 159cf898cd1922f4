"""Data parallelism on the real model at world size 2.

Two processes share the one GPU of the test box (RCCL refuses two ranks on one device, so
the collective is gloo over the same CUDA tensors; the product path is otherwise the one
bench.py runs: ``GradAllReduce`` with the in-place gradient slots, the conv weight gradients
written by the wgrad kernel straight into 256-byte-aligned bucket slices, BN / head
gradients copied in and out, buckets reduced from post-accumulate-grad hooks on the side
stream).  Each rank trains on its own shard of the batch.  Checked against separate
single-process runs of the same shards:
  * every rank's averaged gradient equals the mean of the two per-replica gradients;
  * each replica's logits match the CPU oracle on that replica's shard (per-replica BN).
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hparams():
    from tests import _golden as G
    return G.anat_hparams(10, linear_out=[32])


def _shard(rank):
    from tests import _golden as G
    b = G.batch_for((4, 32, 32, 32), 2, 61)
    return {k: v[2 * rank: 2 * rank + 2] for k, v in b.items()}


def _model():
    import multimodal_alzheimer_amd as M
    from tests import _golden as G
    m = M.Anat_CNN(_hparams())
    G.load_prng_weights(m, 60)
    with torch.no_grad():                     # live logits (the head ends in a ReLU)
        m.model.conv_seg[-2].bias.fill_(0.5)
    return m


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from multimodal_alzheimer_amd.data_parallel import GradAllReduce
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        m = _model().to(DEV)
        red = GradAllReduce(m.parameters(), bucket_mb=4.0)
        batch = {k: v.to(DEV) for k, v in _shard(rank).items()}
        for step in range(2):                 # fresh gradients (set_to_none) each step
            m.zero_grad(set_to_none=True)
            out = m.general_step(batch, 0, "train")
            out["loss"].backward()
            red.finish()
            torch.cuda.synchronize()
        conv = m.model.layer4[0].conv2.weight
        slot_adopted = conv.grad.data_ptr() == conv._mmad_grad_view.data_ptr()
        torch.save({"grads": {k: p.grad.detach().cpu() for k, p in m.named_parameters()},
                    "logits": out["outputs"].detach().cpu(), "slot": slot_adopted},
                   os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_world2_real_model(tmp_path):
    from oracle import models_ref
    ctx = mp.get_context("spawn")
    port = 29600 + os.getpid() % 300
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path))) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    assert res[0]["slot"] and res[1]["slot"], "conv gradient not produced in its bucket slice"

    # per-replica references: the same model, one process, one shard each, two steps of
    # gradients from identical weights (no optimizer step in between)
    per = []
    for rank in range(2):
        m = _model().to(DEV)
        batch = {k: v.to(DEV) for k, v in _shard(rank).items()}
        for _ in range(2):
            m.zero_grad(set_to_none=True)
            out = m.general_step(batch, 0, "train")
            out["loss"].backward()
        torch.cuda.synchronize()
        per.append({k: p.grad.detach().cpu() for k, p in m.named_parameters()})
        # this replica's logits == the rank's logits == the CPU oracle on its shard
        ref = models_ref.AnatCNNRef(_hparams())
        ref.load_state_dict(_model().state_dict())
        r = ref.general_step(_shard(rank), 0, "train")
        got = res[rank]["logits"].numpy()
        assert np.abs(got - r["outputs"].detach().numpy()).max() <= 1e-4
        assert (got.argmax(1) == r["outputs"].detach().numpy().argmax(1)).all()
        assert torch.allclose(res[rank]["logits"], out["outputs"].detach().cpu(), atol=1e-6)
    for k in per[0]:
        mean = (per[0][k] + per[1][k]) / 2
        scale = max(mean.abs().max().item(), 1e-12)
        for rank in range(2):
            err = (res[rank]["grads"][k] - mean).abs().max().item()
            assert err <= 1e-5 * scale + 1e-9, (rank, k, err)
    assert any(not torch.equal(per[0][k], per[1][k]) for k in per[0]), "shards identical"
