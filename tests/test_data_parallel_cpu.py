"""Data-parallel path on CPU with the gloo backend, world_size 2 (the same code runs over
RCCL on GPUs): bucketed asynchronous gradient all-reduce == mean of per-rank gradients ==
the single-process gradient of the concatenated batch; sample-pair sharding is a disjoint
cover of the dataset."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn

from multimodal_alzheimer_amd.data_parallel import (GradAllReduce, broadcast_module_state,
                                                    shard_indices)


def _model():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(16, 64), nn.ReLU(), nn.Linear(64, 64), nn.Tanh(),
                         nn.Linear(64, 3))


def _data():
    g = torch.Generator().manual_seed(1)
    return torch.randn(8, 16, generator=g), torch.randint(0, 3, (8,), generator=g)


def _worker(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank,
                            world_size=world)
    m = _model()
    red = GradAllReduce(m.parameters(), bucket_mb=0.004)   # several tiny buckets
    assert len(red.buckets) > 1
    x, y = _data()
    idx = shard_indices(8, rank, world, shuffle=False)
    for _ in range(2):                                       # hooks re-arm every step
        m.zero_grad(set_to_none=True)
        nn.functional.cross_entropy(m(x[idx]), y[idx]).backward()
        red.finish()
    if rank == 0:
        torch.save({k: p.grad.clone() for k, p in m.named_parameters()}, out_file)
    dist.barrier()
    dist.destroy_process_group()


def test_grad_allreduce_matches_full_batch():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        init_file = os.path.join(td, "init")
        out_file = os.path.join(td, "grads.pt")
        mp.spawn(_worker, args=(world, init_file, out_file), nprocs=world, join=True)
        got = torch.load(out_file, weights_only=True)
    m = _model()
    x, y = _data()
    nn.functional.cross_entropy(m(x), y).backward()   # mean over 8 == mean of 2 shard means
    for k, p in m.named_parameters():
        torch.testing.assert_close(got[k], p.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,world", [(10, 2), (8, 4), (7, 8), (1946, 8)])
def test_shard_indices_cover(n, world):
    shards = [shard_indices(n, r, world, epoch=3) for r in range(world)]
    assert len({len(s) for s in shards}) == 1
    flat = [i for s in shards for i in s]
    assert set(flat) == set(range(n))
    assert len(flat) == -(-n // world) * world
    assert shard_indices(n, 0, world, epoch=3) == shards[0]
    assert shard_indices(n, 0, world, epoch=4) != shards[0] or n < 3


def _bcast_worker(rank, world, init_file, out_file):
    dist.init_process_group("gloo", init_method=f"file://{init_file}", rank=rank,
                            world_size=world)
    torch.manual_seed(100 + rank)                      # deliberately different replicas
    m = nn.Sequential(nn.Linear(4, 8), nn.BatchNorm1d(8))
    m[1].running_mean.fill_(float(rank))
    broadcast_module_state(m)
    torch.save({k: v.clone() for k, v in m.state_dict().items()}, f"{out_file}.{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_module_state_makes_replicas_identical():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        mp.spawn(_bcast_worker, args=(world, os.path.join(td, "init"), os.path.join(td, "sd")),
                 nprocs=world, join=True)
        sds = [torch.load(os.path.join(td, f"sd.{r}"), weights_only=True) for r in range(world)]
    for k in sds[0]:
        assert torch.equal(sds[0][k], sds[1][k]), k
    assert torch.equal(sds[1]["1.running_mean"], torch.zeros(8))


def test_bucket_slices_are_256_byte_aligned():
    """Odd-sized parameters (a 2-float bias) must not misalign the slices after them: torch's
    fused Adam takes its scalar path when any gradient is unaligned (data_parallel.py)."""
    with tempfile.TemporaryDirectory() as d:
        dist.init_process_group("gloo", init_method=f"file://{d}/init", rank=0, world_size=1)
        try:
            m = nn.Sequential(nn.Linear(7, 2), nn.Linear(2, 3), nn.Linear(3, 64))
            red = GradAllReduce(m.parameters(), bucket_mb=1.0)
            for bi, b in enumerate(red.buckets):
                base = red.flats[bi].data_ptr()   # device allocations are >= 256-B aligned
                for p in b:
                    v = red._views[p]
                    assert (v.data_ptr() - base) % 256 == 0
                    assert v.shape == p.shape
            for flat in red.flats:
                assert not flat.any()       # pad lanes start (and stay) zero
            red.remove()
        finally:
            dist.destroy_process_group()
