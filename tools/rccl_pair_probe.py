"""Probe: can two RCCL ranks share the one GPU of a gpurun box?

Launched as `python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1
--master-port P tools/rccl_pair_probe.py`; both ranks bind cuda:0, run one all-reduce and one
broadcast over the "nccl" (= RCCL) backend, and rank 0 prints one JSON line with the result.
If RCCL refuses a duplicated device the ranks exit with its error (no retry)."""
import json
import os

import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    x = torch.full((1 << 20,), float(rank + 1), device="cuda")
    dist.all_reduce(x)
    b = torch.arange(8, device="cuda", dtype=torch.float32) * (rank + 1)
    dist.broadcast(b, src=0)
    torch.cuda.synchronize()
    ok = bool((x == world * (world + 1) / 2).all()) and bool((b == torch.arange(8, device="cuda")).all())
    flags = torch.tensor([1 if ok else 0], device="cuda")
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    if rank == 0:
        print(json.dumps({"probe": "rccl_two_ranks_one_gpu", "world": world,
                          "ok": bool(flags.item() == 1)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
