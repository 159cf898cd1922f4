"""Critical-path cost of one small RCCL all-reduce between two dependent kernels on the
main stream (what the last gradient bucket of a staged step costs), async_op=True + wait()
(ProcessGroupNCCL's internal stream: two cross-stream hops) against async_op=False:

    torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/ar_latency.py
"""
import os
import time

import torch
import torch.distributed as dist


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    x = torch.zeros(1 << 20, device="cuda")
    y = torch.zeros(1 << 18, device="cuda")
    for mode in ("none", "async", "sync", "async", "sync"):
        for rep in range(2):
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(50):
                y.add_(1.0)
                if mode == "async":
                    dist.all_reduce(x, op=dist.ReduceOp.AVG, async_op=True).wait()
                elif mode == "sync":
                    dist.all_reduce(x, op=dist.ReduceOp.AVG)
                y.add_(1.0)
            torch.cuda.synchronize()
            if rep:
                print(f"{mode:6s} {(time.perf_counter() - t) / 50 * 1e6:.1f} us per iteration",
                      flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
