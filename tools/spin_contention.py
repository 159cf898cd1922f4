"""How much does the captured ResNet-10 step (config 2, 8 x 1 x 128^3, bf16) lose when some
CUs are taken by another kernel for part of the backward -- as RCCL's ring kernels take them
when the all-reduce overlaps the backward (graph_step "staged")?  A spinner (tools/spin/
spin.hip: k blocks of 256 threads holding 64 KiB LDS each, so none of our 160-KiB blocks fits
beside them) runs on a side stream for `usec` at each step start; the step replays on the
main stream.

    hipcc --offload-arch=gfx950 -shared -fPIC -o tools/spin/libspin.so tools/spin/spin.hip
    python tools/spin_contention.py
"""
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
import multimodal_alzheimer_amd as M  # noqa: E402
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep  # noqa: E402


def main():
    lib = ctypes.CDLL(os.path.join(REPO, "tools", "spin", "libspin.so"))
    lib.spin_launch.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")
    torch.manual_seed(15)
    model = M.Anat_CNN(bench.hparams("bf16")).cuda()
    opt = model.configure_optimizers()
    g = torch.Generator(device="cuda").manual_seed(1000)
    batch = {"mri": torch.rand((8, 128, 128, 128), device="cuda", dtype=torch.float64, generator=g),
             "label": torch.randint(0, 2, (8,), device="cuda", generator=g)}
    gs = GraphedTrainStep(model, opt, batch, warmup=3)
    side = torch.cuda.Stream()
    res = []
    for blocks, usec in [(0, 0), (8, 1500), (16, 1500), (32, 1500), (16, 3000), (0, 0)]:
        for _ in range(3):
            gs()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        steps = 20
        for _ in range(steps):
            if blocks:
                side.wait_stream(torch.cuda.current_stream())
                lib.spin_launch(blocks, usec, ctypes.c_void_p(side.cuda_stream),
                                ctypes.c_void_p(sink.data_ptr()))
            gs()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / steps * 1e3
        res.append({"spin_blocks": blocks, "spin_us": usec, "ms_per_step": round(ms, 4),
                    "vol_s": round(8 / ms * 1e3, 1)})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
