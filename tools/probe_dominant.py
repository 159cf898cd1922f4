"""Launch only the bench's dominant kernel (layer4.0.conv2 forward, bf16, batch 8,
512->512, 3^3 dilation 4 at 16^3) -- or with ``--op wgrad`` that conv's weight gradient
(lattice_wgrad_kernel + slab reduce) -- a few times, for rocprofv3 --pmc passes:

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv \
        -- python3 tools/probe_dominant.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv \
        -- python3 tools/probe_dominant.py

then ``python tools/prof_summary.py traffic gpurun_out/pmc_fetch gpurun_out/pmc_write [wgrad]``.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import _lib, volume_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--op", default="fwd", choices=["fwd", "wgrad"])
    a = ap.parse_args()
    s = a.size // 8
    dtype = torch.bfloat16
    x = torch.randn((a.batch, 512, s, s, s), device="cuda", dtype=dtype).contiguous(
        memory_format=torch.channels_last_3d)
    w = torch.randn((512, 512, 3, 3, 3), device="cuda") * 0.02
    d = volume_ops.conv_desc(tuple(x.shape), tuple(w.shape), (1, 1, 1), (4, 4, 4), (4, 4, 4))
    dt = _lib.dtype_code(dtype)
    wp = volume_ops.pack_weight(d, dt, w, dtype, False)
    y = torch.empty_like(x)
    lib = _lib.load()
    stats = torch.empty((lib.mmad_conv3d_stats_rows(d, dt), 2, 512), device="cuda")
    # flush the 256 MiB on-die cache between launches so each one reads from HBM
    scrub = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")
    if a.op == "wgrad":
        gy = torch.randn_like(x)
        dw = torch.empty_like(w)
        ws = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, dt) + 3) // 4, device="cuda")
    for _ in range(a.reps):
        scrub.fill_(1)
        if a.op == "wgrad":
            _lib.call("mmad_conv3d_wgrad", d, dt, _lib.ptr(x), _lib.ptr(gy), _lib.ptr(dw), None,
                      _lib.ptr(ws), _lib.stream())
        else:
            _lib.call("mmad_conv3d_fwd", d, dt, _lib.ptr(x), _lib.ptr(wp), None, _lib.ptr(y),
                      _lib.ptr(stats), _lib.stream())
    torch.cuda.synchronize()
    print("ok", a.reps, "launches")


if __name__ == "__main__":
    main()
