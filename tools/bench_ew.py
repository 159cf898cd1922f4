"""Timing of the bandwidth-bound (non-conv) ops at the ResNet-10 @128^3 B=8 shapes, with the
effective HBM rate of each (algorithmic bytes / time).  Usage: python tools/bench_ew.py [--tag T]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import volume_ops as V  # noqa: E402

CL = torch.channels_last_3d


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def vol(n, c, s, dt=torch.bfloat16):
    return torch.randn((n, c, s, s, s), device="cuda").to(dt).contiguous(memory_format=CL)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    rows = []
    # stem: bn1 + relu + maxpool(3,2,1) on (8,64,64^3)
    bn = torch.nn.BatchNorm3d(64).cuda()
    y = vol(8, 64, 64)
    parts = None
    fwd = lambda: V.batchnorm_relu_maxpool(y, bn, parts, 3, 2, 1)  # noqa: E731
    t = timeit(fwd)
    yb = y.numel() * 2
    rows.append(("bnpool fwd (stem)", t, yb + yb / 8 * 2 + yb / 16))
    yr = y.detach().requires_grad_(True)
    out = V.batchnorm_relu_maxpool(yr, bn, parts, 3, 2, 1)
    g = torch.randn_like(out)
    tb = timeit(lambda: torch.autograd.grad(out, yr, g, retain_graph=True))
    rows.append(("bnpool bwd (stem, reduce+apply)", tb, g.numel() * 2 * 2 + yb / 16 * 2 + yb * 2))
    # layer1: bn + relu, bn + residual + relu at (8,64,32^3)
    bn1 = torch.nn.BatchNorm3d(64).cuda()
    x = vol(8, 64, 32)
    r = vol(8, 64, 32)
    xb = x.numel() * 2
    rows.append(("bn+relu fwd (l1)", timeit(lambda: V.batchnorm_act(x, bn1, None, relu=True)), 3 * xb))
    rows.append(("bn+res+relu fwd (l1)",
                 timeit(lambda: V.batchnorm_act(x, bn1, None, relu=True, res=r)), 4 * xb))
    xr = x.detach().requires_grad_(True)
    o = V.batchnorm_act(xr, bn1, None, relu=True)
    go = torch.randn_like(o)
    rows.append(("bn+relu bwd (l1)", timeit(lambda: torch.autograd.grad(o, xr, go, retain_graph=True)),
                 6 * xb))
    for name, t, b in rows:
        print(f"{a.tag}{name:34s} {t * 1e6:8.1f} us  {b / t / 1e12:6.2f} TB/s (algorithmic {b / 1e6:.0f} MB)")


if __name__ == "__main__":
    main()
