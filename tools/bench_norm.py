"""Per-scan MRI quantile min-max normalisation (dataloader.py:244-270) on device vs the
reference's CPU statements (oracle/preprocess_ref.py, torch f64) on the same scans.

    python tools/bench_norm.py [--batch 8] [--size 128]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import preprocess  # noqa: E402
from oracle import preprocess_ref as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    b, s = a.batch, a.size
    g = torch.Generator().manual_seed(0)
    x = torch.randint(0, 1000, (b, s, s, s), generator=g).double()
    zz = torch.arange(s, dtype=torch.float64) - s / 2
    ball = (zz[:, None, None] ** 2 + zz[None, :, None] ** 2 + zz[None, None, :] ** 2) <= (0.45 * s) ** 2
    m = ball.double().expand(b, s, s, s).contiguous()
    xd, md = x.cuda(), m.cuda()
    for _ in range(2):
        preprocess.mri_per_scan_minmax(xd, md, 0.99)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        out = preprocess.mri_per_scan_minmax(xd, md, 0.99)
    torch.cuda.synchronize()
    tg = (time.perf_counter() - t0) / a.reps
    t0 = time.perf_counter()
    ref, _, _ = P.mri_minmax_ref(x[0].clone(), m[0], 0.99)
    tc = time.perf_counter() - t0
    ok = torch.equal(out[0].cpu(), ref)
    print(f"batch {b} x {s}^3: GPU {tg * 1e3:.2f} ms ({b / tg:.0f} scans/s), reference CPU "
          f"statements {tc * 1e3:.1f} ms/scan ({1 / tc:.1f} scans/s, {torch.get_num_threads()} "
          f"threads), bit-exact: {ok}")


if __name__ == "__main__":
    main()
