"""Per-conv timing of the implicit-GEMM kernels on the ResNet-10 @128^3 B=8 geometry
(forward, dgrad, wgrad), with MIOpen (torch F.conv3d, channels_last_3d bf16) beside it
for orientation.  Usage: python tools/bench_conv.py [--reps N] [--no-miopen]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import _lib as L  # noqa: E402
from multimodal_alzheimer_amd import volume_ops as V  # noqa: E402

CL = torch.channels_last_3d
# name, (N, Ci, D), Co, k, stride, pad, dil
LAYERS = [
    ("stem", (8, 1, 128), 64, 7, 2, 3, 1),
    ("l1c", (8, 64, 32), 64, 3, 1, 1, 1),
    ("l2c1", (8, 64, 32), 128, 3, 2, 1, 1),
    ("l2c2", (8, 128, 16), 128, 3, 1, 1, 1),
    ("l2ds", (8, 64, 32), 128, 1, 2, 0, 1),
    ("l3c1", (8, 128, 16), 256, 3, 1, 2, 2),
    ("l3c2", (8, 256, 16), 256, 3, 1, 2, 2),
    ("l3ds", (8, 128, 16), 256, 1, 1, 0, 1),
    ("l4c1", (8, 256, 16), 512, 3, 1, 4, 4),
    ("l4c2", (8, 512, 16), 512, 3, 1, 4, 4),
    ("l4ds", (8, 256, 16), 512, 1, 1, 0, 1),
]


def timeit(fn, reps):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--no-miopen", action="store_true")
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--layers", default="", help="comma-separated subset of layer names")
    ap.add_argument("--tag", default="", help="label printed on every row")
    args = ap.parse_args()
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    code = L.dtype_code(dt)
    lib = L.load()
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'layer':6s} {'GFLOP':>7s} | {'fwd us':>8s} {'TF/s':>6s} | {'dgrad us':>8s} {'TF/s':>6s} |"
          f" {'wgrad us':>8s} {'TF/s':>6s} | {'miopen f/d/w TF/s':>20s}")
    pick = set(args.layers.split(",")) if args.layers else None
    for name, (n, ci, s), co, k, st, p, dl in LAYERS:
        if pick is not None and name not in pick:
            continue
        x = torch.randn((n, ci, s, s, s), device="cuda").to(dt)
        if ci > 1:
            x = x.contiguous(memory_format=CL)
        w = (torch.randn((co, ci, k, k, k), device="cuda") * 0.05)
        d = V.conv_desc(tuple(x.shape), tuple(w.shape), (st,) * 3, (p,) * 3, (dl,) * 3)
        flop = 2.0 * n * d.do_ * d.ho * d.wo * co * ci * k ** 3
        src = x
        if ci == 1:
            src = torch.empty(lib.mmad_conv_unfolded_elems(d), dtype=dt, device="cuda")
            xf = x.float().contiguous()
            L.call("mmad_conv_unfold_input", d, L.F32, L.ptr(xf), code, L.ptr(src), L.stream())
        wp = V.pack_weight(d, code, w, dt, False)
        y = torch.empty((n, co, d.do_, d.ho, d.wo), dtype=dt, device="cuda", memory_format=CL)
        stats = torch.empty((lib.mmad_conv3d_stats_rows(d, code), 2, co), device="cuda")
        t_f = timeit(lambda: L.call("mmad_conv3d_fwd", d, code, L.ptr(src), L.ptr(wp), None,
                                    L.ptr(y), L.ptr(stats), L.stream()), args.reps)
        gy = torch.randn_like(y)
        t_d = float("nan")
        if ci > 1:
            wpt = V.pack_weight(d, code, w, dt, True)
            dx = torch.empty_like(x)
            t_d = timeit(lambda: L.call("mmad_conv3d_dgrad", d, code, L.ptr(gy), L.ptr(wpt),
                                        L.ptr(dx), L.stream()), args.reps)
        ws = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, code) + 3) // 4, device="cuda")
        dw = torch.empty_like(w)
        t_w = timeit(lambda: L.call("mmad_conv3d_wgrad", d, code, L.ptr(src), L.ptr(gy),
                                    L.ptr(dw), None, L.ptr(ws), L.stream()), args.reps)
        mio = ""
        if not args.no_miopen:
            xm = x.detach().requires_grad_(ci > 1)
            wm = w.to(dt).contiguous(memory_format=CL).requires_grad_(True)
            f = lambda: F.conv3d(xm, wm, None, st, p, dl)  # noqa: E731
            tm_f = timeit(f, max(3, args.reps // 4))
            yo = f()
            g = torch.randn_like(yo)
            tm_b = timeit(lambda: torch.autograd.grad(f(), [wm] + ([xm] if ci > 1 else []), g),
                          max(3, args.reps // 4)) - tm_f
            mio = f"{flop / tm_f / 1e12:6.0f} / bwd {flop * (2 if ci > 1 else 1) / tm_b / 1e12:5.0f}"
        tot["fwd"] += t_f
        tot["dgrad"] += 0 if t_d != t_d else t_d
        tot["wgrad"] += t_w
        print(f"{args.tag}{name:6s} {flop / 1e9:7.1f} | {t_f * 1e6:8.1f} {flop / t_f / 1e12:6.0f} | "
              f"{t_d * 1e6:8.1f} {flop / t_d / 1e12:6.0f} | {t_w * 1e6:8.1f} {flop / t_w / 1e12:6.0f} | {mio}")
    print("totals ms:", {k: round(v * 1e3, 3) for k, v in tot.items()},
          "sum", round(sum(tot.values()) * 1e3, 3))


if __name__ == "__main__":
    main()
