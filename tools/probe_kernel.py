"""Run one conv pass of one ResNet-10 @128^3 layer (batch 8, bf16; c5* layers: config 5's
160^3 geometry) a few times, for rocprofv3 counter passes on a single kernel:

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... -d gpurun_out/pmc_x -o run \
        --output-format csv -- python3 tools/probe_kernel.py --layer l4c2 --op wgrad
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import _lib, volume_ops  # noqa: E402

# name: (cin, cout, size at 128^3 input, k, stride, pad, dil)
LAYERS = {
    "stem": (1, 64, 128, 7, 2, 3, 1),
    "l1c": (64, 64, 32, 3, 1, 1, 1),
    "l2c1": (64, 128, 32, 3, 2, 1, 1),
    "l3c1": (128, 256, 16, 3, 1, 2, 2),
    "l3c2": (256, 256, 16, 3, 1, 2, 2),
    "l4c1": (256, 512, 16, 3, 1, 4, 4),
    "l4c2": (512, 512, 16, 3, 1, 4, 4),
    # BASELINE config 5 (160^3 input): layer4 on 20^3 (lattice5.hip), layer3, layer1 at 40^3
    "c5l4c1": (256, 512, 20, 3, 1, 4, 4),
    "c5l4c2": (512, 512, 20, 3, 1, 4, 4),
    "c5l3c2": (256, 256, 20, 3, 1, 2, 2),
    "c5l1c": (64, 64, 40, 3, 1, 1, 1),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="l4c2", choices=sorted(LAYERS))
    ap.add_argument("--op", default="wgrad", choices=["fwd", "dgrad", "wgrad"])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stats", action="store_true", help="fwd: BN partial sums too")
    ap.add_argument("--relu", action="store_true",
                    help="operands ReLU'd (about half zeros, like a post-BN activation)")
    ap.add_argument("--raw", action="store_true",
                    help="stem: read the raw f64 volume (mmad_conv3d_*_raw, the bench's route)")
    ap.add_argument("--time", action="store_true",
                    help="print the median launch time (HIP events) instead of only running")
    a = ap.parse_args()
    ci, co, s, k, st, p, dl = LAYERS[a.layer]
    dtype = torch.bfloat16
    xs = (a.batch, ci, s, s, s)
    ws = (co, ci, k, k, k)
    d = volume_ops.conv_desc(xs, ws, (st,) * 3, (p,) * 3, (dl,) * 3)
    dt = _lib.dtype_code(dtype)
    lib = _lib.load()
    w = torch.randn(ws, device="cuda") * 0.02
    if ci == 1:
        raw = torch.rand(xs, device="cuda", dtype=torch.float64 if a.raw else torch.float32)
        x = torch.empty(lib.mmad_conv_unfolded_elems(d), dtype=dtype, device="cuda")
        _lib.call("mmad_conv_unfold_input", d, _lib.dtype_code(raw.dtype), _lib.ptr(raw), dt,
                  _lib.ptr(x), _lib.stream())
    else:
        x = torch.randn(xs, device="cuda", dtype=dtype).contiguous(
            memory_format=torch.channels_last_3d)
    y = torch.randn((a.batch, co, d.do_, d.ho, d.wo), device="cuda", dtype=dtype).contiguous(
        memory_format=torch.channels_last_3d)
    if a.relu:
        x.relu_()
        y.relu_()
    st = None
    if a.stats and a.op == "fwd":
        rows = lib.mmad_conv3d_stats_rows(d, dt)
        st = torch.empty((rows, 2, co), device="cuda")
    wp = volume_ops.pack_weight(d, dt, w, dtype, a.op == "dgrad") if a.op != "wgrad" else None
    if a.op == "wgrad":
        wsp = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, dt) + 3) // 4, device="cuda")
        dw = torch.empty(ws, device="cuda")
    times = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        if a.op == "fwd" and a.raw:
            _lib.call("mmad_conv3d_fwd_raw", d, _lib.dtype_code(raw.dtype), _lib.ptr(raw), dt,
                      _lib.ptr(wp), None, _lib.ptr(y), None if st is None else _lib.ptr(st),
                      _lib.stream())
        elif a.op == "wgrad" and a.raw:
            _lib.call("mmad_conv3d_wgrad_raw", d, _lib.dtype_code(raw.dtype), _lib.ptr(raw), dt,
                      _lib.ptr(y), _lib.ptr(dw), None, _lib.ptr(wsp), _lib.stream(), None)
        elif a.op == "fwd":
            _lib.call("mmad_conv3d_fwd", d, dt, _lib.ptr(x), _lib.ptr(wp), None, _lib.ptr(y),
                      None if st is None else _lib.ptr(st), _lib.stream())
        elif a.op == "dgrad":
            _lib.call("mmad_conv3d_dgrad", d, dt, _lib.ptr(y), _lib.ptr(wp), _lib.ptr(x),
                      _lib.stream())
        else:
            _lib.call("mmad_conv3d_wgrad", d, dt, _lib.ptr(x), _lib.ptr(y), _lib.ptr(dw), None,
                      _lib.ptr(wsp), _lib.stream())
        e1.record()
        times.append((e0, e1))
    torch.cuda.synchronize()
    if a.time:
        ts = sorted(x.elapsed_time(y) * 1e3 for x, y in times[1:])
        print(f"{a.layer} {a.op}{' stats' if st is not None else ''}"
              f"{' relu' if a.relu else ''} median {ts[len(ts) // 2]:.1f} us (min {ts[0]:.1f}, "
              f"{len(ts)} reps, lib {os.environ.get('MMAD_LIB_PATH', 'default')})")
    else:
        print("ok", a.layer, a.op, a.reps)


if __name__ == "__main__":
    main()
