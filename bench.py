"""Throughput benchmark of the 3D-volume training hot path on MI355X.

BASELINE.json metric: "volumes/sec fwd+bwd, 3D-ResNet-10 @128^3 bf16, 1/2/4/8 MI355X;
% HBM roofline".  Workload (BASELINE config 2): MRI-only Anat_CNN ResNet-10, synthetic
1x128^3 volumes (uniform[0,1) like min-max-normalised MRI, resident in HBM as float64 as
the reference DataLoader delivers them), batch 8 per GPU, weighted CE, bf16 compute with
fp32 master weights.  One step = general_step (forward + loss) + backward + gradient
all-reduce (N>1) + Adam; all parameters trainable (lr_pretrained set).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...      (one process per GPU, RCCL)

The step is captured once as HIP graphs and replayed (``--eager`` launches it from Python
every step).  Under torchrun (``--collectives``):
  * ``staged``: the backward captured as four graphs split at the backbone stages (head +
    layer4 | layer3 | layer2 | layer1 + stem, graph_step "staged"); after each replay that
    stage's gradient bucket is all-reduced over RCCL on a side stream while the next
    stage's graph runs, then the captured Adam;
  * ``staged1``: the same with one cut (head + layer4 + layer3 | the rest): one boundary,
    ~4 MB left exposed;
  * ``after``: one forward + backward graph, every all-reduce after it;
  * ``auto`` (default): each of the three is captured in turn and timed over a few replays
    during warm-up (max over ranks), and the fastest is kept -- overlap pays only while the
    RCCL kernels' CUs cost the backward less than the all-reduce it hides, which depends on
    the node (tools/spin_contention.py: 16 CUs held through a step cost ~0.5 ms);
  * ``inside`` (``--graph``): the all-reduces captured inside the step graph.
Rank 0 prints one JSON line.
``roofline`` times the dominant kernel (layer4.0.conv2 forward, the lattice conv; ``frac`` on
the MACs it executes, ``dense_frac`` on the dense count) and, under ``kernels``, also that
conv's weight gradient (the largest single launch) with HIP events recorded around each of
their launches, on the stream they run on -- inside the timed region when eager, over eager
steps just before the capture when graph-replayed;
``cpu_baseline`` times the CPU oracle (torch fp32, the reference path) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import multimodal_alzheimer_amd as M  # noqa: E402
from multimodal_alzheimer_amd import _lib, volume_ops  # noqa: E402
from multimodal_alzheimer_amd.graph_step import (DEFAULT_CUTS,  # noqa: E402
                                                  GraphedTrainStep, backward_stages)
from multimodal_alzheimer_amd.data_parallel import (GradAllReduce,  # noqa: E402
                                                    broadcast_module_state)

W2 = [0.20314960629921264, 0.7968503937007874]
# fwd+bwd ResNet-10 @128^3, dense MACs of the ops the step runs (413.2 GFLOP,
# i.e. without the stem's input gradient, which the step never computes -- the 424.7 of
# rounds 1-5 counted it)
FLOP_PER_VOL = {128: 413.2e9}
M2_BYTES_PER_VOL = 1.163e9               # unfused eager byte model
PEAK_BF16 = 2.5e15                       # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32 = 157.3e12
PEAK_HBM = 8.0e12
# --collectives modes with a graph_step form: (graph_step collectives, backward cuts)
DP_MODES = {"staged": ("staged", DEFAULT_CUTS), "staged1": ("staged", ("layer3",)),
            "after": ("after", DEFAULT_CUTS)}


def hparams(precision):
    return {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": precision,
            "loss_class_weights": torch.tensor(W2, dtype=torch.float64)}


def dominant_desc(batch, size):
    """layer4.0.conv2 (512->512, 3^3, dilation 4, 16^3 at 128^3 input): the largest conv of
    the step (its forward, dgrad and weight gradient are the three largest launches)."""
    s = size // 8
    d = volume_ops.conv_desc((batch, 512, s, s, s), (512, 512, 3, 3, 3), (1, 1, 1),
                             (4, 4, 4), (4, 4, 4))
    return volume_ops._desc_tuple(d), 2.0 * batch * s ** 3 * 512 * 512 * 27


def _traffic(op):
    tf = os.path.join(REPO, "profiles", f"traffic_layer4_conv2_{op}.json")
    if not os.path.exists(tf):
        return None
    with open(tf) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def kernel_roofline(op, events, batch, size, dtype, where):
    """One launch record of layer4.0.conv2 (``op`` "fwd": lattice_zp_kernel; "wgrad":
    lattice_wgrad_kernel + its slab reduce, one mmad_conv3d_wgrad call): average duration
    from the HIP event pairs volume_ops recorded around each call on its own stream.

    The residue-class kernels skip the MACs that land in the zero padding: per dimension 10
    of the 12 (position, tap) pairs of a 4-point sub-lattice are real.  Both kernels skip
    them in all three dimensions at compile time ((10/12)^3 = 57.9 % of the dense MACs run;
    the weight gradient's plane loop is unrolled by the 4 planes of a sub group, so its
    z-padding taps have no MFMAs either -- rounds 4-5 priced it at (10/12)^2 by mistake).
    ``frac`` = executed FLOP/s / peak (what the MFMA pipes did); ``dense_frac`` prices the
    dense count, as cuDNN / MIOpen report conv FLOPs, and can exceed 1."""
    _, flops = dominant_desc(batch, size)
    if not events:
        return None
    sec = sum(a.elapsed_time(b) for a, b in events) / len(events) / 1e3
    peak = PEAK_BF16 if dtype == torch.bfloat16 else PEAK_F32
    s = size // 8
    lattice = s == 16 and dtype == torch.bfloat16
    executed = flops * ((10 / 12) ** 3 if lattice else 1.0)
    vox = batch * s ** 3 * 512 * 2                         # one bf16 activation tensor
    wbytes = 512 * 512 * 27 * (2 if op == "fwd" else 4)    # bf16 packed in / fp32 dW out
    algo = 2 * vox + wbytes                                # X + Y (or dY) + weights
    name = ("lattice_zp_kernel" if lattice else "igemm_kernel") if op == "fwd" else \
        ("lattice_wgrad_kernel + wgrad_reduce_t_kernel" if lattice else "wgrad_kernel + reduce")
    return {"kernel": f"{name} layer4.0.conv2 {op} (512->512, 3^3 dil 4, {batch}x{s}^3)",
            "bound": "mfma", "achieved": executed / sec / 1e12, "peak": peak / 1e12,
            "unit": "TFLOP/s", "frac": executed / sec / peak, "traffic": _traffic(op),
            "algorithmic_bytes": algo,
            "flop_per_launch": flops, "executed_flop_per_launch": executed,
            "executed_frac": executed / sec / peak, "dense_frac": flops / sec / peak,
            "avg_launch_ms": sec * 1e3, "launches": len(events), "probe": where}


def dominant_kernel_roofline(events, wevents, batch, size, dtype, where="timed region"):
    """``roofline``: the dominant kernel (layer4.0.conv2's forward, the lattice_zp family
    that also runs its dgrad) at top level, and both it and the same conv's weight gradient
    (the step's largest single launch) under ``kernels``."""
    fwd = kernel_roofline("fwd", events, batch, size, dtype, where)
    if fwd is None:
        return None
    out = dict(fwd)
    wg = kernel_roofline("wgrad", wevents, batch, size, dtype, where)
    out["kernels"] = [fwd] + ([wg] if wg is not None else [])
    return out


def host_cores():
    """CPU cores this process may run on: the affinity mask, capped by a cgroup CPU quota
    (the GPU box's share is a quota; os.cpu_count() there reports the whole machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(size, budgets=((1, 10.0), (8, 16.0))):
    """CPU oracle (torch fp32 restatement of the reference path, verified against the real
    reference code in tests/golden) fwd+bwd+Adam on all host cores this process may use, at
    batch 1 and at the bench's batch 8; ``value`` is the batch-8 rate."""
    from oracle import models_ref
    threads = host_cores()
    torch.set_num_threads(threads)
    h = hparams("32")
    m = models_ref.AnatCNNRef(h)
    opt = torch.optim.Adam(models_ref.adam_param_groups(m, h), weight_decay=0)
    rates, samples = {}, []
    for b, budget in budgets:
        g = torch.Generator().manual_seed(15)
        batch = {"mri": torch.rand((b, size, size, size), generator=g, dtype=torch.float64),
                 "label": torch.randint(0, 2, (b,), generator=g)}

        def step():
            opt.zero_grad(set_to_none=True)
            m.general_step(batch, 0, "train")["loss"].backward()
            opt.step()

        step()
        t0 = time.perf_counter()
        n = 0
        while True:
            step()
            n += 1
            el = time.perf_counter() - t0
            if el > budget or n >= 30:
                break
        rates[b] = n * b / el
        samples.append(f"batch {b}: {n} steps in {el:.1f} s")
    return {"value": rates[8], "unit": "volumes/sec", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "machine_cpus": os.cpu_count(),
            "value_batch1": rates[1],
            "sample": f"torch-CPU oracle ResNet-10 fwd+bwd+Adam, 1x{size}^3, fp32, {threads} "
                      f"threads ({'; '.join(samples)})"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", default="128",
                    help="cubic volume edge, or 'mni' for the reference's own 91x109x91 MNI "
                         "volumes (pkg/utils/dataloader.py:228-229; secondary line)")
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--collectives", default="auto", choices=list(DP_MODES) + ["auto", "inside"],
                    help="under torchrun: how the gradient all-reduce meets the replayed step "
                         "(module docstring); auto probes staged / staged1 / after")
    ap.add_argument("--graph", action="store_true", help="= --collectives inside")
    ap.add_argument("--after", action="store_true", help="= --collectives after")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel of every step from Python, the all-reduces from "
                         "the backward's hooks (overlapped with it)")
    ap.add_argument("--workload", default="mri", choices=["mri", "fusion", "three"],
                    help="mri: BASELINE config 2 (the metric); fusion: config 3/4, PET+MRI "
                         "ResNet-10 x2 + MLP head, focal loss, pairs/sec; three: config 5, "
                         "MRI ResNet-34 + PET ResNet-18 + tabular MLP at 160^3, triples/sec")
    args = ap.parse_args()
    mni = args.size == "mni"
    args.size = 128 if mni else int(args.size)
    if mni:
        args.no_roofline = True           # the probe times the 128^3 dominant kernel
        args.no_cpu_baseline = True
    if args.workload != "mri":
        args.no_roofline = True         # the probe times config 2's dominant kernel
        args.no_cpu_baseline = True
        if args.workload == "three" and args.size == 128:
            args.size = 160
    # stdout carries exactly one JSON line: everything else (RCCL's version banner, library
    # chatter) goes to stderr; the result is written to the saved stdout descriptor
    sys.stdout.flush()
    out_fd = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    # MMAD_DP_SELFTEST=1 (under torchrun) runs the RCCL gradient all-reduce path even at N=1
    dp = world > 1 or os.environ.get("MMAD_DP_SELFTEST") == "1"
    if dp:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    torch.manual_seed(15 + rank)
    if args.workload == "mri":
        model = M.Anat_CNN(hparams(args.precision)).cuda()
    elif args.workload == "fusion":
        model = M.PET_MRI_ResNet_Fusion(dict(hparams(args.precision), fl_gamma=2)).cuda()
    else:
        model = M.Tri_ResNet_Tabular_Fusion(dict(hparams(args.precision), fl_gamma=2,
                                             resnet_depth_mri=34, resnet_depth_pet=18)).cuda()
    opt = model.configure_optimizers()
    # every workload replays HIP graphs, at N > 1 too (the launch modes of configs 3-5 are
    # rehearsed at world size 2 in tests/test_dp_graph_world2_gpu.py)
    use_graph = not args.eager
    mode = "inside" if args.graph else "after" if args.after else args.collectives
    if not use_graph:
        mode = "eager"

    def make_reducer(m):
        # staged: one bucket per backward stage -- for ResNet-10 head + layer4 (~43 MB,
        # overlapped by the later stages) ... layer1 + stem (~1 MB, the only one not hidden).
        # Otherwise 4 MiB buckets in reverse order: eager, layer4's big weights go in early
        # (launched from the hooks while backward continues) and the bucket launched last
        # stays ~1 MB instead of ~15 MB.
        if m in DP_MODES and DP_MODES[m][0] == "staged":
            return GradAllReduce(model.parameters(), bucket_mb=None,
                                 stages=backward_stages(model, DP_MODES[m][1])[1])
        if m == "after":
            # every bucket is reduced on the main stream after the backward graph: one bucket,
            # one collective (no overlap to gain from splitting)
            return GradAllReduce(model.parameters(), bucket_mb=None)
        return GradAllReduce(model.parameters(),
                             bucket_mb=float(os.environ.get("MMAD_DP_BUCKET_MB", "4")))

    reducer = None
    if dp:
        broadcast_module_state(model)          # identical replicas, as DDP
        reducer = make_reducer("staged" if mode == "auto" else mode)
    B, S = args.batch, args.size
    VOL = (91, 109, 91) if mni else (S, S, S)
    g = torch.Generator(device="cuda").manual_seed(1000 + rank)   # this rank's shard
    batch = {"mri": torch.rand((B,) + VOL, device="cuda", dtype=torch.float64, generator=g),
             "label": torch.randint(0, 2, (B,), device="cuda", generator=g)}
    if args.workload != "mri":            # z-scored PET (dataloader.py:213-215)
        batch["pet1451"] = torch.randn((B,) + VOL, device="cuda", dtype=torch.float64,
                                       generator=g)
    if args.workload == "three":          # 9 tabular features (dataloader.py:306)
        batch["tabular"] = torch.rand((B, 9), device="cuda", dtype=torch.float64, generator=g)

    dp_events = []                          # (start, end) around each timed finish()

    def step(timed=False):
        opt.zero_grad(set_to_none=True)
        out = model.general_step(batch, 0, "train")
        out["loss"].backward()
        if reducer is not None:
            if timed:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            reducer.finish()
            if timed:
                e1.record()
                dp_events.append((e0, e1))
        opt.step()

    # The step (general_step, backward, Adam) is captured once as HIP graphs and replayed --
    # the same kernels, bit-identical to eager steps (tests/test_graph_step_gpu.py); eager,
    # the host needs ~2.9 of the GPU's ~3.5 ms per step to enqueue it, so a slower or busier
    # host makes the run launch-bound (measured: 1713 vol/s on one box).  N>1 replays the
    # same kernels in the launch mode the warm-up probe picks (--collectives auto): "staged"
    # (the backward as stage graphs, each stage's RCCL all-reduce overlapping the next),
    # "staged1" (one cut) or "after" (one all-reduce after the backward; the pick on one
    # rank) -- tests/test_dp_graph_world2_gpu.py; --graph captures them inside the graph
    # (one-rank checked only), --eager launches them from the backward's hooks (host-bound).
    events, wevents = [], []
    if use_graph:
        if not args.no_roofline:
            # the dominant-kernel probe (HIP events around its launches) cannot sit inside a
            # graph: time it over warm eager steps before the capture instead.  Every rank
            # runs these steps (each issues the bucket all-reduces under RCCL, so the ranks'
            # collective sequences stay aligned); rank 0 records the events.
            for _ in range(3):
                step()
            if rank == 0:
                volume_ops.FWD_PROBES[dominant_desc(B, S)[0]] = events
                volume_ops.WGRAD_PROBES[dominant_desc(B, S)[0]] = wevents
            for _ in range(max(10, args.warmup)):
                step()
            torch.cuda.synchronize()
            volume_ops.FWD_PROBES.clear()
            volume_ops.WGRAD_PROBES.clear()
        probe = {}
        if dp and mode == "auto":
            # capture each candidate in turn, time a few replays (max over ranks), drop it;
            # every rank sees the same times, so every rank picks the same mode
            reducer.remove()
            for cand in DP_MODES:
                red = make_reducer(cand)
                gs = GraphedTrainStep(model, opt, batch, warmup=1, reducer=red,
                                      collectives=DP_MODES[cand][0], cuts=DP_MODES[cand][1])
                gs()
                torch.cuda.synchronize()
                dist.barrier()
                t = time.perf_counter()
                for _ in range(10):
                    gs()
                torch.cuda.synchronize()
                dist.barrier()
                el = torch.tensor([time.perf_counter() - t], device="cuda", dtype=torch.float64)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                probe[cand] = el.item() / 10 * 1e3
                red.remove()
                del gs, red
                torch.cuda.synchronize()
            mode = min(probe, key=probe.get)
            reducer = make_reducer(mode)
        gmode, cuts = DP_MODES.get(mode, (mode, DEFAULT_CUTS)) if dp else ("inside", DEFAULT_CUTS)
        gstep = GraphedTrainStep(model, opt, batch, warmup=max(1, args.warmup),
                                 reducer=reducer, collectives=gmode, cuts=cuts)
        gstep()

        def step(timed=False):
            gstep.finish_events = dp_events if timed and reducer is not None else None
            gstep()
    else:
        for _ in range(args.warmup):
            step()
    if world > 1:
        dist.barrier()
    if rank == 0 and not args.no_roofline and not use_graph:
        volume_ops.FWD_PROBES[dominant_desc(B, S)[0]] = events
        volume_ops.WGRAD_PROBES[dominant_desc(B, S)[0]] = wevents
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    t_issue = time.perf_counter() - t0     # host time to enqueue the K steps (diagnostic)
    torch.cuda.synchronize()
    volume_ops.FWD_PROBES.clear()
    volume_ops.WGRAD_PROBES.clear()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = t.item()
    ms = el / args.steps * 1e3
    value = world * B * args.steps / el
    cdtype = torch.bfloat16 if args.precision == "bf16" else torch.float32
    result = {
        "metric": "volumes/sec fwd+bwd, 3D-ResNet-10 @128^3 bf16, 1/2/4/8 MI355X; % HBM roofline",
        "value": value, "unit": "volumes/sec", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if cdtype == torch.bfloat16 else "f32",
        "data": "synthetic uniform[0,1) f64 volumes resident in HBM, random-init weights",
        "config": {"workload": f"BASELINE config 2: Anat_CNN ResNet-10 MRI-only, 1x{S}^3, "
                               f"batch {B}/GPU, weighted CE, Adam, fwd+bwd+step",
                   "global_batch": B * world, "volume": [1, *VOL],
                   "parallelism": f"dp{world}"},
    }
    if args.workload != "mri":
        unit = "pairs/sec" if args.workload == "fusion" else "triples/sec"
        desc = ("BASELINE config 3/4: PET+MRI ResNet-10 x2 late fusion + MLP head"
                if args.workload == "fusion" else
                "BASELINE config 5: MRI ResNet-34 + PET ResNet-18 + tabular MLP")
        result.update({
            "metric": f"{unit} fwd+bwd, {desc} @{S}^3 bf16 (secondary workload)",
            "unit": unit,
            "config": {"workload": f"{desc}, 2x1x{S}^3 (+9 tabular), batch {B}/GPU, focal "
                                   f"loss gamma 2, Adam, fwd+bwd+step",
                       "global_batch": B * world, "volume": [1, *VOL],
                       "parallelism": f"dp{world}"}})
    if mni:
        result.update({
            "metric": "volumes/sec fwd+bwd, 3D-ResNet-10 @91x109x91 (MNI) bf16 (secondary line)",
            "config": dict(result["config"], workload=(
                f"Anat_CNN ResNet-10 MRI-only on the reference's MNI volumes 1x91x109x91, "
                f"batch {B}/GPU, weighted CE, Adam, fwd+bwd+step"))})
    elif S in FLOP_PER_VOL and args.workload == "mri":
        per_gpu = value / world
        result["step_mfma_frac"] = per_gpu * FLOP_PER_VOL[S] / (
            PEAK_BF16 if cdtype == torch.bfloat16 else PEAK_F32)
        result["step_mfma_frac_basis"] = ("dense GFLOP per volume of the ops run (413.2, "
                                          "SURVEY.md 8d; no stem dgrad) / dense bf16 peak")
        result["hbm_roofline_frac_m2"] = per_gpu * M2_BYTES_PER_VOL / PEAK_HBM
    result["config"]["step_launch"] = (
        "eager" if not use_graph else "hip graph replay" if reducer is None else
        "hip graph replay (fwd+bwd) + eager RCCL all-reduce + graph-replayed Adam"
        if mode == "after" else
        f"hip graph replay: fwd + {len(DP_MODES[mode][1]) + 1} backward-stage graphs, each "
        f"stage's RCCL all-reduce overlapping the next, graph-replayed Adam"
        if mode in DP_MODES else "hip graph replay incl. RCCL all-reduce")
    # host time spent enqueueing each step: close to ms_per_step means the run was bound by
    # the host (Python / launch overhead), not by the GPU
    result["host_issue_ms_per_step"] = t_issue / args.steps * 1e3
    if reducer is not None and dp_events:
        # main-stream time from the end of backward to averaged gradients: the part of the
        # all-reduce that backward did not hide (plus the copies of non-slot gradients)
        result["dp"] = {"buckets_mb": [round(f.numel() * 4 / 2 ** 20, 2) for f in reducer.flats],
                        "exposed_allreduce_ms": sum(a.elapsed_time(b) for a, b in dp_events)
                        / len(dp_events), "backend": "rccl", "collectives": mode}
        if use_graph and probe:
            result["dp"]["auto_probe_ms_per_step"] = {k: round(v, 4) for k, v in probe.items()}
    if rank == 0 and not args.no_roofline:
        result["roofline"] = dominant_kernel_roofline(
            events, wevents, B, S, cdtype,
            "eager steps before the graph capture" if use_graph else "timed region")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(S)
    if rank == 0:
        sys.stdout.flush()
        os.write(out_fd, (json.dumps(result) + "\n").encode())
    if dp:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
