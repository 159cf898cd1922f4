"""Summaries of rocprofv3 csv output, written into profiles/.

    python tools/prof_summary.py stats    <dir> [top]      kernel_stats table
    python tools/prof_summary.py dominant <dir> <grid_x> [name]  per-dispatch durations of
                                                           the forward igemm launches with
                                                           that grid and kernel-name prefix
                                                           (one line per step position)
    python tools/prof_summary.py traffic  <fetch_dir> <write_dir>   HBM bytes per launch of
                                                           the probe kernel (json)

FETCH_SIZE is doubled: on gfx950 it reports half the bytes of 16-B-per-lane streaming
reads, including buffer/global_load ... lds (MI355X_MICROARCH.md, HBM section).
WRITE_SIZE is taken as is (exact for 16-B-per-lane stores).
"""
import collections
import csv
import json
import statistics
import sys


def short(name):
    return name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::",
                                                                      "")


def stats(d, top=30):
    rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"{'total ms':>9} {'%':>5} {'calls':>6} {'avg us':>9}  kernel"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        out.append(f"{float(r['TotalDurationNs']) / 1e6:9.3f} {float(r['Percentage']):5.1f} "
                   f"{r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.1f}  {short(r['Name'])[:110]}")
    out.append(f"all kernels: {tot / 1e6:.3f} ms")
    return "\n".join(out)


def dominant(d, grid_x, name="igemm_kernel<unsigned short, 256, 0, 256"):
    """Forward igemm dispatches (MODE 0) in launch order; those with the given grid and
    kernel-name prefix are grouped by their position inside a step so the layer each one
    belongs to is visible."""
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    fwd = [r for r in rows if "igemm_kernel" in r["Kernel_Name"]
           and r["Kernel_Name"].split("<")[1].split(",")[2].strip() == "0"]
    fwd.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = [r for r in fwd if int(r["Grid_Size_X"]) == grid_x and name in r["Kernel_Name"]]
    out = [f"{len(fwd)} forward igemm dispatches, {len(sel)} with grid_x={grid_x}"]
    # consecutive matching dispatches inside one step form a fixed-length group
    groups = collections.defaultdict(list)
    per = None
    for n in (4, 3, 2, 1):
        if len(sel) % n == 0 and len(sel) // n in (13, 10, 20, 25):   # steps+warmup
            per = n
            break
    for i, r in enumerate(sel):
        groups[i % per].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k in sorted(groups):
        v = groups[k]
        out.append(f"position {k} of {per}: n={len(v)} avg={statistics.mean(v):.1f} us "
                   f"median={statistics.median(v):.1f} us min={min(v):.1f} max={max(v):.1f}")
    return "\n".join(out)


def dispatches(d, name):
    """Every dispatch of a kernel (name prefix) in launch order, grouped by its position
    inside a step (the kernel serves several layers/directions per step)."""
    rows = [r for r in csv.DictReader(open(f"{d}/run_kernel_trace.csv"))
            if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # steps in the trace: 13 = 3 warm-up + 10 timed (eager bench); 27 = the graph-mode bench
    # (3 warm + 10 probed eager steps, 3 capture warm-up steps, 1 + 10 replays); 14 = the
    # graph-mode bench without the probe (3 warm-up, 1 capture, 10 replays)
    per = next((n for n in (6, 5, 4, 3, 2, 1)
                if len(rows) % n == 0 and len(rows) // n in (13, 10, 14, 20, 25, 27)), 1)
    groups = collections.defaultdict(list)
    for i, r in enumerate(rows):
        groups[i % per].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = [f"{len(rows)} dispatches of {name}, {per} per step"]
    for k in sorted(groups):
        v = groups[k]
        out.append(f"position {k} of {per}: n={len(v)} avg={statistics.mean(v):.1f} us "
                   f"median={statistics.median(v):.1f} us min={min(v):.1f} max={max(v):.1f}")
    return "\n".join(out)


FWD_KERNELS = ("igemm_kernel", "lattice_conv_kernel", "lattice_zp_kernel")
WGRAD_KERNELS = ("lattice_wgrad_kernel", "wgrad_reduce_t_kernel")
LABELS = {"fwd": "layer4.0.conv2 fwd residue-class kernel (bf16, 8x512x16^3, 3^3 dil 4)",
          "wgrad": "layer4.0.conv2 wgrad: lattice_wgrad_kernel + its slab reduce "
                   "(bf16, 8x512x16^3, 3^3 dil 4)"}


def counter(d, name, kernels=FWD_KERNELS):
    """per-launch values of one counter, {kernel: [values in launch order]}"""
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    out = collections.defaultdict(list)
    for r in rows:
        k = next((k for k in kernels if k in r["Kernel_Name"]), None)
        if k is not None and r["Counter_Name"] == name:
            out[k].append(float(r["Counter_Value"]))
    return out


def traffic(fetch_dir, write_dir, op="fwd"):
    """HBM bytes per call of the probed op: per kernel the median over launches (FETCH_SIZE
    x2, WRITE_SIZE as reported), summed over the op's kernels (wgrad: the MFMA kernel and
    its slab reduce)"""
    kernels = WGRAD_KERNELS if op == "wgrad" else FWD_KERNELS
    f = counter(fetch_dir, "FETCH_SIZE", kernels)
    w = counter(write_dir, "WRITE_SIZE", kernels)
    # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB
    fb = sum(statistics.median(v) for v in f.values()) * 1024 * 2
    wb = sum(statistics.median(v) for v in w.values()) * 1024
    return {"kernel": LABELS[op],
            "launches": [sum(map(len, f.values())), sum(map(len, w.values()))],
            "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
            "hbm_bytes_per_launch": fb + wb,
            "raw_fetch_size_kib": dict(f), "raw_write_size_kib": dict(w),
            "correction": "FETCH_SIZE x2 (gfx950 half-count of 16B/lane reads); "
                          "WRITE_SIZE as reported; median over launches per kernel; on-die "
                          "cache scrubbed before each call (cold)"}


def _is_opt(name):
    """a step's closing optimizer launch: torch's fused Adam (eager steps) or the captured
    step's fused Adam + repack (csrc/adam.hip)"""
    return ("FusedAdam" in name or "FusedOptimizerTensorListMetadata" in name or
            "adam_repack_kernel" in name)


def step(d):
    """Kernels of the last complete step, in launch order, with durations (us)."""
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with the fused Adam launch(es); take the span between the last two
    ends = [i for i, r in enumerate(rows) if _is_opt(r["Kernel_Name"])]
    if len(ends) < 4:
        sel = rows
    else:
        # group consecutive optimizer launches; step = after the 2nd-last group to the last
        groups, cur = [], [ends[0]]
        for e in ends[1:]:
            if e - cur[-1] <= 3:
                cur.append(e)
            else:
                groups.append(cur)
                cur = [e]
        groups.append(cur)
        sel = rows[groups[-2][-1] + 1:groups[-1][-1] + 1]
    out, tot = [], 0.0
    for r in sel:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += us
        out.append(f"{us:8.1f}  g={r['Grid_Size_X']:>8}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}  "
                   f"{short(r['Kernel_Name']).split('(')[0][:90]}")
    out.append(f"step kernels: {len(sel)}, sum {tot:.1f} us")
    return "\n".join(out)


def stepavg(d, skip=2):
    """Per-position kernel durations (us) averaged over the complete steps of the trace
    (the first `skip` steps dropped), in launch order, plus the mean step sum."""
    rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if _is_opt(r["Kernel_Name"])]
    groups, cur = [], [ends[0]]
    for e in ends[1:]:
        if e - cur[-1] <= 3:
            cur.append(e)
        else:
            groups.append(cur)
            cur = [e]
    groups.append(cur)
    steps = [rows[a[-1] + 1:b[-1] + 1] for a, b in zip(groups, groups[1:])][skip:]
    n = min(len(st) for st in steps)
    steps = [st for st in steps if len(st) == n]
    out, tot = [], 0.0
    for i in range(n):
        us = sum((int(st[i]["End_Timestamp"]) - int(st[i]["Start_Timestamp"])) / 1e3
                 for st in steps) / len(steps)
        tot += us
        r = steps[0][i]
        out.append(f"{us:8.1f}  g={r['Grid_Size_X']:>8}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}  "
                   f"{short(r['Kernel_Name']).split('(')[0][:90]}")
    out.insert(0, f"steps averaged: {len(steps)}, kernels per step {n}, mean sum {tot:.1f} us")
    return "\n".join(out)


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "stats":
        print(stats(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30))
    elif mode == "dominant":
        print(dominant(sys.argv[2], int(sys.argv[3]), *sys.argv[4:5]))
    elif mode == "dispatches":
        print(dispatches(sys.argv[2], sys.argv[3]))
    elif mode == "step":
        print(step(sys.argv[2]))
    elif mode == "stepavg":
        print(stepavg(sys.argv[2]))
    elif mode == "traffic":
        print(json.dumps(traffic(sys.argv[2], sys.argv[3], *sys.argv[4:5]), indent=1))
