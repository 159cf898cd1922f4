"""Wall time per tiny dependent kernel inside a replayed HIP graph (what an extra BN finalize /
head launch costs the captured step): N back-to-back single-block kernels captured in a
graph, replayed, timed with HIP events; also N launches of a 4096-block elementwise kernel.

    python tools/graph_overhead.py
"""
import torch


def run(n, numel, reps=20):
    x = torch.zeros(numel, device="cuda")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def split(n, parts, numel=1 << 20, reps=20):
    """n dependent kernels captured as `parts` graphs replayed back to back"""
    x = torch.zeros(numel, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    gs = []
    for _ in range(parts):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=gs[0].pool() if gs else None):
            for _ in range(n // parts):
                x.add_(1.0)
        gs.append(g)
    for g in gs:
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        for g in gs:
            g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    for numel in (256, 1 << 20):
        t1 = run(1, numel)
        t100 = run(100, numel)
        print(f"numel {numel}: graph of 1 kernel {t1:.1f} us, of 100 kernels {t100:.1f} us -> "
              f"{(t100 - t1) / 99:.2f} us per extra dependent kernel")
    base = split(120, 1)
    for parts in (2, 4, 6):
        t = split(120, parts)
        print(f"120 kernels as {parts} graphs replayed back to back: {t:.1f} us vs one graph "
              f"{base:.1f} us -> {(t - base) / (parts - 1):.2f} us per extra graph boundary")


if __name__ == "__main__":
    main()
