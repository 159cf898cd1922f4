"""Back-to-back cost of tiny launches on one stream: our relu kernel (16 floats), torch's
add_ on 16 floats, and an empty hipMemsetAsync, 2000 each (HIP events)."""
import torch

from multimodal_alzheimer_amd import _lib as L


def timeit(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / n


x = torch.randn(16, device="cuda")
y = torch.empty_like(x)
big = torch.randn(1 << 20, device="cuda")
ybig = torch.empty_like(big)
print("mmad_relu_fwd 16 f32   us/launch %.2f" % timeit(
    lambda: L.call("mmad_relu_fwd", L.F32, 16, L.ptr(x), L.ptr(y), L.stream())))
print("torch add_ 16 f32      us/launch %.2f" % timeit(lambda: x.add_(1.0)))
print("mmad_relu_fwd 1M f32   us/launch %.2f" % timeit(
    lambda: L.call("mmad_relu_fwd", L.F32, 1 << 20, L.ptr(big), L.ptr(ybig), L.stream())))
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    for _ in range(100):
        L.call("mmad_relu_fwd", L.F32, 16, L.ptr(x), L.ptr(y), L.stream())
print("graph of 100 relu 16   us/launch %.2f" % (timeit(lambda: g.replay(), 50) / 100))
