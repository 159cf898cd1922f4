"""Is the training step launch-bound?  Host time to ENQUEUE K steps (no sync) vs the
wall time including the GPU drain, for the bench workload (ResNet-10, 8 x 128^3, bf16)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import multimodal_alzheimer_amd as M  # noqa: E402


def main():
    torch.manual_seed(15)
    model = M.Anat_CNN(bench.hparams("bf16")).cuda()
    opt = model.configure_optimizers()
    g = torch.Generator(device="cuda").manual_seed(1000)
    batch = {"mri": torch.rand((8, 128, 128, 128), device="cuda", dtype=torch.float64,
                               generator=g),
             "label": torch.randint(0, 2, (8,), device="cuda", generator=g)}

    def step():
        opt.zero_grad(set_to_none=True)
        model.general_step(batch, 0, "train")["loss"].backward()
        opt.step()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    k = 20
    t0 = time.perf_counter()
    for _ in range(k):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / k:.3f} ms/step, wall {1e3 * (t2 - t0) / k:.3f} ms/step")


if __name__ == "__main__":
    main()
