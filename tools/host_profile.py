"""Host-side (Python) profile of the eager config-2 training step: where the ~3 ms of host
enqueue time per step goes.  Backward runs on the calling thread here
(torch.autograd.set_multithreading_enabled(False)) so cProfile sees it.
    python tools/host_profile.py [steps]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multimodal_alzheimer_amd as M  # noqa: E402
from bench import hparams  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.autograd.set_multithreading_enabled(False)
    model = M.Anat_CNN(hparams("bf16")).cuda()
    opt = model.configure_optimizers()
    if isinstance(opt, (list, tuple)):
        opt = opt[0]
    if isinstance(opt, dict):
        opt = opt["optimizer"]
    g = torch.Generator(device="cuda").manual_seed(1000)
    batch = {"mri": torch.rand((8, 128, 128, 128), device="cuda", dtype=torch.float64,
                               generator=g),
             "label": torch.randint(0, 2, (8,), device="cuda", generator=g)}

    def step():
        opt.zero_grad(set_to_none=True)
        model.general_step(batch, 0, "train")["loss"].backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(steps):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(35)


if __name__ == "__main__":
    main()
