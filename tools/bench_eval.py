"""Inference throughput of the MRI classifier (Anat_CNN ResNet-10, 1x128^3, bf16, eval mode:
running statistics, no autograd) -- the path `validation_step` / `test_step` / the reference's
pkg/inference/test_*.py take -- with the eval-fused blocks (BN folded into the conv,
residual + ReLU in the epilogue) and with the training-style op sequence.

    python tools/bench_eval.py [--batch 8] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import multimodal_alzheimer_amd as M  # noqa: E402
from multimodal_alzheimer_amd import medicalnet  # noqa: E402
from bench import hparams  # noqa: E402


def run(model, batch, steps, fused):
    medicalnet.EVAL_FUSED = fused
    with torch.no_grad():
        for _ in range(3):
            model.general_step(batch, 0, "val")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = model.general_step(batch, 0, "val")["outputs"]
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    torch.manual_seed(0)
    m = M.Anat_CNN(hparams("bf16")).cuda().eval()
    s = a.size
    batch = {"mri": torch.rand((a.batch, s, s, s), device="cuda", dtype=torch.float64),
             "label": torch.randint(0, 2, (a.batch,), device="cuda")}
    tf, of = run(m, batch, a.steps, True)
    tu, ou = run(m, batch, a.steps, False)
    medicalnet.EVAL_FUSED = True
    print(f"eval ResNet-10 1x{s}^3 batch {a.batch} bf16: fused {a.batch / tf:.0f} vol/s "
          f"({tf * 1e3:.2f} ms/batch), unfused {a.batch / tu:.0f} vol/s ({tu * 1e3:.2f} ms); "
          f"max|logit diff| {(of - ou).abs().max().item():.3e}")


if __name__ == "__main__":
    main()
