"""Locate wrong stem-forward outputs: the HIP stem conv at (8,1,128^3) bf16 against a torch
conv3d reference (fp32 on the bf16-rounded operands); prints where the bad elements sit."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import volume_ops as V  # noqa: E402


def main():
    g = torch.Generator(device="cuda").manual_seed(5)
    n, size = 8, 128
    vol = torch.rand((n, 1, size, size, size), generator=g, device="cuda")
    w = (torch.rand((64, 1, 7, 7, 7), generator=g, device="cuda") * 2 - 1) * 0.09
    y = V.conv3d(vol, w, None, (2,) * 3, (3,) * 3, (1,) * 3, torch.bfloat16).float()
    yr = torch.nn.functional.conv3d(vol.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(),
                                    None, 2, 3)
    err = (y - yr).abs()
    bad = ~(err <= 2 ** -7 * yr.abs() + 1e-2)
    print("bad", int(bad.sum()), "nan", int(torch.isnan(y).sum()))
    idx = bad.nonzero()
    if len(idx):
        for d, name in enumerate("ncdhw"):
            u, c = idx[:, d].unique(return_counts=True)
            print(name, list(zip(u.tolist()[:40], c.tolist()[:40])))


if __name__ == "__main__":
    main()
