"""Replay determinism of a forward + backward-only graph (no reducer, no optimizer in the
graph): replay twice on the same batch with an eager operation in between and compare the
gradients bit for bit.

  python tools/diag_replay.py {none,alloc,eagerstep,adam}
    none       nothing between the replays
    alloc      a large eager allocation, written (1 GiB of 7s), then freed
    eagerstep  another model's eager forward + backward
    adam       an eager optimizer step on the graphed model (parameters change: the
               replays then differ by design, so only the stem/layer1 grads' magnitude is
               printed)"""
import copy
import sys

import torch

sys.path.insert(0, ".")
import multimodal_alzheimer_amd as M  # noqa: E402
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep  # noqa: E402

SCEN = sys.argv[1] if len(sys.argv) > 1 else "none"


def hp():
    return {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": "bf16",
            "loss_class_weights": torch.tensor([0.3, 0.7], dtype=torch.float64)}


def batch(seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return {"mri": torch.rand((2, 32, 32, 32), device="cuda", dtype=torch.float64, generator=g),
            "label": torch.randint(0, 2, (2,), device="cuda", generator=g)}


def main():
    import os
    os.environ["MMAD_GRAPH_DEBUG"] = "noopt"
    torch.manual_seed(13)
    b = M.Anat_CNN(hp()).cuda()
    a = copy.deepcopy(b)
    opt_b = b.configure_optimizers()
    gs = GraphedTrainStep(b, opt_b, batch(40), warmup=2)
    gs.graph.replay()
    torch.cuda.synchronize()
    g1 = {n: p.grad.clone() for n, p in b.named_parameters()}
    ptr = {n: p.grad.data_ptr() for n, p in b.named_parameters()}
    if SCEN == "alloc":
        x = torch.full((1 << 28,), 7.0, device="cuda")
        torch.cuda.synchronize()
        del x
    elif SCEN == "eagerstep":
        a.general_step(batch(41), 0, "train")["loss"].backward()
        torch.cuda.synchronize()
    elif SCEN == "adam":
        opt_b.step()
        torch.cuda.synchronize()
    gs.graph.replay()
    torch.cuda.synchronize()
    bad = []
    for n, p in b.named_parameters():
        moved = p.grad.data_ptr() != ptr[n]
        same = torch.equal(p.grad, g1[n])
        if moved or not same:
            bad.append((n, moved, float((p.grad - g1[n]).abs().nan_to_num(1e38).max())))
    print(f"{SCEN}: {len(bad)} grads differ after the second replay: {bad[:10]}", flush=True)


if __name__ == "__main__":
    main()
