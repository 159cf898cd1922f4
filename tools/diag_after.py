"""Diagnose GraphedTrainStep(collectives="after") against plain eager steps at one RCCL
rank: which parameters' replayed gradients leave the eager ones, under which setup.

  python tools/diag_after.py SCENARIO
    after       GraphedTrainStep(reducer, collectives="after")  (bench.py's N > 1 mode)
    after1      the same with one bucket (bucket_mb 1024)
    inside      GraphedTrainStep(reducer, collectives="inside")
    noslots     "after" with the reducer's gradient slots disabled (MMAD_DP_GRAD_SLOTS=0)
    nopool      "after" with the optimizer graph in its own memory pool
    nofinish    "after" without the eager finish() between the replays
    join / tail "after" with a grad-stream join / a trivial kernel ending the capture
    insidenoopt "inside" without the optimizer step in the graph (stepped eagerly)
    plainnoopt  no reducer, graph = forward + backward only, optimizer stepped eagerly
Prints per step the gradient mismatches after the replay (count, worst, first names)."""
import copy
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
SCEN = sys.argv[1] if len(sys.argv) > 1 else "after"
if SCEN == "noslots":
    os.environ["MMAD_DP_GRAD_SLOTS"] = "0"
if SCEN == "nopool":
    os.environ["MMAD_GRAPH_SHARE_POOL"] = "0"
if SCEN in ("join", "tail", "nodefer"):
    os.environ["MMAD_GRAPH_DEBUG"] = SCEN
if SCEN in ("insidenoopt", "plainnoopt"):
    os.environ["MMAD_GRAPH_DEBUG"] = "noopt"
import multimodal_alzheimer_amd as M  # noqa: E402
from multimodal_alzheimer_amd.data_parallel import GradAllReduce  # noqa: E402
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep  # noqa: E402


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


def cmp(tag, a, b, grads=False):
    bad, worst = [], 0.0
    for (na, pa), (_, pb) in zip(a.named_parameters(), b.named_parameters()):
        x, y = (pa.grad, pb.grad) if grads else (pa.detach(), pb.detach())
        if x is None or y is None:
            bad.append(na + "(None)")
            continue
        if not torch.equal(x, y):
            bad.append(na)
            worst = max(worst, (x.float() - y.float()).abs().nan_to_num(1e38).max().item())
    print(f"{SCEN} {tag}: {len(bad)} differ, worst {worst:.3e}, {bad[:12]}", flush=True)


def main():
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29581", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    torch.manual_seed(13)
    a = M.Anat_CNN(hp()).cuda()
    b = copy.deepcopy(a)
    bs = [batch(40 + i) for i in range(3)]
    opt_a = a.configure_optimizers()
    for grp in opt_a.param_groups:
        grp["capturable"] = True
        grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
    for _ in range(2):
        opt_a.zero_grad(set_to_none=True)
        a.general_step(bs[0], 0, "train")["loss"].backward()
        opt_a.step()
    opt_b = b.configure_optimizers()
    red = None if SCEN == "plainnoopt" else \
        GradAllReduce(b.parameters(), bucket_mb=1024.0 if SCEN == "after1" else 4.0)
    coll = "inside" if SCEN in ("inside", "insidenoopt", "plainnoopt") else "after"
    gs = GraphedTrainStep(b, opt_b, bs[0], warmup=2, reducer=red, collectives=coll)
    torch.cuda.synchronize()
    cmp("after warm-up + capture", a, b)
    for i in range(2):
        opt_a.zero_grad(set_to_none=True)
        a.general_step(bs[i], 0, "train")["loss"].backward()
        for k, v in bs[i].items():
            gs.static[k].copy_(v)
        gs.graph.replay()
        torch.cuda.synchronize()
        cmp(f"step {i} grads after replay", a, b, grads=True)
        if SCEN in ("insidenoopt", "plainnoopt"):
            opt_b.step()
        if coll == "after":
            if SCEN != "nofinish":
                gs.reducer.finish()
            gs.opt_graph.replay()
        opt_a.step()
        torch.cuda.synchronize()
        cmp(f"step {i} params after step", a, b)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
