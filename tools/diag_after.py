"""Diagnose GraphedTrainStep(collectives="after") against plain eager steps at one RCCL
rank: where do model b's parameters leave model a's?  Prints, per step, the gradient and
parameter mismatches (count of tensors, worst element) after the replay, after finish(),
and after the optimizer replay, plus an eager-with-reducer control."""
import copy
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, ".")
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
            worst = max(worst, (x.float() - y.float()).abs().max().item())
    print(f"{tag}: {len(bad)} differ, worst {worst:.3e}, first {bad[:3]}", flush=True)


def main():
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29581", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    torch.manual_seed(13)
    a = M.Anat_CNN(hp()).cuda()
    b = copy.deepcopy(a)
    c = copy.deepcopy(a)
    bs = [batch(40 + i) for i in range(3)]
    opt_a = a.configure_optimizers()
    for m, opt in ((a, opt_a),):
        for grp in opt.param_groups:
            grp["capturable"] = True
            grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
    for _ in range(2):
        opt_a.zero_grad(set_to_none=True)
        a.general_step(bs[0], 0, "train")["loss"].backward()
        opt_a.step()
    # control: eager steps of c with the reducer (defer mode, as the "after" warm-up)
    opt_c = c.configure_optimizers()
    for grp in opt_c.param_groups:
        grp["capturable"] = True
        grp["lr"] = torch.tensor(float(grp["lr"]), device="cuda")
    red_c = GradAllReduce(c.parameters(), bucket_mb=4.0)
    for _ in range(2):
        opt_c.zero_grad(set_to_none=True)
        red_c.defer = True
        c.general_step(bs[0], 0, "train")["loss"].backward()
        red_c.defer = False
        red_c.finish()
        opt_c.step()
    torch.cuda.synchronize()
    cmp("control eager+reducer after warm-up", a, c)

    opt_b = b.configure_optimizers()
    red = GradAllReduce(b.parameters(), bucket_mb=4.0)
    gs = GraphedTrainStep(b, opt_b, bs[0], warmup=2, reducer=red, collectives="after")
    torch.cuda.synchronize()
    cmp("b after warm-up + capture", a, b)
    for i in range(3):
        opt_a.zero_grad(set_to_none=True)
        la = a.general_step(bs[i], 0, "train")["loss"]
        la.backward()
        for k, v in bs[i].items():
            gs.static[k].copy_(v)
        gs.graph.replay()
        torch.cuda.synchronize()
        print(f"step {i}: loss a {la.item():.9g} b {gs.out['loss'].item():.9g}", flush=True)
        cmp(f"step {i} grads after replay", a, b, grads=True)
        gs.reducer.finish()
        torch.cuda.synchronize()
        cmp(f"step {i} grads after finish", a, b, grads=True)
        opt_a.step()
        gs.opt_graph.replay()
        torch.cuda.synchronize()
        cmp(f"step {i} params after step", a, b)
        sa = opt_a.state[next(iter(opt_a.state))]
        sb = opt_b.state[next(iter(opt_b.state))]
        print(f"   adam step a {sa['step'].item()} b {sb['step'].item()}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
