"""A training step replayed from a captured HIP graph (graph_step.GraphedTrainStep) equals the
eager step: same kernels in the same order, so parameters, BN running statistics and the
loss after the same number of steps are bit-identical."""
import copy

import pytest
import torch

import multimodal_alzheimer_amd as M
from multimodal_alzheimer_amd.graph_step import GraphedTrainStep

pytestmark = pytest.mark.gpu


def _hparams(precision):
    return {"n_classes": 2, "resnet_depth": 10, "conv_out": [], "filter_size": [],
            "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
            "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
            "reduce_factor_lr_schedule": None, "precision": precision,
            "loss_class_weights": torch.tensor([0.3, 0.7], dtype=torch.float64)}


@pytest.mark.parametrize("precision", ["bf16", "32"])
def test_graph_replay_equals_eager_steps(precision):
    torch.manual_seed(3)
    a = M.Anat_CNN(_hparams(precision)).cuda()
    b = copy.deepcopy(a)
    g = torch.Generator(device="cuda").manual_seed(4)
    batches = [{"mri": torch.rand((2, 32, 32, 32), device="cuda", dtype=torch.float64,
                                  generator=g),
                "label": torch.randint(0, 2, (2,), device="cuda", generator=g)}
               for _ in range(3)]
    warm, steps = 2, 3

    opt_a = a.configure_optimizers()
    for _ in range(warm):                      # GraphedTrainStep's eager warm-up steps
        opt_a.zero_grad(set_to_none=True)
        a.general_step(batches[0], 0, "train")["loss"].backward()
        opt_a.step()
    losses_a = []
    for i in range(steps):
        opt_a.zero_grad(set_to_none=True)
        out = a.general_step(batches[i], 0, "train")
        out["loss"].backward()
        opt_a.step()
        losses_a.append(out["loss"].detach().clone())

    opt_b = b.configure_optimizers()
    gs = GraphedTrainStep(b, opt_b, batches[0], warmup=warm)
    losses_b = [gs(batches[i])["loss"].detach().clone() for i in range(steps)]
    torch.cuda.synchronize()

    for la, lb in zip(losses_a, losses_b):
        assert torch.equal(la, lb)
    for (na, pa), (nb, pb) in zip(a.state_dict().items(), b.state_dict().items()):
        assert na == nb
        assert torch.equal(pa, pb), na
