"""Generate golden vectors from the REAL reference code (run in the build container only).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

The reference (``/root/reference``, read-only) is imported as a Python package; nothing
of it is copied.  Its missing third-party dependencies are replaced by the minimal stubs
below (pytorch_lightning / torchmetrics / torchvision / seaborn: bookkeeping only, no
arithmetic) and by the oracle's MedicalNet restatement (``oracle/medicalnet_ref.py``),
because MedicalNet is un-vendored and absent offline.

Every weight, volume and label comes from ``oracle.prng`` so the fixtures hold only
seeds, shapes and outputs.  The files are data (inputs and expected outputs); the
reference source never leaves this container.
"""
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)

from oracle import prng, medicalnet_ref, models_ref  # noqa: E402

W2 = [0.20314960629921264, 0.7968503937007874]              # pkg/inference/test_tab.py:25-28
W3 = [0.4651162790697675, 0.6712473572938689, 0.8636363636363636]   # test_tab.py:36-40


def install_stubs():
    """Bookkeeping-only stand-ins for packages the reference imports but this image lacks."""
    pl = types.ModuleType("pytorch_lightning")

    class LightningModule(nn.Module):
        def save_hyperparameters(self, hparams, ignore=()):
            object.__setattr__(self, "hparams", {k: v for k, v in hparams.items()
                                                 if k not in ignore})

        def log(self, *a, **k):
            pass

        def log_dict(self, *a, **k):
            pass

    pl.LightningModule = LightningModule
    sys.modules["pytorch_lightning"] = pl

    tm = types.ModuleType("torchmetrics")
    tmc = types.ModuleType("torchmetrics.classification")

    class _Metric:
        def __init__(self, *a, **k):
            pass

        def __call__(self, *a, **k):
            return None

        def to(self, *a, **k):
            return self

    for n in ("MulticlassF1Score", "MulticlassMatthewsCorrCoef", "MulticlassConfusionMatrix"):
        setattr(tmc, n, _Metric)
    tm.classification = tmc
    tm.ConfusionMatrix = _Metric
    sys.modules["torchmetrics"] = tm
    sys.modules["torchmetrics.classification"] = tmc
    for n in ("torchvision", "seaborn"):
        sys.modules[n] = types.ModuleType(n)

    mn = types.ModuleType("MedicalNet")
    mn_model = types.ModuleType("MedicalNet.model")
    mn_setting = types.ModuleType("MedicalNet.setting")
    mn_model.generate_model = medicalnet_ref.generate_model
    mn_setting.parse_opts = medicalnet_ref.parse_opts
    mn.model, mn.setting = mn_model, mn_setting
    sys.modules.update({"MedicalNet": mn, "MedicalNet.model": mn_model,
                        "MedicalNet.setting": mn_setting})
    os.environ.setdefault("CUDA_VISIBLE_DEVICES", "0")   # anat_cnn.py:20-24 insists
    # The reference's `pkg` is a namespace package (no __init__.py); this repo's `pkg/`
    # import shim is a regular package and would shadow it, so drop the repo from the path
    # (the oracle modules are already imported) and any cached `pkg` modules.
    sys.path[:] = [p for p in sys.path if os.path.abspath(p or ".") != REPO]
    for name in [m for m in sys.modules if m == "pkg" or m.startswith("pkg.")]:
        del sys.modules[name]
    sys.path.insert(0, REF)
    import pkg.models.base_model as _bm
    assert _bm.__file__.startswith(REF), _bm.__file__


def load_prng_weights(model, seed):
    sd = model.state_dict()
    vals = prng.fill_state_dict(sd, seed)
    with torch.no_grad():
        for k, v in vals.items():
            sd[k].copy_(torch.from_numpy(v))


def summarize(prefix, name, t, out, full_limit=4096):
    a = t.detach().double().numpy().ravel()
    if a.size <= full_limit:
        out[f"{prefix}full/{name}"] = a
    else:
        out[f"{prefix}head/{name}"] = a[:256].copy()
        out[f"{prefix}stats/{name}"] = np.array([a.sum(), np.abs(a).sum(), np.sqrt((a * a).sum())])


def run_case(model, batch, out):
    """eval logits on fresh weights, then one train-mode general_step + backward."""
    model.eval()
    with torch.no_grad():
        out["eval_logits"] = model.general_step(batch, 0, "val")["outputs"].numpy()
    model.train()
    res = model.general_step(batch, 0, "train")
    res["loss"].backward()
    out["train_logits"] = res["outputs"].detach().numpy()
    out["train_loss"] = np.array(res["loss"].item())
    for name, p in model.named_parameters():
        if p.grad is not None:
            summarize("grad/", name, p.grad, out)
    for name, b in model.named_buffers():
        if "running" in name:
            summarize("buf/", name, b, out)
    out["state_dict_keys"] = np.array(list(model.state_dict().keys()))


def record_samples(prefix, model, out):
    """Gradients of a config-size case: the elements prng.sample_index picks, + stats."""
    for name, p in model.named_parameters():
        if p.grad is None:
            continue
        a = p.grad.detach().double().numpy().ravel()
        out[f"{prefix}samp/{name}"] = a[prng.sample_index(name, a.size)]
        out[f"{prefix}stats/{name}"] = np.array([a.sum(), np.abs(a).sum(),
                                                 np.sqrt((a * a).sum())])


def run_full_case(model, ref64, batch, inputs, out):
    """A BASELINE-size case (128^3, batch 8): eval logits on fresh weights, one train-mode
    general_step + backward of the reference code in fp32 (gradients at sampled elements,
    running statistics in full), then the same train step in float64 on the oracle
    restatement loaded with the same weights -- the exact answer the GPU tests measure both
    the reference's fp32 error and their own against.  Between the two, the reference's
    train step again under CPU autocast bf16 (``grad16/``, ``train_logits16``): the
    reference's own bf16 error, which bounds the GPU bf16 test."""
    sd0 = {k: v.clone() for k, v in model.state_dict().items()}
    model.eval()
    with torch.no_grad():
        out["eval_logits"] = model.general_step(batch, 0, "val")["outputs"].numpy()
    model.train()
    res = model.general_step(batch, 0, "train")
    res["loss"].backward()
    out["train_logits"] = res["outputs"].detach().numpy()
    out["train_loss"] = np.array(res["loss"].item())
    record_samples("grad/", model, out)
    for name, b in model.named_buffers():
        if "running" in name:
            summarize("buf/", name, b, out)
    out["state_dict_keys"] = np.array(list(model.state_dict().keys()))
    del res
    model.zero_grad(set_to_none=True)
    # the reference's own bf16 path (Lightning precision "bf16" = autocast around the step,
    # backward outside it), on CPU: its error against float64 is the yardstick of the GPU
    # bf16 test (a bf16 step cannot be closer to float64 than rounding allows)
    model.load_state_dict(sd0)
    model.train()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        r16 = model.general_step(batch, 0, "train")
    r16["loss"].backward()
    out["train_logits16"] = r16["outputs"].detach().float().numpy()
    out["train_loss16"] = np.array(r16["loss"].item())
    record_samples("grad16/", model, out)
    del r16
    model.zero_grad(set_to_none=True)
    ref64.load_state_dict(sd0)
    ref64 = ref64.double().train()
    y64 = ref64(*inputs(batch))
    loss64 = ref64.criterion(y64, batch["label"])
    loss64.backward()
    out["train_logits64"] = y64.detach().numpy()
    out["train_loss64"] = np.array(loss64.item())
    record_samples("grad64/", ref64, out)


def batch_for(shape, n_classes, seed, keys=("mri",)):
    b = {"label": torch.from_numpy(prng.labels(seed + 7, shape[0], n_classes))}
    for i, k in enumerate(keys):
        gen = prng.mri_volume if k == "mri" else prng.pet_volume
        b[k] = torch.from_numpy(gen(seed + i, shape)).double()   # dataloader yields f64
    return b


def anat_hparams(depth=10, n_classes=2, **kw):
    h = {"n_classes": n_classes, "resnet_depth": depth, "conv_out": [], "filter_size": [],
         "batchnorm_begin": False, "batchnorm_dense": False, "linear_out": [],
         "fl_gamma": None, "lr": 1e-3, "lr_pretrained": 1e-5, "l2_reg": 0,
         "reduce_factor_lr_schedule": None, "gpu_id": "0",
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


def pet_hparams(n_classes=2, **kw):
    h = {"n_classes": n_classes, "conv_out": (8, 16, 32, 64), "filter_size": (5, 5, 3, 3),
         "batchnorm": False, "linear_out": 64, "lr": 1e-3, "reduce_factor_lr_schedule": None,
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


CASES = {}


def case(fn):
    CASES[fn.__name__] = fn
    return fn


@case
def losses():
    from pkg.loss_functions.focalloss import FocalLoss
    out = {}
    for C in (2, 3):
        x0 = (prng.uniform(100 + C, 8 * C).astype(np.float64) * 6.0 - 3.0).reshape(8, C)
        y = torch.from_numpy(prng.labels(200 + C, 8, C))
        out[f"x_C{C}"], out[f"y_C{C}"] = x0, y.numpy()
        for g in (0, 1, 2, 5):
            x = torch.tensor(x0, requires_grad=True)
            loss = FocalLoss(gamma=g)(x, y)
            loss.backward()
            out[f"focal_g{g}_C{C}_loss"] = np.array(loss.item())
            out[f"focal_g{g}_C{C}_grad"] = x.grad.numpy()
        w = torch.tensor(W2 if C == 2 else W3, dtype=torch.double)
        x = torch.tensor(x0, requires_grad=True)
        loss = nn.CrossEntropyLoss(weight=w)(x, y)
        loss.backward()
        out[f"ce_C{C}_loss"] = np.array(loss.item())
        out[f"ce_C{C}_grad"] = x.grad.numpy()
    # ReLU'd logits with exact ties (anat_cnn.py:76-77): argmax must take the first index
    t = torch.tensor([[0.0, 0.0], [0.3, 0.0], [0.0, 0.7], [0.5, 0.5]])
    out["tie_logits"], out["tie_argmax"] = t.numpy(), torch.argmax(t, 1).numpy()
    return out


def _anat(depth, size, bsz, seed, **kw):
    """size: an int (cubic volume) or a (D, H, W) tuple."""
    from pkg.models.mri_models.anat_cnn import Anat_CNN
    torch.manual_seed(0)
    m = Anat_CNN(anat_hparams(depth, **kw))
    load_prng_weights(m, seed)
    dhw = (size,) * 3 if isinstance(size, int) else tuple(size)
    out = {"seed": np.array(seed), "shape": np.array((bsz,) + dhw)}
    run_case(m, batch_for((bsz,) + dhw, m.hparams["n_classes"], seed + 1), out)
    return out


@case
def anat_r10_32():                           # all logits ReLU'd to 0: argmax tie case
    return _anat(10, 32, 2, 11)


@case
def anat_r10_64():                           # BASELINE config 1 (CPU plumbing config)
    return _anat(10, 64, 2, 12)


def _anat_live(depth, size, bsz, seed, **kw):
    """Weight seed (searched upwards in steps of 1000) whose train logits keep a positive
    entry in every sample, so gradients reach the backbone (the final ReLU,
    anat_cnn.py:77, otherwise zeroes them all)."""
    for s in range(seed, seed + 50000, 1000):
        out = _anat(depth, size, bsz, s, **kw)
        if (out["train_logits"] > 0).any(axis=1).all():
            return out
    raise RuntimeError("no live seed")


@case
def anat_r10_32_live():
    return _anat_live(10, 32, 2, 31)


@case
def anat_r10_64_live():                      # BASELINE config 1 with live gradients
    return _anat_live(10, 64, 2, 32)


@case
def anat_r10_mni():
    """The reference's real input geometry: MNI 2 mm volumes, 91 x 109 x 91
    (pkg/utils/dataloader.py:228-229 nib get_fdata; stride-8 output 12 x 14 x 12,
    pkg/utils/outdated/inspect_model.py:105)."""
    return _anat_live(10, (91, 109, 91), 2, 34)


@case
def anat_r50():
    """ResNet-50 (Bottleneck 1^3 -> 3^3 -> 1^3, 2048 features; anat_cnn.py:42-43)."""
    return _anat_live(50, 32, 2, 35)


@case
def anat_conv_out():
    """conv_seg with a conv_out block (anat_cnn.py:52-63): BN3d(512) -> Conv3d(512, 32, 3,
    'same') -> BN3d(32) -> ReLU -> MaxPool3d(2) -> GAP -> Linear(32, 16) -> ReLU ->
    Linear(16, 3) -> ReLU, at 64^3 (8^3 after the backbone, 4^3 after the pool)."""
    return _anat_live(10, 64, 2, 36, n_classes=3, batchnorm_begin=True, conv_out=[32],
                      filter_size=[3], batchnorm_conv=True, linear_out=[16])


@case
def anat_r18_head():
    return _anat(18, 32, 4, 13, n_classes=3, batchnorm_begin=True, batchnorm_dense=True,
                 linear_out=[64, 32], fl_gamma=2)


@case
def anat_r10_focal():
    return _anat(10, 32, 3, 14, fl_gamma=5, linear_out=[128])


@case
def pet_resnet_r10():
    from pkg.models.pet_models.pet_resnet_cnn import PET_CNN_ResNet
    m = PET_CNN_ResNet(anat_hparams(10, fl_gamma=1))
    load_prng_weights(m, 15)
    out = {"seed": np.array(15), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 2, 16, keys=("pet1451",)), out)
    return out


@case
def small_pet():
    from pkg.models.pet_models.pet_cnn import Small_PET_CNN
    m = Small_PET_CNN(pet_hparams())
    load_prng_weights(m, 17)
    out = {"seed": np.array(17), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 2, 18, keys=("pet1451",)), out)
    return out


@case
def small_pet_bn3():
    from pkg.models.pet_models.pet_cnn import Small_PET_CNN
    m = Small_PET_CNN(pet_hparams(n_classes=3, batchnorm=True, conv_out=(16, 32, 64),
                                  filter_size=(7, 5, 3), linear_out=32))
    load_prng_weights(m, 19)
    out = {"seed": np.array(19), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 3, 20, keys=("pet1451",)), out)
    return out


@case
def anat_pet_fusion():
    from pkg.models.pet_models.pet_cnn import Small_PET_CNN
    from pkg.models.mri_models.anat_cnn import Anat_CNN
    from pkg.models.fusion_models.anat_pet_fusion import Anat_PET_CNN
    stage1 = {"pet.ckpt": (Small_PET_CNN, pet_hparams()),
              "mri.ckpt": (Anat_CNN, anat_hparams(10))}
    orig = {c: c.__dict__.get("load_from_checkpoint") for c in (Small_PET_CNN, Anat_CNN)}
    for cls in (Small_PET_CNN, Anat_CNN):
        cls.load_from_checkpoint = classmethod(
            lambda c, path, **kw: stage1[path][0](stage1[path][1]))
    try:
        h = anat_hparams(10, fl_gamma=2, path_pet="pet.ckpt", path_mri="mri.ckpt")
        m = Anat_PET_CNN(h)
    finally:
        for c, f in orig.items():
            if f is None:
                del c.load_from_checkpoint
    load_prng_weights(m, 21)
    out = {"seed": np.array(21), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 2, 22, keys=("pet1451", "mri")), out)
    return out


TAB_SEED, TAB_ROWS = 4242, 16        # the TabPFN stand-in's seed / training rows


def install_tabpfn_standin():
    """The stage-2 tabular fusion models import pkg.models.tabular_models.dl_approach, which
    imports ``tabpfn`` (absent offline) and, through data_preparation, the reference
    DataLoader module (nibabel, torchvision.transforms: absent, untouched here).  The
    reference modules themselves run; only TabPFN is the build-defined stand-in of
    oracle/tabpfn_standin.py, and ``get_data`` (the training rows of the ADNI table) returns
    the stand-in's synthetic table."""
    from oracle import tabpfn_standin
    tp = types.ModuleType("tabpfn")
    tp.TabPFNClassifier = tabpfn_standin.TabPFNClassifier
    sys.modules["tabpfn"] = tp
    if "nibabel" not in sys.modules:
        sys.modules["nibabel"] = types.ModuleType("nibabel")
    tv = sys.modules.setdefault("torchvision", types.ModuleType("torchvision"))
    tvt = types.ModuleType("torchvision.transforms")
    tvt.ToTensor = tvt.Normalize = object
    tv.transforms = tvt
    sys.modules["torchvision.transforms"] = tvt
    import pkg.models.tabular_models.dl_approach as dl
    assert dl.__file__.startswith(REF), dl.__file__
    dl.get_data = lambda path, binary_classification: tabpfn_standin.training_table(
        TAB_SEED, TAB_ROWS, 9, 2 if binary_classification else 3)
    return dl


def amf_batch(n, size, seed):
    """pet1451 / mri volumes as batch_for, plus the 9 tabular features (float64)."""
    from oracle import tabpfn_standin
    b = batch_for((n, size, size, size), 2, seed, keys=("pet1451", "mri"))
    b["tabular"] = tabpfn_standin.training_table(seed + 50, n)[0]
    return b


def amf_hparams(lr_pretrained):
    """Stage-2 / stage-3 hparams of the all-modalities case (paths are registry keys)."""
    common = dict(ensemble_size=4, lr_pretrained=lr_pretrained)
    return {
        "anat_pet.ckpt": anat_hparams(10, fl_gamma=2, path_pet="pet.ckpt", path_mri="mri.ckpt",
                                      **common),
        "anat_tab.ckpt": anat_hparams(10, path_mri="mri.ckpt", **common),
        "pet_tab.ckpt": anat_hparams(10, fl_gamma=1, simple_dim_red=True, path_pet="pet.ckpt",
                                     **common),
        "stage3": anat_hparams(10, fl_gamma=2, path_anat_pet="anat_pet.ckpt",
                               path_anat_tab="anat_tab.ckpt", path_pet_tab="pet_tab.ckpt",
                               path_pet="pet.ckpt", path_anat="mri.ckpt", **common),
    }


@case
def all_modalities_fusion():
    """The reference's stage-3 ``All_Modalities_Fusion`` (all_modalities_fusion.py:12-96)
    over its real stage-2 classes -- Anat_PET_CNN, Tabular_MRT_Model, PET_TABULAR_CNN -- and
    their stage-1 Small_PET_CNN / Anat_CNN, every ``load_from_checkpoint`` answered from a
    registry of freshly built models (the weights then come from the prng, as everywhere).
    Only TabPFN is the stand-in (install_tabpfn_standin).  lr_pretrained is set at both
    stages so nothing is frozen and every part gets a gradient (the cuts, the concat order
    and the stage-3 head are all on the gradient path); the trainable-parameter names of
    the default (frozen) build are recorded beside it (``frozen_trainable``)."""
    install_tabpfn_standin()
    from pkg.models.pet_models.pet_cnn import Small_PET_CNN
    from pkg.models.mri_models.anat_cnn import Anat_CNN
    from pkg.models.fusion_models.anat_pet_fusion import Anat_PET_CNN
    from pkg.models.fusion_models.tabular_mri_fusion import Tabular_MRT_Model
    from pkg.models.fusion_models.pet_tabular_fusion import PET_TABULAR_CNN
    from pkg.models.fusion_models.all_modalities_fusion import All_Modalities_Fusion

    def build(lr_pretrained):
        hp = amf_hparams(lr_pretrained)
        registry = {"pet.ckpt": (Small_PET_CNN, pet_hparams()),
                    "mri.ckpt": (Anat_CNN, anat_hparams(10)),
                    "anat_pet.ckpt": (Anat_PET_CNN, hp["anat_pet.ckpt"]),
                    "anat_tab.ckpt": (Tabular_MRT_Model, hp["anat_tab.ckpt"]),
                    "pet_tab.ckpt": (PET_TABULAR_CNN, hp["pet_tab.ckpt"])}
        classes = (Small_PET_CNN, Anat_CNN, Anat_PET_CNN, Tabular_MRT_Model, PET_TABULAR_CNN)
        orig = {c: c.__dict__.get("load_from_checkpoint") for c in classes}
        for c in classes:
            c.load_from_checkpoint = classmethod(
                lambda cls, path, **kw: registry[path][0](dict(registry[path][1]), **kw))
        try:
            return All_Modalities_Fusion(hp["stage3"])
        finally:
            for c, f in orig.items():
                if f is None:
                    del c.load_from_checkpoint

    torch.manual_seed(0)
    frozen = build(None)
    torch.manual_seed(0)
    m = build(1e-5)
    load_prng_weights(m, 41)
    out = {"seed": np.array(41), "shape": np.array([2, 32, 32, 32])}
    run_case(m, amf_batch(2, 32, 42), out)
    out["frozen_trainable"] = np.array([n for n, p in frozen.named_parameters()
                                        if p.requires_grad])
    out["frozen_state_dict_keys"] = np.array(list(frozen.state_dict().keys()))
    return out


def ef_hparams(n_classes=2, **kw):
    """train_early_fusion.py:236-254 best configuration, dropout keys removed."""
    h = {"n_classes": n_classes, "conv_out": [8, 16, 32, 64], "filter_size": [7, 5, 3, 3],
         "batchnorm": False, "linear_out": 64, "lr": 1e-3, "reduce_factor_lr_schedule": None,
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


def fmf_hparams(mode, n_classes=2, **kw):
    """train_anat_pet_featuremapfusion.py:282-306 best 2-class maxout configuration,
    dropout keys removed."""
    h = {"n_classes": n_classes, "conv_out": [16, 32, 64], "filter_size": [5, 5, 5],
         "filter_size_fusion": 5, "batchnorm": False, "batchnorm_fusion": False,
         "fusion_mode": mode, "n_layers_fusion": 1, "n_out_fusion": 64, "lr": 2e-4,
         "l2_reg": 0, "reduce_factor_lr_schedule": 0.1,
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


@case
def early_fusion():
    from pkg.models.fusion_models.early_fusion import PET_MRI_EF
    m = PET_MRI_EF(ef_hparams())
    load_prng_weights(m, 23)
    out = {"seed": np.array(23), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 2, 24, keys=("pet1451", "mri")), out)
    return out


@case
def early_fusion_bn3():
    from pkg.models.fusion_models.early_fusion import PET_MRI_EF
    m = PET_MRI_EF(ef_hparams(n_classes=3, batchnorm=True, conv_out=[16, 32, 64],
                              filter_size=[5, 5, 3], linear_out=None))
    load_prng_weights(m, 25)
    out = {"seed": np.array(25), "shape": np.array([3, 32, 32, 32])}
    run_case(m, batch_for((3, 32, 32, 32), 3, 26, keys=("pet1451", "mri")), out)
    return out


@case
def fmf_maxout():
    from pkg.models.fusion_models.anat_pet_featuremapfusion import PET_MRI_FMF
    m = PET_MRI_FMF(fmf_hparams("maxout"))
    load_prng_weights(m, 27)
    out = {"seed": np.array(27), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 2, 28, keys=("pet1451", "mri")), out)
    return out


@case
def fmf_concat_bn():
    from pkg.models.fusion_models.anat_pet_featuremapfusion import PET_MRI_FMF
    m = PET_MRI_FMF(fmf_hparams("concatenate", n_classes=3, batchnorm=True,
                                batchnorm_fusion=True, conv_out=[8, 16, 32],
                                filter_size=[7, 5, 3], filter_size_fusion=3,
                                n_out_fusion=128))
    load_prng_weights(m, 29)
    out = {"seed": np.array(29), "shape": np.array([2, 32, 32, 32])}
    run_case(m, batch_for((2, 32, 32, 32), 3, 30, keys=("pet1451", "mri")), out)
    return out


def _live_seed(build, batch, seed):
    """First weight seed (upwards in steps of 1000) whose train-mode logits keep a positive
    entry in every sample (the head's final ReLU, anat_cnn.py:77, otherwise zeroes every
    gradient); forward only, so the search stays cheap at 128^3."""
    for s in range(seed, seed + 50000, 1000):
        m = build()
        load_prng_weights(m, s)
        m.train()
        with torch.no_grad():
            y = m.general_step(batch, 0, "train")["outputs"]
        if (y > 0).any(dim=1).all():
            return s
    raise RuntimeError("no live seed")


FULL = (8, 128, 128, 128)          # BASELINE configs 2 and 3: batch 8 of 1 x 128^3


def calibrate_bn(model, batch, out):
    """BN running statistics = this batch's statistics (one train-mode forward with a
    cumulative average), so eval mode normalises like train mode instead of running a
    fresh network un-normalised (whose pooled features are huge and nearly parallel);
    num_batches_tracked back to 0.  Recorded as ``init_buf/<name>``; the tests load them."""
    bns = [m for m in model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)]
    with torch.no_grad():
        saved = [b.momentum for b in bns]
        for b in bns:
            b.momentum = None
            b.reset_running_stats()
        model.train()
        model.general_step(batch, 0, "train")
        for b, mo in zip(bns, saved):
            b.momentum = mo
            b.num_batches_tracked.zero_()
    for name, b in model.named_buffers():
        if "running" in name:
            out[f"init_buf/{name}"] = b.detach().numpy().copy()


def mixed_head(model, head, prefix, batch, out):
    """Make a full-size case discriminating.  With random weights the pooled 512-d features
    of different volumes are nearly parallel, so every sample gets the same argmax (and the
    head's closing ReLU, anat_cnn.py:76-77, zeroed all eval rows of the round-3 fixture).
    The final Linear (``head``, parameters ``prefix`` + weight / bias) is replaced by
    w0 = p / 2, w1 = -p / 2 and a bias, with p the least-norm direction that puts each
    sample's train logit difference z0 - z1 at a chosen target t_b while staying orthogonal
    to the mean train and eval features (so neither mode's common part reaches the logits).
    Targets: the argmax is split across the batch, and the per-sample loss gradients
    (p0 - y0, sign fixed by the label) do not cancel: samples of one class sit confidently
    on their side (|t| ~ 3, small gradient), those of the other weakly (|t| ~ 0.4, large
    gradient) -- a symmetric split makes every weight gradient a difference of two nearly
    equal per-sample terms, which is what a bf16 check cannot resolve.  The bias keeps every
    train logit positive (every eval row has a positive entry).  The replaced tensors are
    recorded in the fixture (``head_prefix``, ``head_weight``, ``head_bias``); the tests load
    them after the prng weights.  The model's state (BN running statistics) is restored after
    the probes, and eval is probed first, as run_full_case evaluates."""
    feats = {}
    hook = head.register_forward_hook(
        lambda mod, inp, o: feats.__setitem__("x", inp[0].detach().double()))
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        model.eval()
        model.general_step(batch, 0, "val")
        fe = feats["x"]
        model.train()
        model.general_step(batch, 0, "train")
        ft = feats["x"]
    hook.remove()
    model.load_state_dict(sd)
    model.train()
    labels = batch["label"].numpy()
    n = ft.shape[0]
    jit = np.linspace(-0.1, 0.1, n)
    t = np.empty(n)
    if labels.min() != labels.max():
        # label 0 confidently right (z0 - z1 = +3), label 1 weakly right (-0.4)
        t[:] = np.where(labels == 0, 3.0, -0.4) + jit
    else:
        # one class only: half confidently right, half weakly wrong (same gradient sign)
        s = 1.0 if labels[0] == 0 else -1.0
        t[:] = s * np.where(np.arange(n) % 2 == 0, 3.0, -0.4) + jit
    tb = torch.from_numpy(t)
    mean = ft.mean(0)
    A = torch.cat([ft - mean, mean[None], fe.mean(0)[None]])
    rhs = torch.cat([tb - tb.mean(), torch.zeros(2, dtype=torch.float64)])
    p = torch.linalg.pinv(A) @ rhs
    w = torch.stack([p / 2, -p / 2])
    delta = float(tb.mean())                                     # b0 - b1
    z = ft @ w.t()
    need = max(float(-(z[:, 0] + delta / 2).min()), float(-(z[:, 1] - delta / 2).min()))
    c = need + 0.25
    bias = torch.tensor([c + delta / 2, c - delta / 2], dtype=torch.float32)
    with torch.no_grad():
        head.weight.copy_(w.float())
        head.bias.copy_(bias)
    zt = z + bias.double()
    margin = float((zt[:, 0] - zt[:, 1]).abs().min())
    ze = fe @ w.t() + bias.double()
    out["head_prefix"] = np.array(prefix)
    out["head_weight"] = head.weight.detach().numpy().copy()
    out["head_bias"] = bias.numpy()
    out["head_margin"] = np.array(margin)
    print(f"  mixed head: labels {labels.tolist()}, |p| {float(p.norm()):.3e}, bias "
          f"{bias.tolist()}, train argmax margin {margin:.3e}, train logits {zt.tolist()}, "
          f"eval logits {ze.tolist()}")


@case
def anat_r10_128():
    """BASELINE config 2 at its full size: Anat_CNN ResNet-10, 8 x 1 x 128^3, weighted CE
    (anat_cnn.py:13-109, the reference code itself; MedicalNet from the restatement)."""
    from pkg.models.mri_models.anat_cnn import Anat_CNN
    batch = batch_for(FULL, 2, 1301)
    torch.manual_seed(0)
    seed = 1300
    m = Anat_CNN(anat_hparams(10))
    load_prng_weights(m, seed)
    out = {"seed": np.array(seed), "shape": np.array(FULL)}
    calibrate_bn(m, batch, out)
    mixed_head(m, m.model.conv_seg[-2], "model.conv_seg.2.", batch, out)
    run_full_case(m, models_ref.AnatCNNRef(anat_hparams(10)), batch,
                  lambda b: (b["mri"].unsqueeze(1).double(),), out)
    return out


def pair_stage1(h, depth):
    return dict(h, resnet_depth=depth, linear_out=[], conv_out=[], filter_size=[],
                batchnorm_begin=False, batchnorm_dense=False)


@case
def pair_r10_128():
    """BASELINE config 3 at its full size: PET+MRI ResNet-10 x2 + MLP head, 8 pairs of
    1 x 128^3, focal loss gamma 2.  The two branches are the reference's own PET_CNN_ResNet
    (pet_resnet_cnn.py:12-138) and Anat_CNN (anat_cnn.py:13-109); the two-backbone head
    wiring is a BUILD EXTENSION (oracle ResNetPairFusionRef), so this
    fixture is pinned for the branches and unpinned for the head."""
    from pkg.models.mri_models.anat_cnn import Anat_CNN
    from pkg.models.pet_models.pet_resnet_cnn import PET_CNN_ResNet
    h = anat_hparams(10, fl_gamma=2)
    torch.manual_seed(0)
    m = models_ref.ResNetPairFusionRef(h, PET_CNN_ResNet(pair_stage1(h, 10)),
                                       Anat_CNN(pair_stage1(h, 10)))
    load_prng_weights(m, 1400)
    ref64 = models_ref.ResNetPairFusionRef(h, models_ref.PETResNetRef(pair_stage1(h, 10)),
                                           models_ref.AnatCNNRef(pair_stage1(h, 10)))
    out = {"seed": np.array(1400), "shape": np.array(FULL)}
    run_full_case(m, ref64, batch_for(FULL, 2, 1401, keys=("pet1451", "mri")),
                  lambda b: (b["pet1451"].unsqueeze(1).double(), b["mri"].unsqueeze(1).double()),
                  out)
    return out


PET160 = (2, 160, 160, 160)        # BASELINE config 5's volume size


@case
def pet_r18_160():
    """BASELINE config 5's PET branch at its full size: the reference's own PET_CNN_ResNet
    with depth 18 (pet_resnet_cnn.py:12-138; MedicalNet from the restatement), 2 x 1 x 160^3,
    focal loss gamma 2.  Its layer3 / layer4 run on 20^3 grids (10- and 5-wide dilated
    sub-lattices), the route the config-5 bench takes."""
    from pkg.models.pet_models.pet_resnet_cnn import PET_CNN_ResNet
    h = anat_hparams(18, fl_gamma=2)
    batch = batch_for(PET160, 2, 1501, keys=("pet1451",))
    torch.manual_seed(0)
    m = PET_CNN_ResNet(h)
    load_prng_weights(m, 1500)
    out = {"seed": np.array(1500), "shape": np.array(PET160)}
    calibrate_bn(m, batch, out)
    mixed_head(m, m.model.conv_seg[-2], "model.conv_seg.2.", batch, out)
    run_full_case(m, models_ref.PETResNetRef(h), batch,
                  lambda b: (b["pet1451"].unsqueeze(1).double(),), out)
    return out


# batch 4: at batch 2 the head's gradient is two per-sample loss-gradient scalars times the
# features, too few for a normwise bf16 comparison of the 36-layer chain (round 5)
R34_160 = (4, 160, 160, 160)


@case
def anat_r34_160():
    """BASELINE config 5's MRI branch at its full size: Anat_CNN on MedicalNet ResNet-34,
    4 x 1 x 160^3, focal loss gamma 2.  The reference's Anat_CNN rejects depth 34 (its depth
    match, anat_cnn.py:37-46, has no case for it; config 5 names it), so this case runs the
    oracle restatement in fp32 as the "reference" (parity unpinned against the reference
    code itself; the ResNet-34 wiring -- 3 / 4 / 6 / 3 BasicBlocks, MedicalNet's depth table
    -- checked against an independent CPU implementation instead of the HIP path's own fp32
    run)."""
    h = anat_hparams(34, fl_gamma=2)
    batch = batch_for(R34_160, 2, 1601)
    torch.manual_seed(0)
    m = models_ref.AnatCNNRef(h)
    load_prng_weights(m, 1600)
    out = {"seed": np.array(1600), "shape": np.array(R34_160)}
    calibrate_bn(m, batch, out)
    mixed_head(m, m.model.conv_seg[-2], "model.conv_seg.2.", batch, out)
    run_full_case(m, models_ref.AnatCNNRef(h), batch,
                  lambda b: (b["mri"].unsqueeze(1).double(),), out)
    return out


TRI160 = (2, 160, 160, 160)


def tri_hparams():
    """config 5's network: MRI ResNet-34 + PET ResNet-18 + tabular MLP (as
    tests/test_fusion_configs_gpu._hp("three"))."""
    return anat_hparams(10, fl_gamma=2, resnet_depth_mri=34, resnet_depth_pet=18)


def tri_ref(h):
    st = dict(h, linear_out=[], conv_out=[], filter_size=[], batchnorm_begin=False,
              batchnorm_dense=False)
    return models_ref.TriResNetTabularRef(h, models_ref.AnatCNNRef(dict(st, resnet_depth=34)),
                                          models_ref.PETResNetRef(dict(st, resnet_depth=18)))


@case
def tri_160():
    """BASELINE config 5's whole network at its full size (Tri_ResNet_Tabular_Fusion, a build
    extension: MRI ResNet-34 + PET ResNet-18 + tabular MLP, 2 x 160^3 pairs + 9 tabular
    features, focal loss gamma 2).  No reference class exists for it, so the "reference" is
    the oracle restatement (oracle/models_ref.py TriResNetTabularRef) in fp32, with its float64
    and CPU-autocast bf16 evaluations beside it: the GPU test measures the HIP path against an
    independent CPU implementation at full size (its branches are pinned to the reference
    code by pet_r18_160 and, for the ResNet-34 wiring, by anat_r34_160)."""
    from oracle import tabpfn_standin
    h = tri_hparams()
    batch = batch_for(TRI160, 2, 1701, keys=("pet1451", "mri"))
    batch["tabular"] = tabpfn_standin.training_table(1751, TRI160[0])[0]
    torch.manual_seed(0)
    m = tri_ref(h)
    load_prng_weights(m, 1700)
    out = {"seed": np.array(1700), "shape": np.array(TRI160)}
    calibrate_bn(m, batch, out)
    mixed_head(m, m.cls3, "cls3.", batch, out)
    run_full_case(m, tri_ref(h), batch, lambda b: m.inputs(b, torch.float64), out)
    return out


def main(names=None):
    install_stubs()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    for name, fn in CASES.items():
        if names and name not in names:
            continue
        out = fn()
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(f"{name}: {len(out)} arrays -> {os.path.getsize(path) / 1024:.1f} KiB")


if __name__ == "__main__":
    main(sys.argv[1:] or None)
