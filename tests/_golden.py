"""Helpers shared by the parity tests: rebuild the golden cases' models and batches."""
import os

import numpy as np
import torch

from oracle import prng, models_ref

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
W2 = [0.20314960629921264, 0.7968503937007874]
W3 = [0.4651162790697675, 0.6712473572938689, 0.8636363636363636]


def load(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


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


def ef_hparams(n_classes=2, **kw):
    """PET_MRI_EF case hparams (mirror of tests/golden/make_golden.py)."""
    h = {"n_classes": n_classes, "conv_out": [8, 16, 32, 64], "filter_size": [7, 5, 3, 3],
         "batchnorm": False, "linear_out": 64, "lr": 1e-3, "reduce_factor_lr_schedule": None,
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


def fmf_hparams(mode, n_classes=2, **kw):
    """PET_MRI_FMF case hparams (mirror of tests/golden/make_golden.py)."""
    h = {"n_classes": n_classes, "conv_out": [16, 32, 64], "filter_size": [5, 5, 5],
         "filter_size_fusion": 5, "batchnorm": False, "batchnorm_fusion": False,
         "fusion_mode": mode, "n_layers_fusion": 1, "n_out_fusion": 64, "lr": 2e-4,
         "l2_reg": 0, "reduce_factor_lr_schedule": 0.1,
         "loss_class_weights": torch.tensor(W2 if n_classes == 2 else W3, dtype=torch.double)}
    h.update(kw)
    return h


TAB_SEED, TAB_ROWS = 4242, 16        # make_golden.install_tabpfn_standin


def amf_hparams(lr_pretrained):
    """Stage-2 / stage-3 hparams of the all_modalities_fusion case (mirror of
    make_golden.amf_hparams; the paths are file names inside the checkpoint directory)."""
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


def tabpfn_backend():
    from oracle import tabpfn_standin
    return tabpfn_standin.make_backend(TAB_SEED, TAB_ROWS)


def amf_checkpoint_chain(tmp_dir, lr_pretrained=1e-5):
    """The reference's three-stage chain on the drop-in classes, through PL checkpoint
    files: stage-1 Small_PET_CNN / Anat_CNN saved, stage-2 Anat_PET_CNN /
    Tabular_MRT_Model / PET_TABULAR_CNN built from those paths and saved, then
    All_Modalities_Fusion(hparams) loading all five (all_modalities_fusion.py:17-26).
    TabPFN is the oracle stand-in (registered with tabular.set_backend).  Returns the
    stage-3 model (on the CPU, weights as built)."""
    import multimodal_alzheimer_amd as M
    from multimodal_alzheimer_amd import tabular
    tabular.set_backend(tabpfn_backend())
    hp = amf_hparams(lr_pretrained)
    path = {k: os.path.join(tmp_dir, k) for k in
            ("pet.ckpt", "mri.ckpt", "anat_pet.ckpt", "anat_tab.ckpt", "pet_tab.ckpt")}

    def fix(h):
        return {k: (path[v] if isinstance(v, str) and v in path else v) for k, v in h.items()}

    torch.manual_seed(0)
    M.Small_PET_CNN(pet_hparams()).save_checkpoint(path["pet.ckpt"])
    M.Anat_CNN(anat_hparams(10)).save_checkpoint(path["mri.ckpt"])
    h = fix(hp["anat_pet.ckpt"])
    M.Anat_PET_CNN(h, path_pet=h["path_pet"], path_anat=h["path_mri"]).save_checkpoint(
        path["anat_pet.ckpt"])
    h = fix(hp["anat_tab.ckpt"])
    M.Tabular_MRT_Model(h, path_mri=h["path_mri"]).save_checkpoint(path["anat_tab.ckpt"])
    h = fix(hp["pet_tab.ckpt"])
    M.PET_TABULAR_CNN(h, path_pet=h["path_pet"]).save_checkpoint(path["pet_tab.ckpt"])
    return M.All_Modalities_Fusion(fix(hp["stage3"]))


def build_amf_oracle(h3):
    hp = amf_hparams(1e-5)
    load = tabpfn_backend()
    ap = models_ref.AnatPETCNNRef(hp["anat_pet.ckpt"], models_ref.SmallPETCNNRef(pet_hparams()),
                                  models_ref.AnatCNNRef(anat_hparams(10)))
    at = models_ref.TabularMRTRef(hp["anat_tab.ckpt"], models_ref.AnatCNNRef(anat_hparams(10)),
                                  load(None, True, 4))
    pt = models_ref.PETTabularRef(hp["pet_tab.ckpt"], models_ref.SmallPETCNNRef(pet_hparams()),
                                  load(None, True, 4))
    return models_ref.AllModalitiesFusionRef(h3, ap, at, pt)


def batch_for(shape, n_classes, seed, keys=("mri",)):
    b = {"label": torch.from_numpy(prng.labels(seed + 7, shape[0], n_classes))}
    for i, k in enumerate(keys):
        gen = prng.mri_volume if k == "mri" else prng.pet_volume
        b[k] = torch.from_numpy(gen(seed + i, shape)).double()
    return b


def load_prng_weights(model, seed):
    sd = model.state_dict()
    vals = prng.fill_state_dict(sd, seed)
    with torch.no_grad():
        for k, v in vals.items():
            sd[k].copy_(torch.from_numpy(v))


def load_fixture_weights(model, g):
    """A fixture's weights: the prng tensors of its seed, then (full-size cases) the BN
    running statistics and the discriminating final Linear the generator recorded
    (make_golden.calibrate_bn / mixed_head)."""
    load_prng_weights(model, int(g["seed"]))
    bufs = dict(model.named_buffers())
    with torch.no_grad():
        for k in g:
            if k.startswith("init_buf/"):
                bufs[k[len("init_buf/"):]].copy_(torch.from_numpy(g[k]))
    if "head_prefix" in g:
        params = dict(model.named_parameters())
        with torch.no_grad():
            params[str(g["head_prefix"]) + "weight"].copy_(torch.from_numpy(g["head_weight"]))
            params[str(g["head_prefix"]) + "bias"].copy_(torch.from_numpy(g["head_bias"]))


# name -> (hparams-builder, kind, batch seed, keys); weights seed = fixture 'seed'
CASES = {
    "anat_r10_32": (lambda: anat_hparams(10), "anat", 12, ("mri",)),
    "anat_r10_64": (lambda: anat_hparams(10), "anat", 13, ("mri",)),
    "anat_r10_32_live": (lambda: anat_hparams(10), "anat", 32, ("mri",)),
    "anat_r10_64_live": (lambda: anat_hparams(10), "anat", 33, ("mri",)),
    "anat_r10_mni": (lambda: anat_hparams(10), "anat", 1035, ("mri",)),
    "anat_r50": (lambda: anat_hparams(50), "anat", 36, ("mri",)),
    "anat_conv_out": (lambda: anat_hparams(10, n_classes=3, batchnorm_begin=True,
                                           conv_out=[32], filter_size=[3],
                                           batchnorm_conv=True, linear_out=[16]),
                      "anat", 37, ("mri",)),
    "anat_r18_head": (lambda: anat_hparams(18, n_classes=3, batchnorm_begin=True,
                                           batchnorm_dense=True, linear_out=[64, 32],
                                           fl_gamma=2), "anat", 14, ("mri",)),
    "anat_r10_focal": (lambda: anat_hparams(10, fl_gamma=5, linear_out=[128]), "anat", 15,
                       ("mri",)),
    "pet_resnet_r10": (lambda: anat_hparams(10, fl_gamma=1), "petres", 16, ("pet1451",)),
    "small_pet": (lambda: pet_hparams(), "smallpet", 18, ("pet1451",)),
    "small_pet_bn3": (lambda: pet_hparams(n_classes=3, batchnorm=True, conv_out=(16, 32, 64),
                                          filter_size=(7, 5, 3), linear_out=32),
                      "smallpet", 20, ("pet1451",)),
    "anat_pet_fusion": (lambda: anat_hparams(10, fl_gamma=2), "fusion", 22,
                        ("pet1451", "mri")),
    "all_modalities_fusion": (lambda: amf_hparams(1e-5)["stage3"], "amf", 42,
                              ("pet1451", "mri")),
    "early_fusion": (lambda: ef_hparams(), "ef", 24, ("pet1451", "mri")),
    "early_fusion_bn3": (lambda: ef_hparams(n_classes=3, batchnorm=True, conv_out=[16, 32, 64],
                                            filter_size=[5, 5, 3], linear_out=None),
                         "ef", 26, ("pet1451", "mri")),
    "fmf_maxout": (lambda: fmf_hparams("maxout"), "fmf", 28, ("pet1451", "mri")),
    "fmf_concat_bn": (lambda: fmf_hparams("concatenate", n_classes=3, batchnorm=True,
                                          batchnorm_fusion=True, conv_out=[8, 16, 32],
                                          filter_size=[7, 5, 3], filter_size_fusion=3,
                                          n_out_fusion=128), "fmf", 30, ("pet1451", "mri")),
}


def build_oracle(name):
    hp_fn, kind, _, _ = CASES[name]
    h = hp_fn()
    if kind == "anat":
        return models_ref.AnatCNNRef(h)
    if kind == "petres":
        m = models_ref.PETResNetRef(h)
        return m
    if kind == "smallpet":
        return models_ref.SmallPETCNNRef(h)
    if kind == "fusion":
        pet = models_ref.SmallPETCNNRef(pet_hparams())
        mri = models_ref.AnatCNNRef(anat_hparams(10))
        return models_ref.AnatPETCNNRef(h, pet, mri)
    if kind == "amf":
        return build_amf_oracle(h)
    if kind == "ef":
        return models_ref.EarlyFusionRef(h)
    if kind == "fmf":
        return models_ref.FeatureMapFusionRef(h)
    raise KeyError(kind)


def batch_of(name, g):
    _, kind, bseed, keys = CASES[name]
    shape = tuple(int(v) for v in g["shape"])
    n_classes = g["train_logits"].shape[1]
    b = batch_for(shape, n_classes, bseed, keys)
    if kind == "amf":                      # make_golden.amf_batch
        from oracle import tabpfn_standin
        b["tabular"] = tabpfn_standin.training_table(bseed + 50, shape[0])[0]
    return b


def fusion_via_stage1_checkpoints(tmp_dir):
    """The reference's stage chain (anat_pet_fusion.py:17-32): stage-1 Small_PET_CNN and
    Anat_CNN saved as PL checkpoints, the fusion built from the two paths.  Weights are the
    golden `anat_pet_fusion` case's: the backbone tensors travel through the checkpoints,
    the stage-2 head is loaded afterwards.  Returns (fusion model, golden state dict)."""
    import multimodal_alzheimer_amd as M
    g = load("anat_pet_fusion")
    h = CASES["anat_pet_fusion"][0]()
    fus0 = M.Anat_PET_CNN(h, pet_model=M.Small_PET_CNN(pet_hparams()),
                          mri_model=M.Anat_CNN(anat_hparams(10)))
    load_prng_weights(fus0, int(g["seed"]))
    sd = fus0.state_dict()
    pet, mri = M.Small_PET_CNN(pet_hparams()), M.Anat_CNN(anat_hparams(10))
    with torch.no_grad():
        for prefix, mdl, sub in (("model_pet.", pet, "model."), ("model_mri.", mri, "")):
            own = mdl.state_dict()
            for k, v in sd.items():
                if k.startswith(prefix):
                    own[sub + k[len(prefix):]].copy_(v)
    p_pet, p_mri = os.path.join(tmp_dir, "pet.ckpt"), os.path.join(tmp_dir, "mri.ckpt")
    pet.save_checkpoint(p_pet)
    mri.save_checkpoint(p_mri)
    fus = M.Anat_PET_CNN(h, path_pet=p_pet, path_anat=p_mri)
    head = {k: v for k, v in sd.items() if not k.startswith(("model_pet.", "model_mri."))}
    missing, unexpected = fus.load_state_dict(head, strict=False)
    assert not unexpected
    assert all(k.startswith(("model_pet.", "model_mri.")) for k in missing)
    return fus, sd
