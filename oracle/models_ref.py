"""torch-CPU restatement of the reference hot-path modules (TEST INFRASTRUCTURE ONLY).

Each class / function cites the reference file:line it restates.  Parameter and buffer
names are kept identical to the reference modules so one state_dict (and one PRNG fill,
``oracle.prng.fill_state_dict``) drives the reference, this oracle and the HIP product.
Pinned by ``tests/golden/*.npz`` (produced from the real reference code by
``tests/golden/make_golden.py``) in ``tests/test_oracle_golden.py``.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .medicalnet_ref import ResNetRef

RESNET_OUT = {10: 512, 18: 512, 34: 512, 50: 2048}


def build_conv_seg(hparams, n_in):
    """Replacement ``conv_seg`` head: anat_cnn.py:33-79 (same in pet_resnet_cnn.py:37-81).

    [BN3d(n_in)] -> [Conv3d 'same' -> [BN3d] -> ReLU -> MaxPool3d(2)]* -> GAP -> Flatten
    -> [Linear -> [BN1d] -> ReLU]* -> Linear(., C) -> ReLU (sic: logits are >= 0).
    """
    mods = []
    if hparams.get("batchnorm_begin"):
        mods.append(nn.BatchNorm3d(n_in))
    if "conv_out" in hparams:
        for n_out, k in zip(hparams["conv_out"], hparams["filter_size"]):
            mods.append(nn.Conv3d(n_in, n_out, k, padding="same"))
            if hparams["batchnorm_conv"]:
                mods.append(nn.BatchNorm3d(n_out))
            mods += [nn.ReLU(), nn.MaxPool3d(2)]
            n_in = n_out
    mods += [nn.AdaptiveAvgPool3d(1), nn.Flatten()]
    for n_out in hparams["linear_out"]:
        mods.append(nn.Linear(n_in, n_out))
        if hparams.get("batchnorm_dense"):
            mods.append(nn.BatchNorm1d(n_out))
        mods.append(nn.ReLU())
        n_in = n_out
    mods += [nn.Linear(n_in, hparams["n_classes"]), nn.ReLU()]
    return nn.Sequential(*mods)


class FocalLossRef(nn.Module):
    """pkg/loss_functions/focalloss.py:10-39 with alpha=None (every caller).

    logpt = log_softmax(x)[y]; pt = exp(logpt) DETACHED (focalloss.py:29,
    ``Variable(logpt.data.exp())``); loss = mean(-(1 - pt)**gamma * logpt).
    """

    def __init__(self, gamma=0):
        super().__init__()
        self.gamma = gamma

    def forward(self, x, y):
        logpt = F.log_softmax(x, dim=1).gather(1, y.view(-1, 1)).view(-1)
        pt = logpt.detach().exp()
        return (-1 * (1 - pt) ** self.gamma * logpt).mean()


def make_criterion(hparams):
    """anat_cnn.py:81-85: focal loss iff hparams['fl_gamma'] is truthy, else weighted CE."""
    if hparams.get("fl_gamma"):
        return FocalLossRef(hparams["fl_gamma"])
    return nn.CrossEntropyLoss(weight=hparams["loss_class_weights"])


class _StepMixin:
    batch_key = "mri"

    def general_step(self, batch, batch_idx=0, mode="train"):
        """anat_cnn.py:99-109: unsqueeze(1), cast fp32, forward, cast logits fp64, loss."""
        x = batch[self.batch_key].unsqueeze(1).to(dtype=torch.float32)
        y = batch["label"]
        y_hat = self(x).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, y), "outputs": y_hat, "labels": y}


class AnatCNNRef(_StepMixin, nn.Module):
    """Anat_CNN (pkg/models/mri_models/anat_cnn.py:13-109) on the MedicalNet restatement."""

    def __init__(self, hparams):
        super().__init__()
        self.hparams = dict(hparams)
        self.model = ResNetRef(hparams["resnet_depth"])
        self.model.conv_seg = build_conv_seg(hparams, RESNET_OUT[hparams["resnet_depth"]])
        self.criterion = make_criterion(hparams)

    def forward(self, x):
        return self.model(x)


class PETResNetRef(AnatCNNRef):
    """PET_CNN_ResNet (pkg/models/pet_models/pet_resnet_cnn.py:12-138): same net, PET key."""
    batch_key = "pet1451"


class SmallPETCNNRef(_StepMixin, nn.Module):
    """Small_PET_CNN (pkg/models/pet_models/pet_cnn.py:10-70); always weighted CE (:47-48)."""
    batch_key = "pet1451"

    def __init__(self, hparams):
        super().__init__()
        self.hparams = dict(hparams)
        mods = []
        n_in = 1
        n_out = None
        for n_out, k in zip(hparams["conv_out"], hparams["filter_size"]):
            mods.append(nn.Conv3d(n_in, n_out, k, padding="same"))
            if hparams.get("batchnorm"):
                mods.append(nn.BatchNorm3d(n_out))
            mods += [nn.ReLU(), nn.MaxPool3d(2)]
            if "dropout_conv_p" in hparams:
                mods.append(nn.Dropout(p=hparams["dropout_conv_p"]))
            n_in = n_out
        mods += [nn.AdaptiveAvgPool3d(1), nn.Flatten()]
        if hparams.get("linear_out"):
            n_out = hparams["linear_out"]
            if "dropout_dense_p" in hparams:
                mods.append(nn.Dropout(p=hparams["dropout_dense_p"]))
            mods += [nn.Linear(n_in, n_out), nn.ReLU()]
        mods.append(nn.Linear(n_out, hparams["n_classes"]))
        self.model = nn.Sequential(*mods)
        self.criterion = nn.CrossEntropyLoss(weight=hparams["loss_class_weights"])

    def forward(self, x):
        return self.model(x)


class AnatPETCNNRef(nn.Module):
    """Anat_PET_CNN late fusion (pkg/models/fusion_models/anat_pet_fusion.py:11-92).

    ``model_pet`` is a stage-1 Small_PET_CNN cut after GAP+Flatten(+Linear/ReLU)
    (:28-31), ``model_mri`` a stage-1 Anat_CNN whose conv_seg is cut to [:2] (:32);
    head: cat(pet 64, reduce_dim_mri(512->64)+ReLU) -> Linear(128,64) -> ReLU ->
    Linear(64,C) (:42-51), no final ReLU.
    """

    def __init__(self, hparams, pet_stage1, mri_stage1):
        super().__init__()
        self.hparams = dict(hparams)
        if hparams["n_classes"] == 2:
            self.model_pet = pet_stage1.model[:-3]
        else:
            self.model_pet = pet_stage1.model[:-1]
        self.model_mri = mri_stage1
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.stage2out = nn.Linear(128, 64)
        self.cls2 = nn.Linear(64, hparams["n_classes"])
        self.relu = nn.ReLU()
        self.reduce_dim_mri = nn.Sequential(nn.Linear(512, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)

    def forward(self, x_pet, x_mri):
        bs = x_mri.shape[0]
        out_pet = self.model_pet(x_pet)
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        return self.model_fuse(torch.cat((out_pet, out_mri), dim=1))

    def general_step(self, batch, batch_idx=0, mode="train"):
        """anat_pet_fusion.py:80-92."""
        x_pet = batch["pet1451"].unsqueeze(1).to(dtype=torch.float32)
        x_mri = batch["mri"].unsqueeze(1).to(dtype=torch.float32)
        y = batch["label"]
        y_hat = self(x_pet, x_mri).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, y), "outputs": y_hat, "labels": y}


def tabpfn_features(classifier, x_tab, num_ensemble, training_size):
    """tabular_mri_fusion.py:58-74 (= pet_tabular_fusion.py:80-97): hook TabPFN's first
    decoder Linear, predict_proba on the CPU copy, average the test rows over the ensemble
    members (dl_approach.py:71-78)."""
    acts = {}
    h = classifier.model[2].decoder[0].register_forward_hook(
        lambda mod, inp, out: acts.__setitem__("dec", out.detach()))
    classifier.predict_proba(x_tab.cpu().squeeze(dim=1), normalize_with_test=False)
    h.remove()
    out = None
    for i in range(num_ensemble):
        a = acts["dec"][training_size:, i:i + 1, :]
        out = a if out is None else out + a
    return torch.transpose(out / num_ensemble, 0, 1).squeeze(dim=0)


class TabularMRTRef(nn.Module):
    """Tabular_MRT_Model (pkg/models/fusion_models/tabular_mri_fusion.py:11-93): stage-1
    Anat_CNN cut to conv_seg[:2]; TabPFN features -> reduce_tab Linear(1024,512)+ReLU;
    cat(tabular, mri) -> Linear(1024,64) -> ReLU -> Linear(64,C).  ``tabpfn`` = (fitted
    classifier, n_train) as dl_approach.load_model returns it."""

    def __init__(self, hparams, mri_stage1, tabpfn):
        super().__init__()
        self.hparams = dict(hparams)
        self.model_mri = mri_stage1
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.model_tabular, self.tabular_training_size = tabpfn
        self.stage2out = nn.Linear(512 + 512, 64)
        self.cls2 = nn.Linear(64, hparams["n_classes"])
        self.relu = nn.ReLU()
        self.reduce_tab = nn.Sequential(nn.Linear(1024, 512), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)

    def forward(self, x_tabular, x_mri):
        acts = tabpfn_features(self.model_tabular, x_tabular, self.hparams["ensemble_size"],
                               self.tabular_training_size)
        out_tabular = self.reduce_tab(acts.to(self.stage2out.weight.dtype))
        out_mri = self.model_mri(x_mri).squeeze()
        return self.model_fuse(torch.cat((out_tabular, out_mri), dim=1))


class PETTabularRef(nn.Module):
    """PET_TABULAR_CNN (pkg/models/fusion_models/pet_tabular_fusion.py:15-104): stage-1
    Small_PET_CNN cut after GAP+Flatten (model[:-3] / [:-1], :28-31); TabPFN features ->
    reduce_tab (simple_dim_red: 1024->512->64 with ReLUs, else 1024->64 + ReLU, :54-57);
    cat(pet, tabular) -> Linear(128,64) -> ReLU -> Linear(64,C)."""

    def __init__(self, hparams, pet_stage1, tabpfn):
        super().__init__()
        self.hparams = dict(hparams)
        self.model_pet = (pet_stage1.model[:-3] if hparams["n_classes"] == 2
                          else pet_stage1.model[:-1])
        self.model_tabular, self.tabular_training_size = tabpfn
        self.stage2out = nn.Linear(64 + 64, 64)
        self.cls2 = nn.Linear(64, hparams["n_classes"])
        self.relu = nn.ReLU()
        if hparams["simple_dim_red"]:
            self.reduce_tab = nn.Sequential(nn.Linear(1024, 512), self.relu,
                                            nn.Linear(512, 64), self.relu)
        else:
            self.reduce_tab = nn.Sequential(nn.Linear(1024, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)

    def forward(self, x_pet, x_tabular):
        out_pet = self.model_pet(x_pet)
        acts = tabpfn_features(self.model_tabular, x_tabular, self.hparams["ensemble_size"],
                               self.tabular_training_size)
        out_tab = self.reduce_tab(acts.to(self.stage2out.weight.dtype))
        return self.model_fuse(torch.cat((out_pet, out_tab), dim=1))


class AllModalitiesFusionRef(nn.Module):
    """All_Modalities_Fusion (pkg/models/fusion_models/all_modalities_fusion.py:12-96):
    the three stage-2 models with their classifiers cut (model_fuse[:-2] = stage2out
    alone, :29-31), cat(anat_pet, anat_tab, pet_tab) 192 -> Linear(192,64) -> ReLU ->
    Linear(64,C) (:50-57, :74-79)."""

    def __init__(self, hparams, anat_pet, anat_tab, pet_tab):
        super().__init__()
        self.hparams = dict(hparams)
        self.model_anat_pet, self.model_anat_tab, self.model_pet_tab = anat_pet, anat_tab, pet_tab
        for m in (anat_pet, anat_tab, pet_tab):
            m.model_fuse = m.model_fuse[:-2]
        self.stage3out = nn.Linear(64 + 64 + 64, 64)
        self.cls3 = nn.Linear(64, hparams["n_classes"])
        self.relu = nn.ReLU()
        self.model_fuse = nn.Sequential(self.stage3out, self.relu, self.cls3)
        self.criterion = make_criterion(hparams)

    def forward(self, x_pet, x_mri, x_tab):
        out = torch.cat((self.model_anat_pet(x_pet, x_mri), self.model_anat_tab(x_tab, x_mri),
                         self.model_pet_tab(x_pet, x_tab)), dim=1)
        return self.model_fuse(out)

    def inputs(self, batch, dtype=torch.float32):
        return (batch["pet1451"].unsqueeze(1).to(dtype), batch["mri"].unsqueeze(1).to(dtype),
                batch["tabular"].unsqueeze(1).to(torch.float32))

    def general_step(self, batch, batch_idx=0, mode="train"):
        """all_modalities_fusion.py:81-96."""
        y_hat = self(*self.inputs(batch)).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, batch["label"]), "outputs": y_hat,
                "labels": batch["label"]}


class ResNetPairFusionRef(nn.Module):
    """BUILD EXTENSION (BASELINE config 3/4): "ResNet-10 x2 + MLP head".

    Both branches are stage-1 ResNet models cut to conv_seg[:2] (512-d), each reduced
    by Linear(512,64)+ReLU (mirroring ``reduce_dim_mri``, anat_pet_fusion.py:49), then
    the unchanged Anat_PET_CNN head (anat_pet_fusion.py:42-51).  No reference parity.
    """

    def __init__(self, hparams, pet_stage1, mri_stage1):
        super().__init__()
        self.hparams = dict(hparams)
        self.model_pet = pet_stage1
        self.model_pet.model.conv_seg = self.model_pet.model.conv_seg[:2]
        self.model_mri = mri_stage1
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.stage2out = nn.Linear(128, 64)
        self.cls2 = nn.Linear(64, hparams["n_classes"])
        self.relu = nn.ReLU()
        self.reduce_dim_pet = nn.Sequential(nn.Linear(512, 64), self.relu)
        self.reduce_dim_mri = nn.Sequential(nn.Linear(512, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)

    def forward(self, x_pet, x_mri):
        bs = x_mri.shape[0]
        out_pet = self.reduce_dim_pet(self.model_pet(x_pet).view(bs, -1))
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        return self.model_fuse(torch.cat((out_pet, out_mri), dim=1))

    general_step = AnatPETCNNRef.general_step


class TabularMLPRef(nn.Module):
    """BUILD EXTENSION (config 5): 9 tabular features (pkg/utils/dataloader.py:306) ->
    Linear(9,64) -> ReLU -> Linear(64,64) -> ReLU."""

    def __init__(self, n_features=9, width=64):
        super().__init__()
        self.net = nn.Sequential(nn.Linear(n_features, width), nn.ReLU(),
                                 nn.Linear(width, width), nn.ReLU())

    def forward(self, x):
        return self.net(x.reshape(x.shape[0], -1))


class TriResNetTabularRef(nn.Module):
    """BUILD EXTENSION (BASELINE config 5, ``Tri_ResNet_Tabular_Fusion``): the stage-3 head
    of All_Modalities_Fusion (all_modalities_fusion.py:50-79: three 64-d features -> cat 192 ->
    Linear(192,64) -> ReLU -> Linear(64,C)) over an MRI ResNet, a PET ResNet (both cut to
    conv_seg[:2] and reduced 512 -> 64 + ReLU as reduce_dim_mri, anat_pet_fusion.py:49) and
    the tabular MLP that replaces the TabPFN branch.  Concat order pet, mri, tabular (the
    build extension's own; the reference concatenates its three stage-2 pair models'
    outputs, all_modalities_fusion.py:74-77, two of which embed TabPFN)."""

    def __init__(self, hparams, mri_stage1, pet_stage1):
        super().__init__()
        self.hparams = dict(hparams)
        self.model_mri = mri_stage1
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.model_pet = pet_stage1
        self.model_pet.model.conv_seg = self.model_pet.model.conv_seg[:2]
        self.model_tabular = TabularMLPRef(hparams.get("n_tabular_features", 9))
        self.relu = nn.ReLU()
        self.reduce_dim_mri = nn.Sequential(nn.Linear(512, 64), self.relu)
        self.reduce_dim_pet = nn.Sequential(nn.Linear(512, 64), self.relu)
        self.stage3out = nn.Linear(64 * 3, 64)
        self.cls3 = nn.Linear(64, hparams["n_classes"])
        self.model_fuse = nn.Sequential(self.stage3out, self.relu, self.cls3)
        self.criterion = make_criterion(hparams)

    def forward(self, x_pet, x_mri, x_tab):
        bs = x_mri.shape[0]
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        out_pet = self.reduce_dim_pet(self.model_pet(x_pet).view(bs, -1))
        out_tab = self.model_tabular(x_tab)
        return self.model_fuse(torch.cat((out_pet, out_mri, out_tab), dim=1))

    def inputs(self, batch, dtype=torch.float32):
        return (batch["pet1451"].unsqueeze(1).to(dtype), batch["mri"].unsqueeze(1).to(dtype),
                batch["tabular"].unsqueeze(1).to(dtype))

    def general_step(self, batch, batch_idx=0, mode="train"):
        y_hat = self(*self.inputs(batch)).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, batch["label"]), "outputs": y_hat,
                "labels": batch["label"]}


def _small_cnn_stack(hparams, n_in):
    """Conv3d 'same' (+bias) [BN3d] ReLU MaxPool3d(2) [Dropout] per conv_out entry:
    early_fusion.py:33-43, anat_pet_featuremapfusion.py:37-58."""
    mods = []
    for n_out, k in zip(hparams["conv_out"], hparams["filter_size"]):
        mods.append(nn.Conv3d(n_in, n_out, k, padding="same"))
        if hparams.get("batchnorm"):
            mods.append(nn.BatchNorm3d(n_out))
        mods += [nn.ReLU(), nn.MaxPool3d(2)]
        if "dropout_conv_p" in hparams:
            mods.append(nn.Dropout(p=hparams["dropout_conv_p"]))
        n_in = n_out
    return mods, n_in


class EarlyFusionRef(nn.Module):
    """PET_MRI_EF (pkg/models/fusion_models/early_fusion.py:19-112): stack(pet, mri) as two
    input channels (:77-80), the small-CNN stack (:33-43), GAP, Flatten, [Dropout, Linear,
    ReLU] (:49-55), Linear(n_out, C) where n_out is the loop variable when linear_out is
    falsy (:56), weighted CE (:61-62)."""

    def __init__(self, hparams):
        super().__init__()
        self.hparams = dict(hparams)
        mods, n_in = _small_cnn_stack(hparams, 2)
        n_out = n_in
        mods += [nn.AdaptiveAvgPool3d(1), nn.Flatten()]
        if hparams.get("linear_out"):
            n_out = hparams["linear_out"]
            if "dropout_dense_p" in hparams:
                mods.append(nn.Dropout(p=hparams["dropout_dense_p"]))
            mods += [nn.Linear(n_in, n_out), nn.ReLU()]
        mods.append(nn.Linear(n_out, hparams["n_classes"]))
        self.model = nn.Sequential(*mods)
        self.criterion = nn.CrossEntropyLoss(weight=hparams["loss_class_weights"])

    def forward(self, x):
        return self.model(x)

    def inputs(self, batch, dtype=torch.float32):
        return (torch.stack((batch["pet1451"], batch["mri"]), dim=1).to(dtype=dtype),)

    def general_step(self, batch, batch_idx=0, mode="train"):
        """early_fusion.py:75-91."""
        y = batch["label"]
        y_hat = self(*self.inputs(batch)).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, y), "outputs": y_hat, "labels": y}


class FeatureMapFusionRef(nn.Module):
    """PET_MRI_FMF (pkg/models/fusion_models/anat_pet_featuremapfusion.py:20-132): two
    small-CNN branches (:37-62), fused by channel concat or voxel-wise max (:112-118), then
    n_layers_fusion x (Conv 'same' [BN] ReLU MaxPool(2)) (:71-78; n_in_fusion doubles per
    layer, sic), GAP, Flatten, [Dropout], Linear(n_out_fusion, 64), ReLU, Linear(64, C)
    (:81-92); weighted CE (:94-95)."""

    def __init__(self, hparams):
        super().__init__()
        self.hparams = dict(hparams)
        self.fusion_mode = hparams["fusion_mode"]
        pet, n_in = _small_cnn_stack(hparams, 1)
        mri, _ = _small_cnn_stack(hparams, 1)
        self.backbone_pet = nn.Sequential(*pet)
        self.backbone_mri = nn.Sequential(*mri)
        n_in_fusion = 2 * n_in if self.fusion_mode == "concatenate" else n_in
        fused = []
        for _ in range(hparams["n_layers_fusion"]):
            fused.append(nn.Conv3d(n_in_fusion, hparams["n_out_fusion"],
                                   hparams["filter_size_fusion"], padding="same"))
            if hparams.get("batchnorm_fusion"):
                fused.append(nn.BatchNorm3d(hparams["n_out_fusion"]))
            fused += [nn.ReLU(), nn.MaxPool3d(2)]
            n_in_fusion = n_in_fusion * 2
        fused += [nn.AdaptiveAvgPool3d(1), nn.Flatten()]
        if "dropout_dense_p" in hparams:
            fused.append(nn.Dropout(p=hparams["dropout_dense_p"]))
        fused += [nn.Linear(hparams["n_out_fusion"], 64), nn.ReLU(),
                  nn.Linear(64, hparams["n_classes"])]
        self.fuse_model = nn.Sequential(*fused)
        self.criterion = nn.CrossEntropyLoss(weight=hparams["loss_class_weights"])

    def forward(self, x_pet, x_mri):
        out_pet = self.backbone_pet(x_pet)
        out_mri = self.backbone_mri(x_mri)
        if self.fusion_mode == "concatenate":
            out = torch.cat((out_pet, out_mri), dim=1)
        else:
            out, _ = torch.max(torch.stack((out_pet, out_mri), dim=0), dim=0)
        return self.fuse_model(out)

    def inputs(self, batch, dtype=torch.float32):
        return (batch["pet1451"].unsqueeze(1).to(dtype=dtype),
                batch["mri"].unsqueeze(1).to(dtype=dtype))

    def general_step(self, batch, batch_idx=0, mode="train"):
        """anat_pet_featuremapfusion.py:120-141."""
        y = batch["label"]
        y_hat = self(*self.inputs(batch)).to(dtype=torch.double)
        return {"loss": self.criterion(y_hat, y), "outputs": y_hat, "labels": y}


def adam_param_groups(model, hparams):
    """anat_cnn.py:111-136: head lr = lr; backbone lr = lr_pretrained or frozen."""
    groups = []
    for name, p in model.model.named_parameters():
        if "conv_seg" in name:
            groups.append({"params": p, "lr": hparams["lr"]})
        elif not hparams.get("lr_pretrained"):
            p.requires_grad = False
            groups.append({"params": p})
        else:
            p.requires_grad = True
            groups.append({"params": p, "lr": hparams["lr_pretrained"]})
    return groups
