"""Drop-in replacements for the reference's ``pkg.models`` / ``pkg.loss_functions`` classes.

Same class names, constructor signatures, hparams keys, ``general_step`` contract
(``{'loss', 'outputs', 'labels'}``), attribute paths (``.model``, ``.model.conv_seg``,
``.model_fuse``, ``.reduce_dim_mri``, ``.stage2out``, ``.cls2``) and state_dict keys as

  pkg/models/base_model.py                         Base_Model
  pkg/models/mri_models/anat_cnn.py                Anat_CNN
  pkg/models/pet_models/pet_cnn.py                 Small_PET_CNN, Random_Benchmark_All_CN
  pkg/models/pet_models/pet_resnet_cnn.py          PET_CNN_ResNet
  pkg/models/fusion_models/anat_pet_fusion.py      Anat_PET_CNN
  pkg/models/fusion_models/tabular_mri_fusion.py   Tabular_MRT_Model
  pkg/models/fusion_models/pet_tabular_fusion.py   PET_TABULAR_CNN
  pkg/models/fusion_models/all_modalities_fusion.py All_Modalities_Fusion
  pkg/loss_functions/focalloss.py                  FocalLoss

but every forward / backward op runs on the MI355X kernels of libmmad_hip.so.

Additions beyond the reference (documented build extensions, BASELINE configs 3-5):
  * hparams['precision'] in {'32' (default, the reference's fp32), 'bf16'};
  * resnet_depth 34 (n_in 512) is accepted (the reference match rejects it,
    anat_cnn.py:37-46);
  * PET_MRI_ResNet_Fusion -- "ResNet-10 x2 + MLP head" (config 3/4);
  * Tri_ResNet_Tabular_Fusion -- MRI ResNet + PET ResNet + tabular MLP trained in one
    stage (config 5's network; not a reference class).

The stage-2 / stage-3 tabular fusion classes (Tabular_MRT_Model, PET_TABULAR_CNN,
All_Modalities_Fusion) follow the reference; their TabPFN feature extractor comes from
tabular.py (tabpfn, or a registered backend).
"""
import os
from abc import ABC, abstractmethod

import torch
import torch.nn as nn
from torch.optim.lr_scheduler import ReduceLROnPlateau

from . import head_ops
from . import tabular
from . import layers as Lyr
from . import medicalnet
from .lightning_compat import (LightningModule, MulticlassF1Score, MulticlassMatthewsCorrCoef)
from .preprocess import apply_batch_spec
from .volume_ops import cast

PRETRAIN_TEMPLATE = ("/vol/chameleon/projects/adni/adni_1/MedicalNet/pretrain/"
                     "resnet_{}_23dataset.pth")      # anat_cnn.py:19


# ------------------------------------------------------------------------------ losses
class FocalLoss(nn.Module):
    """FocalLoss(gamma, alpha=None, size_average=True) -- pkg/loss_functions/focalloss.py.

    loss = mean_i( -(1 - pt_i)^gamma * log pt_i ), pt detached (focalloss.py:29).
    """

    def __init__(self, gamma=0, alpha=None, size_average=True):
        super().__init__()
        if alpha is not None:
            raise NotImplementedError("FocalLoss alpha weighting (no reference caller sets it)")
        self.gamma = gamma
        self.alpha = alpha
        self.size_average = size_average

    def forward(self, input, target):
        loss = head_ops.focal_loss(input, target, self.gamma)
        if not self.size_average:
            loss = loss * target.numel()
        return loss

    def fused_spec(self):
        """(weight, gamma, mode) for head_ops.logits_and_loss"""
        return (None, float(self.gamma), 1) if self.size_average else None


def make_criterion(hparams):
    """anat_cnn.py:81-85: focal loss iff hparams['fl_gamma'] is truthy, else weighted CE."""
    if "fl_gamma" in hparams and hparams["fl_gamma"]:
        return FocalLoss(gamma=hparams["fl_gamma"])
    return Lyr.CrossEntropyLoss(weight=hparams["loss_class_weights"])


def _to_f64(y_hat):
    return cast(y_hat, torch.float64)


def _logits_and_loss(criterion, out, y):
    """(y_hat = out as f64, criterion(y_hat, y)) -- anat_cnn.py:102-104 -- with the cast
    and our losses fused into one launch each way when the criterion allows it."""
    spec = getattr(criterion, "fused_spec", None)
    spec = spec() if spec is not None else None
    if spec is not None and out.dim() == 2 and out.dtype in (torch.float32, torch.float64) \
            and out.is_cuda:
        return head_ops.logits_and_loss(out, y, *spec)
    y_hat = _to_f64(out)
    return y_hat, criterion(y_hat, y)


# -------------------------------------------------------------------------- base model
class Base_Model(LightningModule, ABC):
    """pkg/models/base_model.py:11-239 (metrics / logging surface; hot path in general_step)."""

    def __init__(self, hparams, gpu_id=None):
        super().__init__()
        self.save_hyperparameters(hparams, ignore=["gpu_id"])
        nc = self.hparams["n_classes"]
        self.label_ind_by_names = ({"CN": 0, "MCI": 1, "AD": 2} if nc == 3
                                   else {"CN": 0, "AD": 1})
        for split in ("train", "val", "test"):
            setattr(self, f"f1_score_{split}", MulticlassF1Score(num_classes=nc, average="macro"))
            setattr(self, f"f1_score_{split}_per_class",
                    MulticlassF1Score(num_classes=nc, average="none"))

    @abstractmethod
    def forward(self, *x):
        pass

    @abstractmethod
    def general_step(self, batch, batch_idx, mode) -> dict:
        pass

    @staticmethod
    def prepare_batch(batch):
        """Opt-in device normalisation (dataset.MultiModalDataset(device_normalize=True)):
        a batch carrying the loader's normalisation settings gets them applied here, on the
        device, before any model math; every other batch passes through unchanged (the
        default dataset already normalised it on fetch, as the reference loader does)."""
        return apply_batch_spec(batch)

    def on_after_batch_transfer(self, batch, dataloader_idx=0):
        """Lightning hook (runs after the batch reaches the device)."""
        return self.prepare_batch(batch)

    @property
    def is_cuda(self):
        return next(self.parameters()).is_cuda

    def save(self, path):
        print("Saving model... %s" % path)
        torch.save(self, path)

    def _step(self, batch, batch_idx, split):
        out = self.general_step(batch, batch_idx, split)
        getattr(self, f"f1_score_{split}")(out["outputs"], out["labels"])
        getattr(self, f"f1_score_{split}_per_class")(out["outputs"], out["labels"])
        return out

    def training_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, "train")

    def validation_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, "val")

    def test_step(self, batch, batch_idx):
        return self._step(batch, batch_idx, "test")

    def predict_step(self, batch, batch_idx):
        return self.general_step(batch, batch_idx, "pred")

    @abstractmethod
    def configure_optimizers(self):
        pass

    def _epoch_end(self, outputs, split):
        avg = torch.stack([o["loss"].detach() for o in outputs]).mean()
        f1 = getattr(self, f"f1_score_{split}")
        f1c = getattr(self, f"f1_score_{split}_per_class")
        f1_epoch, f1_per_class = f1.compute(), f1c.compute()
        f1.reset()
        f1c.reset()
        d = {f"{split}_loss_epoch": avg, f"{split}_f1_epoch": f1_epoch,
             "step": float(self.current_epoch)}
        for i in range(self.hparams["n_classes"]):
            d[f"{split}_f1_epoch_class_{i}"] = f1_per_class[i]
        return d

    def training_epoch_end(self, outputs):
        self.log_dict(self._epoch_end(outputs, "train"))

    def validation_epoch_end(self, outputs):
        self.log_dict(self._epoch_end(outputs, "val"))

    def test_epoch_end(self, outputs):
        d = self._epoch_end(outputs, "test")
        y_hat = torch.cat([o["outputs"].detach() for o in outputs])
        y = torch.cat([o["labels"] for o in outputs])
        nc = self.hparams["n_classes"]
        d["test_f1_epoch_boot"], d["test_f1_epoch_ci"] = self.bootstrap_metric(
            MulticlassF1Score(num_classes=nc, average="macro"), y_hat, y)
        d["test_mcc_epoch_boot"], d["test_mcc_epoch_ci"] = self.bootstrap_metric(
            MulticlassMatthewsCorrCoef(num_classes=nc), y_hat, y)
        self.log_dict(d)

    def bootstrap_metric(self, metric, y_hat, y_labels, n_drawings=1000):
        """base_model.py:219-239: mean and 1.96*std over n_drawings resamples.

        Macro F1 / MCC metrics on device tensors run all drawings in one launch
        (mmad_bootstrap_cls_metrics, one block per drawing).  The drawings' indices come
        from the same global torch RNG calls as the reference loop (one (n_drawings, n)
        randint = n_drawings successive (n,) draws, element for element), so the sampled
        sets are identical.  Other metric objects keep the reference's loop."""
        kind = _bootstrap_kind(metric)
        if kind is not None and y_hat.is_cuda and y_hat.dim() == 2:
            n = len(y_hat)
            idx = torch.randint(0, n, (n_drawings, n))
            f1, mcc = head_ops.bootstrap_cls_metrics(y_hat, y_labels, idx)
            ms = head_ops.mean_std(f1 if kind == "f1" else mcc).cpu()
            return ms[0].float(), (1.96 * ms[1]).float()
        metric.to(self.device)
        vals = torch.zeros(n_drawings)
        n = len(y_hat)
        for i in range(n_drawings):
            idx = torch.randint(0, n, (n,))
            metric(y_hat[idx.to(y_hat.device)], y_labels[idx.to(y_labels.device)])
            vals[i] = metric.compute()
            metric.reset()
        return torch.mean(vals), 1.96 * torch.std(vals)


def _bootstrap_kind(metric):
    """'f1' for a macro MulticlassF1Score, 'mcc' for MulticlassMatthewsCorrCoef, else None
    (torchmetrics classes or the lightning_compat stand-ins)."""
    name = type(metric).__name__
    if name == "MulticlassF1Score" and getattr(metric, "average", "macro") == "macro":
        return "f1"
    if name == "MulticlassMatthewsCorrCoef":
        return "mcc"
    return None


# ---------------------------------------------------------------------------- heads
def resnet_features(depth):
    """anat_cnn.py:37-46 depth -> backbone width (34 is a build extension)."""
    if depth not in medicalnet.FEATURES:
        raise ValueError("hparams['resnet_depth'] is not in [10, 18, 34, 50]")
    return medicalnet.FEATURES[depth]


def build_conv_seg(hparams, n_in):
    """Replacement conv_seg head (anat_cnn.py:33-79; pet_resnet_cnn.py:37-81)."""
    mods = []
    if hparams.get("batchnorm_begin"):
        mods.append(Lyr.BatchNorm3d(n_in))
    if "conv_out" in hparams:
        for n_out, k in zip(hparams["conv_out"], hparams["filter_size"]):
            mods.append(Lyr.Conv3d(n_in, n_out, k, padding="same"))
            if hparams["batchnorm_conv"]:
                mods.append(Lyr.BatchNorm3d(n_out))
            mods += [Lyr.ReLU(), Lyr.MaxPool3d(2)]
            n_in = n_out
    mods += [Lyr.AdaptiveAvgPool3d(1), nn.Flatten()]
    for n_out in hparams["linear_out"]:
        mods.append(Lyr.Linear(n_in, n_out))
        if hparams.get("batchnorm_dense"):
            mods.append(Lyr.BatchNorm1d(n_out))
        mods.append(Lyr.ReLU())
        n_in = n_out
    mods += [Lyr.Linear(n_in, hparams["n_classes"]), Lyr.ReLU()]
    return Lyr.Sequential(*mods)


def _resnet_backbone(hparams):
    opts = medicalnet.parse_opts()
    depth = hparams["resnet_depth"]
    opts.model_depth = depth
    opts.pretrain_path = hparams.get("pretrain_path") or PRETRAIN_TEMPLATE.format(depth)
    wrapped, _ = medicalnet.generate_model(opts)
    return wrapped.module


def _adam_groups_backbone(model, hparams):
    """anat_cnn.py:111-136: head lr; backbone lr_pretrained or frozen (requires_grad off)."""
    groups = []
    for name, p in model.named_parameters():
        if "conv_seg" in name:
            groups.append({"params": p, "lr": hparams["lr"]})
        elif not hparams.get("lr_pretrained"):
            p.requires_grad = False
            groups.append({"params": p})
        else:
            p.requires_grad = True
            groups.append({"params": p, "lr": hparams["lr_pretrained"]})
    return groups


def _merge_groups(groups):
    """The reference builds one Adam param group per tensor (anat_cnn.py:112-126); groups
    that share a learning rate are merged (Adam is element-wise, so the update is
    identical) so the fused optimizer runs one multi-tensor launch per learning rate
    instead of one per tensor."""
    merged = {}
    for grp in groups:
        params = grp["params"]
        params = list(params) if not isinstance(params, torch.Tensor) else [params]
        key = grp.get("lr", None)
        merged.setdefault(key, []).extend(params)
    out = []
    for lr, params in merged.items():
        out.append({"params": params} if lr is None else {"params": params, "lr": lr})
    return out


class MergedAdam(torch.optim.Adam):
    """torch.optim.Adam built from the reference's param-group list (one group per tensor,
    anat_cnn.py:112-126, anat_pet_fusion.py:94-114) that RUNS on the merged groups
    (``_merge_groups``: one fused multi-tensor launch per learning rate) but SPEAKS the
    reference's layout in ``state_dict()`` / ``load_state_dict()``: a checkpoint's
    ``optimizer_states`` written by the reference resumes here and ours resumes in the
    reference (Lightning calls exactly these two methods for ``ckpt_path=`` resumes).

    ``load_state_dict`` accepts either layout: the reference's per-tensor groups (mapped into
    the merged groups; tensors of one merged group share every hyperparameter, the lr
    included, because they were merged on it and a scheduler scales them alike) or the
    merged layout torch's own ``Adam.state_dict`` of this object would have produced."""

    def __init__(self, groups, **kw):
        self._ref_groups = []
        for grp in groups:
            ps = grp["params"]
            ps = [ps] if isinstance(ps, torch.Tensor) else list(ps)
            self._ref_groups.append(ps)
        super().__init__(_merge_groups(groups), **kw)

    def _merged_index(self):
        order = [p for g in self.param_groups for p in g["params"]]
        gidx = [gi for gi, g in enumerate(self.param_groups) for _ in g["params"]]
        return {id(p): i for i, p in enumerate(order)}, gidx

    def state_dict(self):
        sd = super().state_dict()
        for g in sd["param_groups"]:
            # a captured step's 0-d device lr (graph_step) is saved as the plain float the
            # reference's torch 1.13 Adam keeps (it feeds lr straight into addcdiv_'s value)
            if torch.is_tensor(g.get("lr")):
                g["lr"] = float(g["lr"])
        if len(self._ref_groups) == len(self.param_groups):
            return sd                      # nothing was merged: the layouts coincide
        idx, gidx = self._merged_index()
        state, groups, j = {}, [], 0
        for ps in self._ref_groups:
            ids = []
            for p in ps:
                i = idx[id(p)]
                if i in sd["state"]:
                    state[j] = sd["state"][i]
                ids.append(j)
                j += 1
            g = {k: v for k, v in sd["param_groups"][gidx[idx[id(ps[0])]]].items()
                 if k != "params"}
            g["params"] = ids
            groups.append(g)
        return {"state": state, "param_groups": groups}

    def ref_group_index(self):
        """merged group of each reference (per-tensor) group, in reference order"""
        idx, gidx = self._merged_index()
        return [gidx[idx[id(ps[0])]] for ps in self._ref_groups]

    # optimizer-implementation keys: how THIS optimizer runs, not training state.  A
    # checkpoint from the reference (torch 1.13 Adam: fused None, capturable False) must not
    # turn off the fused multi-tensor Adam here, nor a captured step's device-resident lr.
    _IMPL_KEYS = ("fused", "foreach", "capturable", "differentiable")

    def load_state_dict(self, state_dict):
        saved = state_dict["param_groups"]
        per_tensor = (len(self._ref_groups) != len(self.param_groups) and
                      len(saved) == len(self._ref_groups) and
                      all(len(g["params"]) == len(ps) for g, ps in zip(saved, self._ref_groups)))
        if per_tensor:
            idx, gidx = self._merged_index()
            state, first = {}, {}
            for g, ps in zip(saved, self._ref_groups):
                for j, p in zip(g["params"], ps):
                    i = idx[id(p)]
                    first.setdefault(gidx[i], g)
                    if j in state_dict["state"]:
                        state[i] = state_dict["state"][j]
            groups, base = [], 0
            for gi, g in enumerate(self.param_groups):
                src = {k: v for k, v in first[gi].items() if k != "params"}
                src["params"] = list(range(base, base + len(g["params"])))
                base += len(g["params"])
                groups.append(src)
            state_dict = {"state": state, "param_groups": groups}
        groups = [dict(g) for g in state_dict["param_groups"]]
        if len(groups) == len(self.param_groups):
            for g, cur in zip(groups, self.param_groups):
                for k in self._IMPL_KEYS:
                    if k in cur:
                        g[k] = cur[k]    # also moves Adam's step counters where fused needs them
        lrs = [cur["lr"] for cur in self.param_groups]
        super().load_state_dict({"state": state_dict["state"], "param_groups": groups})
        for cur, old in zip(self.param_groups, lrs):
            if torch.is_tensor(old):     # a captured step reads this tensor: keep it, refill it
                new = cur["lr"]
                old.fill_(new.item() if torch.is_tensor(new) else float(new))
                cur["lr"] = old


class MergedPlateau(ReduceLROnPlateau):
    """ReduceLROnPlateau over a MergedAdam whose ``state_dict`` lists ``min_lrs`` and
    ``_last_lr`` per reference (per-tensor) group, as torch 1.13's scheduler on the
    reference's optimizer does (anat_cnn.py:129-134): a checkpoint resumes in either
    direction.  ``load_state_dict`` takes either length."""

    def _ref_index(self):
        opt = self.optimizer
        return opt.ref_group_index() if isinstance(opt, MergedAdam) else None

    def state_dict(self):
        sd = super().state_dict()
        ri = self._ref_index()
        if ri is not None and len(ri) != len(self.optimizer.param_groups):
            for k in ("min_lrs", "_last_lr"):
                if isinstance(sd.get(k), (list, tuple)) and \
                        len(sd[k]) == len(self.optimizer.param_groups):
                    sd[k] = [sd[k][m] for m in ri]
        return sd

    def load_state_dict(self, state_dict):
        sd = dict(state_dict)
        ri = self._ref_index()
        n = len(self.optimizer.param_groups)
        if ri is not None and len(ri) != n:
            for k in ("min_lrs", "_last_lr"):
                v = sd.get(k)
                if isinstance(v, (list, tuple)) and len(v) == len(ri):
                    merged = [None] * n
                    for r, m in enumerate(ri):
                        if merged[m] is None:
                            merged[m] = v[r]
                    sd[k] = merged
        super().load_state_dict(sd)


def _adam(groups, hparams, device):
    fused = device.type == "cuda"
    return MergedAdam(groups, weight_decay=hparams.get("l2_reg", 0) or 0, fused=fused)


def _with_scheduler(opt, hparams):
    if hparams.get("reduce_factor_lr_schedule"):
        return {"optimizer": opt,
                "lr_scheduler": MergedPlateau(opt, factor=hparams["reduce_factor_lr_schedule"]),
                "monitor": "val_loss_epoch"}
    return opt


# ------------------------------------------------------------------------- MRI model
class Anat_CNN(Base_Model):
    """MRI classifier: MedicalNet 3D-ResNet + conv_seg head (anat_cnn.py:13-136)."""

    batch_key = "mri"

    def __init__(self, hparams, gpu_id=None):
        super().__init__(hparams)
        self.model = _resnet_backbone(hparams)
        self.model.conv_seg = build_conv_seg(hparams, resnet_features(hparams["resnet_depth"]))
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x):
        return self.model(x)

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x = batch[self.batch_key].unsqueeze(1)   # raw f64 volume; conv 1 unfolds + casts it
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self.forward(x), y)
        if mode != "pred":
            self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        opt = _adam(_adam_groups_backbone(self.model, self.hparams), self.hparams, self.device)
        return _with_scheduler(opt, self.hparams)


class PET_CNN_ResNet(Anat_CNN):
    """PET classifier on the same backbone (pet_resnet_cnn.py:12-198).

    The reference subclasses LightningModule directly with its own step / epoch-end code;
    the observable differences kept here: PET batch key, train / val macro-F1 updated inside
    general_step, no scheduler in configure_optimizers.
    """

    batch_key = "pet1451"

    def general_step(self, batch, batch_idx, mode):
        out = super().general_step(batch, batch_idx, mode)
        if mode in ("train", "val"):
            getattr(self, f"f1_score_{mode}")(out["outputs"], out["labels"])
        return out

    def training_step(self, batch, batch_idx):
        return self.general_step(batch, batch_idx, "train")

    def validation_step(self, batch, batch_idx):
        return self.general_step(batch, batch_idx, "val")

    def configure_optimizers(self):
        return _adam(_adam_groups_backbone(self.model, self.hparams), self.hparams, self.device)


# ------------------------------------------------------------------------- PET model
class Small_PET_CNN(Base_Model):
    """pet_cnn.py:10-82: n x (Conv 'same' (+bias) [BN] ReLU MaxPool(2) [Dropout]) -> GAP ->
    [Dropout, Linear, ReLU] -> Linear; always weighted CE (pet_cnn.py:47-48)."""

    batch_key = "pet1451"

    def __init__(self, hparams, gpu_id=None):
        super().__init__(hparams, gpu_id=gpu_id)
        mods = []
        n_in, n_out = 1, None
        for n_out, k in zip(self.hparams["conv_out"], self.hparams["filter_size"]):
            mods.append(Lyr.Conv3d(n_in, n_out, k, padding="same"))
            if self.hparams.get("batchnorm"):
                mods.append(Lyr.BatchNorm3d(n_out))
            mods += [Lyr.ReLU(), Lyr.MaxPool3d(2)]
            if "dropout_conv_p" in self.hparams:
                mods.append(Lyr.Dropout(p=self.hparams["dropout_conv_p"]))
            n_in = n_out
        mods += [Lyr.AdaptiveAvgPool3d(1), nn.Flatten()]
        if self.hparams.get("linear_out"):
            n_out = self.hparams["linear_out"]
            if "dropout_dense_p" in self.hparams:
                mods.append(Lyr.Dropout(p=self.hparams["dropout_dense_p"]))
            mods += [Lyr.Linear(n_in, n_out), Lyr.ReLU()]
        mods.append(Lyr.Linear(n_out, self.hparams["n_classes"]))
        self.model = nn.Sequential(*mods)
        self.criterion = Lyr.CrossEntropyLoss(weight=hparams["loss_class_weights"])
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x):
        return self.model(x)

    general_step = Anat_CNN.general_step

    def configure_optimizers(self):
        opt = torch.optim.Adam(self.model.parameters(), lr=self.hparams["lr"],
                               fused=self.device.type == "cuda")
        return _with_scheduler(opt, self.hparams)


class Random_Benchmark_All_CN(Small_PET_CNN):
    """pet_cnn.py:85-90: constant 'all CN' prediction baseline."""

    def forward(self, x):
        y = super().forward(x)
        one_hot = torch.zeros_like(y)
        one_hot[..., 0] = 1
        return one_hot


# ---------------------------------------------------------------------- fusion models
def _freeze(*mods):
    for m in mods:
        for p in m.parameters():
            p.requires_grad = False


class Anat_PET_CNN(Base_Model):
    """PET-MRI late fusion (anat_pet_fusion.py:11-127).

    Stage-1 models come from checkpoints (``path_pet``/``path_anat`` or the hparams
    ``path_pet``/``path_mri``), or -- an addition for tests / benchmarks -- as live modules
    via ``pet_model=`` / ``mri_model=``.  ``path_mri=`` is accepted as an alias of
    ``path_anat`` (pkg/inference/test_anat_pet_fusion.py passes it).
    """

    def __init__(self, hparams, path_pet=None, path_anat=None, path_mri=None, pet_model=None,
                 mri_model=None):
        super().__init__(hparams)
        path_anat = path_anat or path_mri
        if pet_model is None or mri_model is None:
            if path_pet and path_anat:
                pet_model = Small_PET_CNN.load_from_checkpoint(path_pet)
                mri_model = Anat_CNN.load_from_checkpoint(path_anat)
            else:
                pet_model = Small_PET_CNN.load_from_checkpoint(hparams["path_pet"])
                mri_model = Anat_CNN.load_from_checkpoint(hparams["path_mri"])
        cut = -3 if hparams["n_classes"] == 2 else -1
        self.model_pet = pet_model.model[:cut]
        self.model_mri = mri_model
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        if not hparams.get("lr_pretrained"):
            _freeze(self.model_pet, self.model_mri)
        self.stage2out = Lyr.Linear(64 + 64, 64)
        self.cls2 = Lyr.Linear(64, hparams["n_classes"])
        self.relu = Lyr.ReLU()
        self.reduce_dim_mri = nn.Sequential(Lyr.Linear(512, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_mri):
        bs = x_mri.shape[0]
        out_pet = self.model_pet(x_pet)
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        return self.model_fuse(head_ops.concat_features(out_pet, out_mri))

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_pet = batch["pet1451"].unsqueeze(1)
        x_mri = batch["mri"].unsqueeze(1)
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self(x_pet, x_mri), y)
        self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def _fusion_groups(self):
        groups = [{"params": p, "lr": self.hparams["lr"]}
                  for m in (self.model_fuse, self.reduce_dim_mri) for p in m.parameters()]
        if self.hparams.get("lr_pretrained"):
            groups += [{"params": p, "lr": self.hparams["lr_pretrained"]}
                       for m in self._stage1() for p in m.parameters()]
        return groups

    def _stage1(self):
        return (self.model_pet, self.model_mri)

    def configure_optimizers(self):
        return _with_scheduler(_adam(self._fusion_groups(), self.hparams, self.device),
                               self.hparams)


def _small_cnn_stack(hparams, n_in):
    """n x (Conv3d 'same' (+bias) [BN3d] ReLU MaxPool3d(2) [Dropout]) as built by
    early_fusion.py:33-43 and anat_pet_featuremapfusion.py:37-58 (same as pet_cnn.py:18-30).
    Returns (modules, n_in after the stack, n_out of the last conv or None)."""
    mods, n_out = [], None
    for n_out, k in zip(hparams["conv_out"], hparams["filter_size"]):
        mods.append(Lyr.Conv3d(n_in, n_out, k, padding="same"))
        if hparams.get("batchnorm"):
            mods.append(Lyr.BatchNorm3d(n_out))
        mods += [Lyr.ReLU(), Lyr.MaxPool3d(2)]
        if "dropout_conv_p" in hparams:
            mods.append(Lyr.Dropout(p=hparams["dropout_conv_p"]))
        n_in = n_out
    return mods, n_in, n_out


class PET_MRI_EF(Base_Model):
    """PET-MRI early fusion (pkg/models/fusion_models/early_fusion.py:19-112): the PET and
    MRI volumes stacked as 2 input channels of one small CNN.

    general_step hands the first conv the two raw f64 volumes as a StackedVolumes (the
    reference's torch.stack + .to(float32), :77-80, is done inside the conv's gather pass:
    mmad_gather_channels).  Head (:45-56): GAP, Flatten, [Dropout, Linear(n_in, linear_out),
    ReLU], Linear(., C) -- with no ``linear_out`` the reference's last Linear takes the loop
    variable ``n_out`` (the last conv width), reproduced here.  Always weighted CE (:61-62),
    one Adam group over ``self.model`` without weight decay (:99-106)."""

    def __init__(self, hparams, gpu_id=None):
        super().__init__(hparams, gpu_id=gpu_id)
        mods, n_in, n_out = _small_cnn_stack(self.hparams, 2)
        mods += [Lyr.AdaptiveAvgPool3d(1), nn.Flatten()]
        if self.hparams.get("linear_out"):
            n_out = self.hparams["linear_out"]
            if "dropout_dense_p" in self.hparams:
                mods.append(Lyr.Dropout(p=self.hparams["dropout_dense_p"]))
            mods += [Lyr.Linear(n_in, n_out), Lyr.ReLU()]
        mods.append(Lyr.Linear(n_out, self.hparams["n_classes"]))
        self.model = nn.Sequential(*mods)
        self.criterion = Lyr.CrossEntropyLoss(weight=hparams["loss_class_weights"])
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x):
        return self.model(x)

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        from .volume_ops import StackedVolumes
        x = StackedVolumes([batch["pet1451"], batch["mri"]])
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self.forward(x), y)
        if mode != "pred":
            self.log(mode + "_loss", loss, on_step=True)
        if mode in ("train", "val"):
            getattr(self, f"f1_score_{mode}")(y_hat, y)
            getattr(self, f"f1_score_{mode}_per_class")(y_hat, y)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        opt = torch.optim.Adam(self.model.parameters(), lr=self.hparams["lr"],
                               fused=self.device.type == "cuda")
        return _with_scheduler(opt, self.hparams)


class Random_Benchmark_All_CN_EF(PET_MRI_EF):
    """early_fusion.py:113-118 (``Random_Benchmark_All_CN`` there): constant 'all CN'."""

    def forward(self, x):
        y = super().forward(x)
        one_hot = torch.zeros_like(y)
        one_hot[..., 0] = 1
        return one_hot


class PET_MRI_FMF(Base_Model):
    """PET-MRI feature-map fusion (pkg/models/fusion_models/anat_pet_featuremapfusion.py:20-
    172): two identical small-CNN branches (``backbone_pet``, ``backbone_mri``), their
    feature maps fused voxel-wise -- channel concat ('concatenate', mmad_concat_channels)
    or voxel-wise max ('maxout', mmad_max2_fwd) -- then ``fuse_model``: n_layers_fusion x
    (Conv3d 'same' [BN3d] ReLU MaxPool3d(2)), GAP, Flatten, [Dropout], Linear(n_out_fusion,
    64), ReLU, Linear(64, C).  The reference doubles ``n_in_fusion`` after every fusion
    layer (:78) instead of using n_out_fusion, so only configurations it can run (one
    fusion layer, as in its search space :69) build here too.  Weighted CE (:94-95); Adam
    with weight decay l2_reg over all three parts at lr (:135-152)."""

    def __init__(self, hparams, gpu_id=None):
        super().__init__(hparams, gpu_id=gpu_id)
        mode = hparams["fusion_mode"]
        assert mode in ("concatenate", "maxout")
        self.fusion_mode = mode
        pet, n_in, _ = _small_cnn_stack(self.hparams, 1)
        mri, _, _ = _small_cnn_stack(self.hparams, 1)
        self.backbone_pet = nn.Sequential(*pet)
        self.backbone_mri = nn.Sequential(*mri)
        n_in_fusion = 2 * n_in if mode == "concatenate" else n_in
        fused = []
        for _ in range(hparams["n_layers_fusion"]):
            fused.append(Lyr.Conv3d(n_in_fusion, hparams["n_out_fusion"],
                                    hparams["filter_size_fusion"], padding="same"))
            if self.hparams.get("batchnorm_fusion"):
                fused.append(Lyr.BatchNorm3d(hparams["n_out_fusion"]))
            fused += [Lyr.ReLU(), Lyr.MaxPool3d(2)]
            n_in_fusion = n_in_fusion * 2
        fused += [Lyr.AdaptiveAvgPool3d(1), nn.Flatten()]
        if "dropout_dense_p" in self.hparams:
            fused.append(Lyr.Dropout(p=self.hparams["dropout_dense_p"]))
        fused += [Lyr.Linear(hparams["n_out_fusion"], 64), Lyr.ReLU(),
                  Lyr.Linear(64, self.hparams["n_classes"])]
        self.fuse_model = nn.Sequential(*fused)
        self.criterion = Lyr.CrossEntropyLoss(weight=hparams["loss_class_weights"])
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_mri):
        from .volume_ops import cat_channels, maxout
        out_pet = self.backbone_pet(x_pet)
        out_mri = self.backbone_mri(x_mri)
        if self.fusion_mode == "concatenate":
            fused = cat_channels(out_pet, out_mri)
        else:
            fused = maxout(out_pet, out_mri)
        return self.fuse_model(fused)

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_pet = batch["pet1451"].unsqueeze(1)      # raw f64; conv 1 unfolds + casts (:124-127)
        x_mri = batch["mri"].unsqueeze(1)
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self.forward(x_pet=x_pet, x_mri=x_mri), y)
        if mode != "pred":
            self.log(mode + "_loss", loss, on_step=True)
        if mode in ("train", "val"):
            getattr(self, f"f1_score_{mode}")(y_hat, y)
            getattr(self, f"f1_score_{mode}_per_class")(y_hat, y)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        params = [p for m in (self.backbone_mri, self.backbone_pet, self.fuse_model)
                  for p in m.parameters()]
        opt = torch.optim.Adam([{"params": params, "lr": self.hparams["lr"]}],
                               weight_decay=self.hparams.get("l2_reg", 0) or 0,
                               fused=self.device.type == "cuda")
        return _with_scheduler(opt, self.hparams)


class Random_Benchmark_All_CN_FMF(PET_MRI_FMF):
    """anat_pet_featuremapfusion.py:173-178 (``Random_Benchmark_All_CN`` there)."""

    def forward(self, x_pet, x_mri):
        y = super().forward(x_pet, x_mri)
        one_hot = torch.zeros_like(y)
        one_hot[..., 0] = 1
        return one_hot


def _stage1_resnet(cls, hparams, depth, precision):
    h = dict(hparams)
    h.update({"resnet_depth": depth, "linear_out": [], "conv_out": [], "filter_size": [],
              "batchnorm_begin": False, "batchnorm_dense": False, "precision": precision})
    return cls(h)


class PET_MRI_ResNet_Fusion(Anat_PET_CNN):
    """BUILD EXTENSION -- BASELINE config 3/4 "ResNet-10 x2 + MLP head" (SURVEY.md sec. 7).

    PET branch = PET_CNN_ResNet, MRI branch = Anat_CNN, both cut to conv_seg[:2] (512-d),
    each reduced by Linear(512,64)+ReLU (``reduce_dim_pet`` mirrors ``reduce_dim_mri``,
    anat_pet_fusion.py:49); head unchanged (anat_pet_fusion.py:42-51).  Stage-1 models from
    ``path_pet``/``path_anat`` checkpoints, live modules, or fresh from hparams
    (``resnet_depth_pet`` / ``resnet_depth_mri``, default 10).
    """

    def __init__(self, hparams, path_pet=None, path_anat=None, pet_model=None, mri_model=None):
        Base_Model.__init__(self, hparams)
        prec = hparams.get("precision", "32")
        if pet_model is None:
            pet_model = (PET_CNN_ResNet.load_from_checkpoint(path_pet) if path_pet else
                         _stage1_resnet(PET_CNN_ResNet, hparams,
                                        hparams.get("resnet_depth_pet", 10), prec))
        if mri_model is None:
            mri_model = (Anat_CNN.load_from_checkpoint(path_anat) if path_anat else
                         _stage1_resnet(Anat_CNN, hparams, hparams.get("resnet_depth_mri", 10),
                                        prec))
        self.model_pet = pet_model
        self.model_pet.model.conv_seg = self.model_pet.model.conv_seg[:2]
        self.model_mri = mri_model
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        if not hparams.get("lr_pretrained"):
            _freeze(self.model_pet, self.model_mri)
        self.stage2out = Lyr.Linear(64 + 64, 64)
        self.cls2 = Lyr.Linear(64, hparams["n_classes"])
        self.relu = Lyr.ReLU()
        self.reduce_dim_pet = nn.Sequential(Lyr.Linear(512, 64), self.relu)
        self.reduce_dim_mri = nn.Sequential(Lyr.Linear(512, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_mri):
        bs = x_mri.shape[0]
        out_pet = self.reduce_dim_pet(self.model_pet(x_pet).view(bs, -1))
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        return self.model_fuse(head_ops.concat_features(out_pet, out_mri))

    def _fusion_groups(self):
        groups = super()._fusion_groups()
        groups += [{"params": p, "lr": self.hparams["lr"]} for p in self.reduce_dim_pet.parameters()]
        return groups


class Tabular_MLP(nn.Module):
    """BUILD EXTENSION (config 5): 9 tabular features (dataloader.py:306) -> 64 -> 64."""

    def __init__(self, n_features=9, width=64):
        super().__init__()
        self.net = nn.Sequential(Lyr.Linear(n_features, width), Lyr.ReLU(),
                                 Lyr.Linear(width, width), Lyr.ReLU())

    def forward(self, x):
        return self.net(x.reshape(x.shape[0], -1))


class Tri_ResNet_Tabular_Fusion(Base_Model):
    """BUILD EXTENSION -- BASELINE config 5 "MRI ResNet-34 + PET ResNet-18 + tabular MLP,
    160^3" (SURVEY.md sec. 7), trained end to end in one stage.

    Not the reference's ``All_Modalities_Fusion`` (that class fuses three *trained stage-2
    models* loaded from checkpoints, two of them TabPFN-based; it is restated below under
    its own name).  Branches: MRI ResNet (``resnet_depth_mri``, default 34), PET ResNet
    (``resnet_depth_pet``, default 18), both cut to conv_seg[:2] and reduced 512 -> 64 + ReLU
    (as reduce_dim_mri, anat_pet_fusion.py:49), Tabular_MLP -> 64 -> cat (pet, mri, tab) 192
    -> Linear(192, 64) -> ReLU -> Linear(64, C) (the reference's stage-3 head,
    all_modalities_fusion.py:50-57).
    """

    def __init__(self, hparams):
        super().__init__(hparams)
        prec = hparams.get("precision", "32")
        self.model_mri = _stage1_resnet(Anat_CNN, hparams, hparams.get("resnet_depth_mri", 34),
                                        prec)
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.model_pet = _stage1_resnet(PET_CNN_ResNet, hparams,
                                        hparams.get("resnet_depth_pet", 18), prec)
        self.model_pet.model.conv_seg = self.model_pet.model.conv_seg[:2]
        self.model_tabular = Tabular_MLP(hparams.get("n_tabular_features", 9))
        self.relu = Lyr.ReLU()
        self.reduce_dim_mri = nn.Sequential(Lyr.Linear(512, 64), self.relu)
        self.reduce_dim_pet = nn.Sequential(Lyr.Linear(512, 64), self.relu)
        self.stage3out = Lyr.Linear(64 * 3, 64)
        self.cls3 = Lyr.Linear(64, hparams["n_classes"])
        self.model_fuse = nn.Sequential(self.stage3out, self.relu, self.cls3)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_mri, x_tab):
        bs = x_mri.shape[0]
        out_mri = self.reduce_dim_mri(self.model_mri(x_mri).view(bs, -1))
        out_pet = self.reduce_dim_pet(self.model_pet(x_pet).view(bs, -1))
        out_tab = self.model_tabular(x_tab)
        return self.model_fuse(head_ops.concat_features(out_pet, out_mri, out_tab))

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_pet = batch["pet1451"].unsqueeze(1)
        x_mri = batch["mri"].unsqueeze(1)
        x_tab = cast(batch["tabular"].unsqueeze(1), torch.float32)
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self(x_pet, x_mri, x_tab), y)
        self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        groups = [{"params": p, "lr": self.hparams["lr"]} for p in self.model_fuse.parameters()]
        rest = (self.model_mri, self.model_pet, self.model_tabular, self.reduce_dim_mri,
                self.reduce_dim_pet)
        lr_pre = self.hparams.get("lr_pretrained")
        for m in rest:
            for p in m.parameters():
                p.requires_grad = bool(lr_pre) or m in (self.model_tabular,)
                groups.append({"params": p, "lr": lr_pre or self.hparams["lr"]})
        return _with_scheduler(_adam(groups, self.hparams, self.device), self.hparams)


# ------------------------------------------------------- stage-2 / stage-3 tabular fusion
def _tabpfn_params(classifier):
    """Parameters of TabPFN's transformer (``model_tabular.model[2]``), which the reference
    hands to Adam at lr_pretrained (tabular_mri_fusion.py:113-116); none for a stand-in
    that is not an nn.Module."""
    net = classifier.model[2] if getattr(classifier, "model", None) is not None else None
    return list(net.parameters()) if isinstance(net, nn.Module) else []


class _TabularStage2(Base_Model):
    """Shared forward / step of the two TabPFN stage-2 models (tabular_mri_fusion.py:50-93,
    pet_tabular_fusion.py:69-116): TabPFN decoder features of the CPU copy of the batch
    (``tabular.decoder_features``), ``reduce_tab``, the volume branch, cat, ``model_fuse``."""

    def _tab_features(self, x_tabular):
        acts = tabular.decoder_features(self.model_tabular, x_tabular,
                                        self.hparams["ensemble_size"],
                                        self.tabular_training_size)
        dev = next(self.reduce_tab.parameters()).device
        return acts.to(device=dev, dtype=torch.float32)

    def _tab_groups(self, stage1):
        groups = [{"params": p, "lr": self.hparams["lr"]}
                  for m in (self.model_fuse, self.reduce_tab) for p in m.parameters()]
        if self.hparams.get("lr_pretrained"):
            groups += [{"params": p, "lr": self.hparams["lr_pretrained"]}
                       for p in list(stage1.parameters()) + _tabpfn_params(self.model_tabular)]
        return groups


class Tabular_MRT_Model(_TabularStage2):
    """Stage-2 MRI + tabular fusion (pkg/models/fusion_models/tabular_mri_fusion.py:11-129):
    Anat_CNN from ``path_mri`` (or hparams['path_mri']) cut to conv_seg[:2] (512-d), TabPFN
    decoder features [B, 1024] -> reduce_tab = Linear(1024, 512) + ReLU, cat (tabular, mri)
    1024 -> model_fuse = Linear(1024, 64) -> ReLU -> Linear(64, C).  TabPFN comes from
    ``tabular.load_model`` (fails loudly when neither tabpfn nor a registered backend is
    present).  The MRI output is flattened per sample (the reference's ``.squeeze()``,
    :77, which equals it for batches > 1)."""

    def __init__(self, hparams, path_mri=None):
        super().__init__(hparams)
        self.model_mri = Anat_CNN.load_from_checkpoint(path_mri or hparams["path_mri"])
        self.model_mri.model.conv_seg = self.model_mri.model.conv_seg[:2]
        self.model_tabular, self.tabular_training_size = tabular.load_model(
            tabular.TRAINPATH, hparams["n_classes"] == 2, ensemble_size=hparams["ensemble_size"])
        if not hparams.get("lr_pretrained"):
            _freeze(self.model_mri)         # (TabPFN's own freeze is a no-op typo, :29-30)
        self.stage2out = Lyr.Linear(512 + 512, 64)
        self.cls2 = Lyr.Linear(64, hparams["n_classes"])
        self.relu = Lyr.ReLU()
        self.reduce_tab = nn.Sequential(Lyr.Linear(1024, 512), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_tabular, x_mri):
        bs = x_mri.shape[0]
        out_tabular = self.reduce_tab(self._tab_features(x_tabular))
        out_mri = self.model_mri(x_mri).reshape(bs, -1)
        return self.model_fuse(head_ops.concat_features(out_tabular, out_mri))

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_mri = batch["mri"].unsqueeze(1)
        y = batch["label"]
        x_tab = cast(batch["tabular"].unsqueeze(1), torch.float32)
        y_hat, loss = _logits_and_loss(self.criterion, self(x_tab, x_mri), y)
        self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        return _with_scheduler(_adam(self._tab_groups(self.model_mri), self.hparams,
                                     self.device), self.hparams)


class PET_TABULAR_CNN(_TabularStage2):
    """Stage-2 PET + tabular fusion (pkg/models/fusion_models/pet_tabular_fusion.py:15-148):
    Small_PET_CNN from ``path_pet`` (or hparams['path_pet']) cut after GAP + flatten
    (``model[:-3]`` for 2 classes, ``model[:-1]`` otherwise, :28-31), TabPFN decoder
    features -> reduce_tab (``simple_dim_red``: Linear(1024, 512) ReLU Linear(512, 64) ReLU,
    else Linear(1024, 64) ReLU, :54-57), cat (pet, tabular) 128 -> model_fuse =
    Linear(128, 64) -> ReLU -> Linear(64, C)."""

    def __init__(self, hparams, path_pet=None):
        super().__init__(hparams)
        pet = Small_PET_CNN.load_from_checkpoint(path_pet or hparams["path_pet"])
        self.model_pet = pet.model[:-3] if hparams["n_classes"] == 2 else pet.model[:-1]
        self.model_tabular, self.tabular_training_size = tabular.load_model(
            tabular.TRAINPATH, hparams["n_classes"] == 2, ensemble_size=hparams["ensemble_size"])
        if not hparams.get("lr_pretrained"):
            _freeze(self.model_pet)
        self.stage2out = Lyr.Linear(64 + 64, 64)
        self.cls2 = Lyr.Linear(64, hparams["n_classes"])
        self.relu = Lyr.ReLU()
        if self.hparams["simple_dim_red"]:
            self.reduce_tab = nn.Sequential(Lyr.Linear(1024, 512), self.relu,
                                            Lyr.Linear(512, 64), self.relu)
        else:
            self.reduce_tab = nn.Sequential(Lyr.Linear(1024, 64), self.relu)
        self.model_fuse = nn.Sequential(self.stage2out, self.relu, self.cls2)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_tabular):
        out_pet = self.model_pet(x_pet)
        out_tab = self.reduce_tab(self._tab_features(x_tabular))
        return self.model_fuse(head_ops.concat_features(out_pet, out_tab))

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_pet = batch["pet1451"].unsqueeze(1)
        y = batch["label"]
        x_tab = cast(batch["tabular"].unsqueeze(1), torch.float32)
        y_hat, loss = _logits_and_loss(self.criterion, self(x_pet, x_tab), y)
        self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        return _with_scheduler(_adam(self._tab_groups(self.model_pet), self.hparams,
                                     self.device), self.hparams)


class All_Modalities_Fusion(Base_Model):
    """Stage-3 fusion of the three stage-2 models (pkg/models/fusion_models/
    all_modalities_fusion.py:12-137).

    * stage-2 models from checkpoints (:17-26): ``Anat_PET_CNN`` from
      hparams['path_anat_pet'] (with path_pet / path_anat), ``Tabular_MRT_Model`` from
      'path_anat_tab' (path_mri = path_anat), ``PET_TABULAR_CNN`` from 'path_pet_tab'
      (path_pet); each one's classifier cut off, ``model_fuse[:-2]`` = its stage2out alone
      (64-d, no ReLU; :29-31);
    * without lr_pretrained the stage-2 reduce / fuse layers are frozen (:34-47);
    * cat (anat_pet, anat_tab, pet_tab) 192 -> model_fuse = stage3out Linear(192, 64) ->
      ReLU -> cls3 Linear(64, C) (:50-57, :74-79); focal loss or weighted CE (:60-64);
    * Adam over model_fuse at lr, plus the stage-1/2 parts at lr_pretrained (:98-137; the
      reference lists ``model_tabular`` -- a TabPFNClassifier, not a Module -- which raises
      there; its transformer's parameters are taken here, as the stage-2 models do).

    The two tabular stage-2 models need TabPFN (``tabular.load_model``: tabpfn, or a
    registered backend, else ``TabPFNUnavailable``).  The config-5 benchmark network
    (ResNet-34 + ResNet-18 + tabular MLP, one stage) is ``Tri_ResNet_Tabular_Fusion``.
    """

    def __init__(self, hparams):
        super().__init__(hparams)
        self.model_anat_pet = Anat_PET_CNN.load_from_checkpoint(
            hparams["path_anat_pet"], path_pet=hparams["path_pet"],
            path_anat=hparams["path_anat"])
        self.model_anat_tab = Tabular_MRT_Model.load_from_checkpoint(
            hparams["path_anat_tab"], path_mri=hparams["path_anat"])
        self.model_pet_tab = PET_TABULAR_CNN.load_from_checkpoint(
            hparams["path_pet_tab"], path_pet=hparams["path_pet"])
        for m in (self.model_anat_pet, self.model_anat_tab, self.model_pet_tab):
            m.model_fuse = m.model_fuse[:-2]
        if not hparams.get("lr_pretrained"):
            _freeze(self.model_anat_pet.reduce_dim_mri, self.model_anat_pet.model_fuse,
                    self.model_anat_tab.reduce_tab, self.model_anat_tab.model_fuse,
                    self.model_pet_tab.model_fuse, self.model_pet_tab.reduce_tab)
        self.stage3out = Lyr.Linear(64 + 64 + 64, 64)
        self.cls3 = Lyr.Linear(64, hparams["n_classes"])
        self.relu = Lyr.ReLU()
        self.model_fuse = nn.Sequential(self.stage3out, self.relu, self.cls3)
        self.criterion = make_criterion(hparams)
        Lyr.set_compute_dtype(self, Lyr.precision_dtype(hparams))

    def forward(self, x_pet, x_mri, x_tab):
        out_anat_pet = self.model_anat_pet(x_pet, x_mri)
        out_anat_tab = self.model_anat_tab(x_tab, x_mri)
        out_pet_tab = self.model_pet_tab(x_pet, x_tab)
        out = head_ops.concat_features(out_anat_pet, out_anat_tab, out_pet_tab)
        return self.model_fuse(out)

    def general_step(self, batch, batch_idx, mode):
        batch = self.prepare_batch(batch)
        x_pet = batch["pet1451"].unsqueeze(1)
        x_mri = batch["mri"].unsqueeze(1)
        x_tab = cast(batch["tabular"].unsqueeze(1), torch.float32)
        y = batch["label"]
        y_hat, loss = _logits_and_loss(self.criterion, self(x_pet, x_mri, x_tab), y)
        self.log(mode + "_loss", loss, on_step=True, prog_bar=True)
        return {"loss": loss, "outputs": y_hat, "labels": y}

    def configure_optimizers(self):
        groups = [{"params": p, "lr": self.hparams["lr"]} for p in self.model_fuse.parameters()]
        if self.hparams.get("lr_pretrained"):
            ap, pt, at = self.model_anat_pet, self.model_pet_tab, self.model_anat_tab
            prev = [ap.model_pet, ap.model_mri, ap.stage2out, ap.reduce_dim_mri,
                    pt.model_pet, pt.model_tabular, pt.stage2out, pt.reduce_tab,
                    at.model_mri, at.model_tabular, at.stage2out, at.reduce_tab]
            for m in prev:
                ps = m.parameters() if isinstance(m, nn.Module) else _tabpfn_params(m)
                groups += [{"params": p, "lr": self.hparams["lr_pretrained"]} for p in ps]
        return _with_scheduler(_adam(groups, self.hparams, self.device), self.hparams)
