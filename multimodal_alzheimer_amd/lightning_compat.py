"""PyTorch-Lightning 1.x surface used by the reference models, with an offline fallback.

When ``pytorch_lightning`` is importable the drop-in models subclass the real
``LightningModule`` and the reference ``train_*.py`` drivers run unchanged.  This image
has no Lightning, so a minimal stand-in provides exactly what the reference models touch:
``save_hyperparameters`` -> ``self.hparams``, ``log`` / ``log_dict``, ``device``,
``current_epoch``, and PL-1.7.7-format ``save_checkpoint`` / ``load_from_checkpoint``
(keys: state_dict, hyper_parameters, epoch, global_step, pytorch-lightning_version,
optimizer_states, lr_schedulers, callbacks, loops).  The same goes for the two
torchmetrics classes Base_Model uses (pkg/models/base_model.py:3-4, :21-32).
None of this is on the hot path.
"""
import copy

import torch
import torch.nn as nn

try:  # pragma: no cover - not installed in this image
    import pytorch_lightning as _pl
    LightningModule = _pl.LightningModule
    HAVE_LIGHTNING = True
except ImportError:
    _pl = None
    HAVE_LIGHTNING = False

    class AttributeDict(dict):
        def __getattr__(self, k):
            try:
                return self[k]
            except KeyError as e:
                raise AttributeError(k) from e

        def __setattr__(self, k, v):
            self[k] = v

    class LightningModule(nn.Module):
        """Offline stand-in for pytorch_lightning.LightningModule (1.7 API subset)."""

        def __init__(self, *a, **k):
            super().__init__()
            self._hparams = AttributeDict()
            self.logged = {}
            self.current_epoch = 0
            self.global_step = 0
            self.logger = None

        @property
        def hparams(self):
            return self._hparams

        def save_hyperparameters(self, hparams=None, ignore=()):
            src = dict(hparams or {})
            self._hparams = AttributeDict({k: v for k, v in src.items() if k not in ignore})

        def log(self, name, value, *a, **k):
            # detached, as Lightning's result collection stores logged tensors: a logged loss
            # that kept its grad_fn would hold the step's whole autograd graph -- and the
            # parameters' AccumulateGrad nodes with the stream they were created on -- alive
            # into the next step (torch then warns of an AccumulateGrad stream mismatch, and
            # a graph capture after eager default-stream steps faulted at capture_end)
            self.logged[name] = value.detach() if torch.is_tensor(value) else value

        def log_dict(self, d, *a, **k):
            for name, value in d.items():
                self.log(name, value)

        @property
        def device(self):
            for p in self.parameters():
                return p.device
            return torch.device("cpu")

        def save_checkpoint(self, path, epoch=0, global_step=0, optimizer_states=()):
            torch.save({
                "epoch": epoch, "global_step": global_step,
                "pytorch-lightning_version": "1.7.7",
                "state_dict": self.state_dict(),
                "hyper_parameters": dict(self.hparams),
                "optimizer_states": list(optimizer_states), "lr_schedulers": [],
                "callbacks": {}, "loops": {},
            }, path)

        @classmethod
        def load_from_checkpoint(cls, checkpoint_path, map_location=None, strict=True,
                                 **kwargs):
            ck = torch.load(checkpoint_path, map_location=map_location or "cpu",
                            weights_only=True)
            hp = dict(ck.get("hyper_parameters", {}))
            model = cls(hp, **kwargs) if hp else cls(**kwargs)
            model.load_state_dict(ck["state_dict"], strict=strict)
            return model

try:  # pragma: no cover - not installed in this image
    from torchmetrics.classification import MulticlassF1Score, MulticlassMatthewsCorrCoef
    HAVE_TORCHMETRICS = True
except ImportError:
    HAVE_TORCHMETRICS = False

    class _ConfMat(nn.Module):
        def __init__(self, num_classes):
            super().__init__()
            self.num_classes = num_classes
            self.cm = None

        def to(self, *a, **k):
            return self

        def update(self, preds, target):
            if preds.dim() == 2:
                preds = preds.argmax(1)
            idx = (target.long() * self.num_classes + preds.long()).detach().cpu()
            cm = torch.bincount(idx, minlength=self.num_classes ** 2).reshape(
                self.num_classes, self.num_classes).double()
            self.cm = cm if self.cm is None else self.cm + cm

        def reset(self):
            self.cm = None

        def forward(self, preds, target):
            self.update(preds, target)

    class MulticlassF1Score(_ConfMat):
        """torchmetrics' macro / per-class F1 from a confusion matrix (rows = target)."""

        def __init__(self, num_classes, average="macro"):
            super().__init__(num_classes)
            self.average = average

        def compute(self):
            cm = self.cm if self.cm is not None else torch.zeros(self.num_classes,
                                                                 self.num_classes,
                                                                 dtype=torch.double)
            tp = cm.diag()
            denom = 2 * tp + (cm.sum(0) - tp) + (cm.sum(1) - tp)
            f1 = torch.where(denom > 0, 2 * tp / denom.clamp(min=1e-300), torch.zeros_like(tp))
            if self.average == "none":
                return f1.float()
            present = (cm.sum(1) + cm.sum(0)) > 0
            return (f1[present].mean() if present.any() else f1.sum() * 0).float()

    class MulticlassMatthewsCorrCoef(_ConfMat):
        def compute(self):
            cm = self.cm if self.cm is not None else torch.zeros(self.num_classes,
                                                                 self.num_classes,
                                                                 dtype=torch.double)
            t = cm.sum(1)
            p = cm.sum(0)
            c = cm.trace()
            s = cm.sum()
            num = c * s - (t * p).sum()
            den = torch.sqrt((s * s - (p * p).sum()) * (s * s - (t * t).sum()))
            return (num / den if den > 0 else den * 0).float()


def clone_hparams(h):
    return copy.copy(dict(h))
