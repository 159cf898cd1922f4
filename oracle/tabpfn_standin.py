"""Build-defined stand-in for TabPFN -- TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference's stage-2 tabular fusion models (pkg/models/fusion_models/
tabular_mri_fusion.py:11-80, pet_tabular_fusion.py:15-104) embed TabPFN
(``tabpfn==0.1.8``, pkg/models/tabular_models/dl_approach.py:9, :47-54): a pretrained
transformer fitted on the tabular training rows at construction time.  The fusion models
do not use its predictions; they hook ``classifier.model[2].decoder[0]`` (the first
decoder Linear, output [n_train + n_test, n_ensemble, 1024]), call
``predict_proba(x_test, normalize_with_test=False)`` and average the test rows over the
ensemble members (dl_approach.py:71-78).  TabPFN and its pretrained prior are absent
offline, so parity of that feature extractor is unpinned; what the fixtures pin is
everything around it (the hook, the averaging, reduce_tab, the cuts, the concatenation
order and the stage-3 head).

This stand-in has exactly the surface those call sites touch -- ``fit(X, y,
overwrite_warning=...)``, ``predict_proba(X, normalize_with_test=...)``, ``model[2].decoder``
as ``Sequential(Linear(F, 1024), GELU, Linear(1024, C))``, ``classes_`` -- with seeded
weights (``oracle.prng``): ensemble member i sees the [train; test] rows with its features
rolled by i (TabPFN's ensemble members differ by feature order).  The classifier is a
plain object, not an nn.Module, like TabPFNClassifier, so it adds nothing to a fusion
model's state_dict; its ``model[2]`` is an nn.Module, as TabPFN's transformer is.  The golden generator installs it as ``tabpfn.TabPFNClassifier`` under the
reference code; the GPU tests hand it to ``multimodal_alzheimer_amd.tabular.set_backend``.
"""
import numpy as np
import torch
import torch.nn as nn

from . import prng

HIDDEN = 1024          # TabPFN decoder width (nhid), the 1024 of reduce_tab's Linear(1024, .)


def training_table(seed, n_rows, n_features=9, n_classes=2):
    """Synthetic tabular training rows (the 9 ADNI features, dataloader.py:306) and labels,
    as ``data_preparation.get_data`` returns them (float64 tensor, int64 labels)."""
    x = prng.uniform(seed, n_rows * n_features).astype(np.float64).reshape(n_rows, n_features)
    y = prng.labels(seed + 1, n_rows, n_classes)
    y[:n_classes] = np.arange(n_classes)          # every class present
    return torch.from_numpy(x * 2.0 - 1.0), torch.from_numpy(y)


class _Transformer(nn.Module):
    """``classifier.model[2]`` (an nn.Module, as TabPFN's TransformerModel; the fusion models
    freeze / optimise its parameters and hook its decoder)."""

    def __init__(self, n_features, n_classes, seed):
        super().__init__()
        self.decoder = nn.Sequential(nn.Linear(n_features, HIDDEN), nn.GELU(),
                                     nn.Linear(HIDDEN, n_classes))
        with torch.no_grad():
            for i, p in enumerate(self.decoder.parameters()):
                u = prng.uniform(seed * 16 + i, p.numel()).astype(np.float64)
                p.copy_(torch.from_numpy((2.0 * u - 1.0) * 0.5).float().reshape(p.shape))


class TabPFNClassifier:
    """Stand-in for ``tabpfn.TabPFNClassifier(device=..., N_ensemble_configurations=E)``."""

    def __init__(self, device="cpu", N_ensemble_configurations=4, seed=4242):
        self.device = device
        self.n_ensemble = int(N_ensemble_configurations)
        self.seed = seed
        self.model = None

    def fit(self, X, y, overwrite_warning=False):
        X = torch.as_tensor(np.asarray(X), dtype=torch.float32)
        self.X_ = X
        self.classes_ = np.unique(np.asarray(y))
        self.model = (None, None, _Transformer(X.shape[1], len(self.classes_), self.seed))
        return self

    def predict_proba(self, X, normalize_with_test=False):
        X = torch.as_tensor(np.asarray(X), dtype=torch.float32).reshape(-1, self.X_.shape[1])
        rows = torch.cat([self.X_, X], 0)
        members = torch.stack([torch.roll(rows, i, dims=1) for i in range(self.n_ensemble)], 1)
        with torch.no_grad():
            out = self.model[2].decoder(members)
        n_train = self.X_.shape[0]
        return torch.softmax(out[n_train:], -1).mean(1).numpy()


def make_backend(seed=4242, n_rows=16, n_features=9):
    """``load_model(path, binary_classification, ensemble_size)`` over the synthetic table:
    (fitted stand-in, n_train) -- dl_approach.py:65-68's contract."""
    def load_model(path, binary_classification=True, ensemble_size=4):
        n_classes = 2 if binary_classification else 3
        x, y = training_table(seed, n_rows, n_features, n_classes)
        clf = TabPFNClassifier(N_ensemble_configurations=ensemble_size, seed=seed)
        clf.fit(x, y, overwrite_warning=True)
        return clf, x.shape[0]
    return load_model
