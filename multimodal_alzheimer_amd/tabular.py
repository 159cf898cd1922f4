"""TabPFN boundary of the stage-2 tabular fusion models.

The reference's ``Tabular_MRT_Model`` (pkg/models/fusion_models/tabular_mri_fusion.py:11-80)
and ``PET_TABULAR_CNN`` (pet_tabular_fusion.py:15-104) take their tabular features from
TabPFN (``tabpfn==0.1.8``, a third-party pretrained transformer, absent offline): at
construction ``load_model`` fits a ``TabPFNClassifier`` on the tabular training rows
(pkg/models/tabular_models/dl_approach.py:47-54, :65-68); at every forward the models hook
its first decoder Linear (``model[2].decoder[0]``), run ``predict_proba`` on the CPU copy of
the batch and average the test rows' activations over the ensemble members
(dl_approach.py:71-78) -- a detached [B, 1024] input to ``reduce_tab``.

This module restates those three pieces with the reference's names and contracts:

* ``load_model(path, binary_classification, ensemble_size)`` -> (classifier, n_train).
  With ``tabpfn`` importable it does what dl_approach.py:65-68 does (the tabular rows of the
  sample table at ``path`` -- data_preparation.py:19-38 -- then ``TabPFNClassifier(device=
  'cuda', N_ensemble_configurations=ensemble_size).fit(...)``).  Without it, a backend
  registered by ``set_backend`` supplies the classifier (the tests register the seeded
  stand-in of ``oracle/tabpfn_standin.py``); with neither, ``TabPFNUnavailable`` names the
  missing package -- no silent substitute.
* ``get_avg_activation`` -- dl_approach.py:71-78.
* ``decoder_features`` -- the hook / predict_proba / average sequence of
  tabular_mri_fusion.py:58-74 and pet_tabular_fusion.py:80-97.

TabPFN is not on the volume hot path (its output is detached; the reference runs it on
the CPU copy of the batch, ``x_tabular.cpu()``); everything after it runs on libmmad_hip.so.
"""
import os

import torch

# data_preparation.py:15-16 (resolved against the working directory at import, as there)
BASEPATH = os.getcwd()
TRAINPATH = os.path.join(BASEPATH, "data/train_path_data_labels.csv")

_BACKEND = None


class TabPFNUnavailable(RuntimeError):
    """TabPFN (tabpfn==0.1.8 and its pretrained prior) is needed and not installed."""


def set_backend(load_model_fn):
    """Register ``load_model_fn(path, binary_classification, ensemble_size) ->
    (classifier, n_train)`` for builds without TabPFN; ``None`` clears it.  The classifier
    must expose ``predict_proba(x, normalize_with_test=False)`` and a hookable
    ``model[2].decoder[0]`` module, as TabPFNClassifier does."""
    global _BACKEND
    _BACKEND = load_model_fn


def get_data(path, binary_classification):
    """data_preparation.py:19-38: every tabular row of the sample table at ``path`` (the
    dataset's tabular modality, one shuffled batch) -> (features, labels)."""
    from torch.utils.data import DataLoader
    from .dataset import MultiModalDataset
    ds = MultiModalDataset(path=path, binary_classification=binary_classification,
                           modalities=["tabular"])
    batch = next(iter(DataLoader(ds, batch_size=len(ds), shuffle=True)))
    return batch["tabular"], batch["label"]


def load_model(path, binary_classification=True, ensemble_size=4):
    """dl_approach.py:65-68: a TabPFN classifier fitted on the training rows, and their
    count (the offset of the test rows in the decoder activations)."""
    if _BACKEND is not None:
        return _BACKEND(path, binary_classification, ensemble_size)
    try:
        import tabpfn
    except ImportError as e:
        raise TabPFNUnavailable(
            "the stage-2 tabular fusion models (Tabular_MRT_Model, PET_TABULAR_CNN) need "
            "TabPFN (tabpfn==0.1.8 with its pretrained prior), which is not installed; "
            "install it, or register a feature backend with "
            "multimodal_alzheimer_amd.tabular.set_backend(load_model_fn)") from e
    x_train, y_train = get_data(path, binary_classification)
    clf = tabpfn.TabPFNClassifier(device="cuda", N_ensemble_configurations=ensemble_size)
    clf.fit(x_train, y_train, overwrite_warning=True)          # dl_approach.py:51-52
    return clf, x_train.shape[0]


def get_avg_activation(activations, num_ensemble, training_size):
    """dl_approach.py:71-78: the test rows of the [n_train + B, E, 1024] decoder activations,
    summed over the ensemble members in member order and divided by E -> [B, 1024]."""
    out = None
    for i in range(num_ensemble):
        a = activations[training_size:, i:i + 1, :]
        out = a if out is None else out + a
    out = out / num_ensemble
    return torch.transpose(out, 0, 1).squeeze(dim=0)


def decoder_features(classifier, x_tabular, num_ensemble, training_size):
    """tabular_mri_fusion.py:58-74 / pet_tabular_fusion.py:80-97: hook the first decoder
    Linear, run predict_proba on the CPU copy of the (B, 1, F) batch, return the averaged
    activations (detached)."""
    acts = {}

    def hook(module, inp, output):
        acts["dec"] = output.detach()

    handle = classifier.model[2].decoder[0].register_forward_hook(hook)
    try:
        classifier.predict_proba(x_tabular.detach().cpu().squeeze(dim=1),
                                 normalize_with_test=False)
    finally:
        handle.remove()
    return get_avg_activation(acts["dec"], num_ensemble, training_size)
