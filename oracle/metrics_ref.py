"""CPU restatement of the test-set bootstrap metrics (TEST INFRASTRUCTURE ONLY).

Base_Model.bootstrap_metric (pkg/models/base_model.py:219-239): n_drawings times, draw n
indices with torch.randint(0, n, (n,)), evaluate the metric on the drawn (y_hat, y) and
record metric.compute(); return mean and 1.96 * std (unbiased) of the recorded values.
The metrics are torchmetrics 0.10.2's (absent offline; environment.yml pins the version):
  * MulticlassF1Score(average='macro') on argmax predictions: per-class F1 = 2tp /
    (2tp + fp + fn), mean over the classes with tp + fp + fn > 0;
  * MulticlassMatthewsCorrCoef: (c*s - sum tk*pk) / sqrt((s^2 - sum pk^2)(s^2 - sum tk^2)),
    0 when the denominator vanishes.
Pinned against scikit-learn's f1_score(average='macro') / matthews_corrcoef in
tests/test_oracle_golden.py (an independent implementation of the same definitions).
"""
import numpy as np
import torch


def confusion(pred, target, n_classes):
    cm = np.zeros((n_classes, n_classes), dtype=np.int64)
    np.add.at(cm, (np.asarray(target), np.asarray(pred)), 1)
    return cm


def macro_f1(cm):
    tp = np.diag(cm).astype(np.float64)
    fp = cm.sum(0) - tp
    fn = cm.sum(1) - tp
    used = (tp + fp + fn) > 0
    if not used.any():
        return 0.0
    return float(np.mean(2 * tp[used] / (2 * tp[used] + fp[used] + fn[used])))


def mcc(cm):
    cm = cm.astype(np.float64)
    tk, pk = cm.sum(1), cm.sum(0)
    c, s = np.trace(cm), cm.sum()
    cov_tp = c * s - (tk * pk).sum()
    cov_pp = s * s - (pk * pk).sum()
    cov_tt = s * s - (tk * tk).sum()
    den = cov_pp * cov_tt
    return 0.0 if den == 0 else float(cov_tp / np.sqrt(den))


def bootstrap(kind, y_hat, y, n_drawings=1000):
    """base_model.py:219-239 with the metric above; draws from torch's global CPU RNG."""
    fn = macro_f1 if kind == "f1" else mcc
    n, c = y_hat.shape
    pred = torch.argmax(y_hat, dim=1).numpy()
    yy = y.numpy()
    vals = np.zeros(n_drawings, dtype=np.float32)
    for i in range(n_drawings):
        m = torch.randint(0, n, (n,)).numpy()
        vals[i] = np.float32(fn(confusion(pred[m], yy[m], c)))
    v = torch.from_numpy(vals)
    return torch.mean(v), 1.96 * torch.std(v), vals
