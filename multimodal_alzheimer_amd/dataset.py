"""The multimodal sample table: per-modality rows merged into PET/MRI/tabular pairs and
triples (``MultiModalDataset``, pkg/utils/dataloader.py:21-344), the unit the data-parallel
path shards (data_parallel.shard_indices / ShardSampler).

The reference builds the merged table row by row: for every row of the base table
(``df_base.iterrows()``, :141-156) it filters the next modality's table by ID and label and
a time window (``find_corresponding_samples``, :347-396), then fixes up the matches
(``merge_two_dfs``, :398-436) and appends them with ``pd.concat`` -- quadratic in the table
length.  :func:`merge_modalities` computes the same table in one vectorised pass per
modality:

* candidate pairs = equi-join of (ID, label) between the base rows and the new modality's
  rows, ordered base-row-major and, within a base row, in the new table's row order (the
  order the reference appends them in);
* time window (:386-393): keep a pair when ``ses - min_time <= days`` and
  ``max_time - ses <= days`` (whole days; the reference's ``Timedelta.days``);
* ``min_time`` / ``max_time`` (:419-426) become ``ses`` when it lies before / after them;
* fill (:431-435): for every base row's group of matches and every column, when any match
  has a null in that column and the base row has a value, the WHOLE column of the group
  takes the base row's value (non-null entries included, as the reference's
  ``df2[col2] = df1[col2]`` does).

The result is identical to the reference's table (IDs, labels, paths, tabular values,
``min_time`` / ``max_time``, row order; tests/test_dataset_cpu.py against fixtures
generated from the reference class itself, tests/golden/make_merge_golden.py).

``__getitem__`` reads the NIfTI volumes with :mod:`.nifti` (float64, nibabel's
``get_fdata`` layout) and, like the reference (:197-321), returns them normalised per
``normalize_pet`` / ``normalize_mri`` / ``quantile`` -- the loader's own float64 statements
(preprocess.loader_normalize_*), so an unchanged ``train_*.py`` sees the reference's tensors.
``device_normalize=True`` (opt-in) moves that work to the GPU: ``__getitem__`` then returns
the raw volumes, the brain mask (``mri_mask``) and the settings (``preprocess.NORM_SPEC_KEY``),
and the model applies them batched on the device before its first conv
(classifiers.Base_Model.prepare_batch -> preprocess.VolumeNormalizer, norm.hip).
"""
import numpy as np
import pandas as pd
import torch

from . import nifti
from .preprocess import (NORM_SPEC_KEY, VolumeNormalizer, loader_normalize_mri,
                         loader_normalize_pet, spec_string)

MODALITIES = ("pet1451", "t1w", "tabular")
# the column whose presence selects each modality's rows (dataloader.py:108-121)
_PRESENCE = {"pet1451": "path_pet1451", "t1w": "path_anat", "tabular": "AGE"}
DATE_FORMAT = "%Y-%m-%d"                       # dataloader.py:129


def _day_numbers(col):
    """datetime column -> int64 day numbers (the reference's dates are whole days)"""
    return pd.to_datetime(col).values.astype("datetime64[D]").astype(np.int64)


def _isnull(values):
    return pd.isna(np.asarray(values, dtype=object))


def _merge_step(base, new, days_threshold):
    """One round of dataloader.py:141-155: ``base`` (columns + min_time / max_time, no
    ses) against the next modality ``new`` (with ses as datetime)."""
    if len(base) == 0 or "ID" not in base.columns:
        return pd.DataFrame()
    lb = pd.DataFrame({"ID": base["ID"].values, "label": base["label"].values,
                       "_l": np.arange(len(base))})
    rb = pd.DataFrame({"ID": new["ID"].values, "label": new["label"].values,
                       "_r": np.arange(len(new))})
    # ``df['ID'] == id`` never matches a missing key (pandas' merge would pair NaN with NaN)
    lb = lb[lb["ID"].notna() & lb["label"].notna()]
    rb = rb[rb["ID"].notna() & rb["label"].notna()]
    pairs = lb.merge(rb, on=["ID", "label"], how="inner")
    pairs = pairs.sort_values(["_l", "_r"], kind="stable")
    li, ri = pairs["_l"].to_numpy(np.int64), pairs["_r"].to_numpy(np.int64)
    ses = _day_numbers(new["ses"])[ri]
    mn = _day_numbers(base["min_time"])[li]
    mx = _day_numbers(base["max_time"])[li]
    ok = (ses - mn <= days_threshold) & (mx - ses <= days_threshold)
    li, ri, ses, mn, mx = li[ok], ri[ok], ses[ok], mn[ok], mx[ok]
    if len(li) == 0:
        return pd.DataFrame()

    ses_ts = pd.to_datetime(new["ses"]).values[ri]
    cols = [c for c in new.columns if c != "ses"] + ["min_time", "max_time"]
    out = {}
    # group boundaries: one group per base row (li is sorted)
    starts = np.flatnonzero(np.r_[True, li[1:] != li[:-1]])
    group = np.cumsum(np.r_[False, li[1:] != li[:-1]])
    for c in cols:
        if c == "min_time":
            vals = np.where(mn - ses > 0, ses_ts, base["min_time"].values[li])
        elif c == "max_time":
            vals = np.where(mx - ses < 0, ses_ts, base["max_time"].values[li])
        else:
            vals = new[c].values[ri]
        if c not in base.columns:
            raise KeyError(c)              # the reference indexes df1 by every df2 column
        null = _isnull(vals)
        if null.any():
            grp_any = np.logical_or.reduceat(null, starts)[group]
            bvals = base[c].values[li]
            take = grp_any & ~_isnull(bvals)
            if take.any():
                vals = np.where(take, bvals, vals) if vals.dtype == bvals.dtype else \
                    np.where(take, bvals.astype(object), vals.astype(object))
        out[c] = vals
    df = pd.DataFrame(out, columns=cols)
    return df.infer_objects()


def merge_modalities(frames, days_threshold=180):
    """dataloader.py:124-156: the merged sample table of the per-modality tables ``frames``
    (``modality_tables``; the first is the base).  Like the reference, the first table
    gains ``min_time`` / ``max_time`` (= its session date) in place."""
    if len(frames) == 1:
        return pd.concat([pd.DataFrame(), frames[0]], ignore_index=True)
    for f in frames:
        f["ses"] = pd.to_datetime(f["ses"], format=DATE_FORMAT)
    base = frames[0]
    base["min_time"] = base["ses"]
    base["max_time"] = base["ses"]
    base = base.drop(columns="ses")
    for new in frames[1:]:
        base = _merge_step(base, new, days_threshold)
    return base


def modality_tables(table, modalities):
    """dataloader.py:106-121: the rows of each requested modality (index reset), in the
    reference's FIXED order PET, MRI, tabular -- whatever order ``modalities`` lists them
    in (the first present one is the merge's base table)."""
    return [table.dropna(subset=_PRESENCE[m]).reset_index(drop=True)
            for m in MODALITIES if m in modalities]


class MultiModalDataset(torch.utils.data.Dataset):
    """Drop-in for pkg.utils.dataloader.MultiModalDataset (dataloader.py:21-344): same
    constructor arguments, merged table ``ds``, ``label_mapping``, ``__len__``,
    ``get_label_distribution`` and ``__getitem__`` (normalised float64 volumes, the 9
    tabular features, the label).

    ``device_normalize`` (build extension, default False = the reference's behaviour):
    ``__getitem__`` returns raw volumes + ``mri_mask`` (per-scan MRI modes) + the settings
    string, and the model normalises the collated batch on the GPU (``normalize_batch``
    does the same for a caller that wants it explicitly)."""

    def __init__(self, path, binary_classification=False,
                 modalities=("pet1451", "t1w", "tabular"), days_threshold=180,
                 transform_pet=None, transform_mri=None, transform_tabular=None,
                 normalize_pet=None, normalize_mri=None, quantile=0.99,
                 device_normalize=False):
        self.entire_ds = pd.read_csv(path)
        if binary_classification == 2:
            binary_classification = True
        elif binary_classification == 3:
            binary_classification = False
        self.binary_classification = binary_classification
        if self.binary_classification:
            self.entire_ds = self.entire_ds[self.entire_ds["label"] != "MCI"]
            self.label_mapping = {"CN": 0, "Dementia": 1}
        else:
            self.label_mapping = {"CN": 0, "MCI": 1, "Dementia": 2}
        self.days_threshold = days_threshold
        self.modalities = list(modalities)
        if len(self.modalities) not in (1, 2, 3) or \
                any(m not in MODALITIES for m in self.modalities) or \
                len(set(self.modalities)) != len(self.modalities):
            raise AssertionError(f"modalities must be 1-3 distinct of {MODALITIES}")
        self.df_list = modality_tables(self.entire_ds, self.modalities)
        for m, df in zip([m for m in MODALITIES if m in self.modalities], self.df_list):
            setattr(self, {"pet1451": "df_pet", "t1w": "df_anat", "tabular": "df_tab"}[m], df)
        self.ds = merge_modalities(self.df_list, days_threshold)
        self.ds = self.ds.replace({np.nan: None})
        self.transform_pet = transform_pet
        self.transform_mri = transform_mri
        self.transform_tabular = transform_tabular
        if normalize_pet:
            assert isinstance(normalize_pet.get("mean"), float)
            assert isinstance(normalize_pet.get("std"), float)
        self.normalize_pet = normalize_pet
        self.normalize_mri = normalize_mri
        self.quantile = quantile
        self.device_normalize = bool(device_normalize)
        # the reference checks normalize_mri when a sample is fetched (:236-281); the device
        # path checks it here, where its settings are fixed
        if self.device_normalize:
            self.normalizer                                      # validates the settings
        self._spec = spec_string(normalize_mri, normalize_pet, quantile)

    def __len__(self):
        return len(self.ds)

    def _volume(self, path, transform):
        data = nifti.load(path)
        if transform:
            data = transform(data)
        return torch.as_tensor(data)

    def __getitem__(self, index):
        sample = self.ds.iloc[index]
        host = not self.device_normalize
        data = {}
        p = sample.get("path_pet1451")
        if p is not None:
            pet = self._volume(p, self.transform_pet)
            if self.normalize_pet and host:
                pet = loader_normalize_pet(pet, self.normalize_pet)      # :213-215
            data["pet1451"] = pet
        p = sample.get("path_anat")
        if p is not None:
            mri = self._volume(p, self.transform_mri)
            nm = self.normalize_mri
            if nm:
                per_scan = isinstance(nm, dict) and "per_scan_norm" in nm
                mask = (torch.as_tensor(nifti.load(sample["path_anat_mask"]))
                        if per_scan else None)                           # :240-242
                if host:
                    mri = loader_normalize_mri(mri, mask, nm, self.quantile)   # :236-281
                elif per_scan:
                    data["mri_mask"] = mask
            data["mri"] = mri
        if sample.get("AGE") is not None:
            # dataloader.py:294-306, including its 'whole_brain' read from PTEDUCAT
            keys = ("AGE", "PTEDUCAT", "Ventricles", "Hippocampus", "PTEDUCAT", "Entorhinal",
                    "Fusiform", "MidTemp", "ICV")
            data["tabular"] = torch.tensor([sample[k] for k in keys])
        data["label"] = torch.tensor(self.label_mapping[sample["label"]])
        if not host and (self.normalize_mri or self.normalize_pet):
            data[NORM_SPEC_KEY] = self._spec
        # the reference's key order: pet1451, mri, tabular, label
        order = ("pet1451", "mri", "mri_mask", "tabular", "label", NORM_SPEC_KEY)
        return {k: data[k] for k in order if k in data}

    @property
    def normalizer(self):
        return VolumeNormalizer(self.normalize_mri or None, self.normalize_pet or None,
                                self.quantile)

    def normalize_batch(self, batch):
        """The reference's per-sample normalisation (dataloader.py:213-282), on a collated
        device batch."""
        return self.normalizer(batch)

    def get_label_distribution(self):
        """dataloader.py:323-344: (absolute, normalised) class counts in label order."""
        order = ["CN", "Dementia"] if self.binary_classification else ["CN", "MCI", "Dementia"]
        counts_n = self.ds["label"].value_counts(normalize=True).reindex(index=order)
        counts = self.ds["label"].value_counts().reindex(index=order)
        return torch.tensor(counts.to_numpy()), torch.tensor(counts_n.to_numpy())
