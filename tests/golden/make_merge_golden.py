"""Golden fixtures for the multimodal sample merge, generated from the REAL reference class
``pkg.utils.dataloader.MultiModalDataset`` (build container only).

    python tests/golden/make_merge_golden.py     # writes merge_samples.csv, merge_golden.json

1. A synthetic sample table in the reference's CSV schema (pkg/utils/create_csv/
   data_labels.py:204, 257, 266-274: one row per scan or tabular visit, written with the
   index column) is drawn from a fixed numpy seed: subjects with several sessions per
   modality, session dates straddling the 90 / 180 / 365-day thresholds, label changes
   between visits (mismatches), MCI rows, tabular rows with missing features, and a few
   rows carrying two modalities at once (so a group of matches can be partly null in a
   column).
2. The reference class is imported from /root/reference with bookkeeping stubs for the
   packages this image lacks (nibabel, torchvision.transforms; nothing of them runs during
   construction) and built on that CSV for a list of settings; its merged table ``ds``
   and ``get_label_distribution()`` are written as JSON.
The reference source never leaves this container; the fixtures are data.
"""
import json
import os
import sys
import types

import numpy as np
import pandas as pd

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
CSV = os.path.join(HERE, "merge_samples.csv")
OUT = os.path.join(HERE, "merge_golden.json")

# (modalities, binary_classification, days_threshold)
SETTINGS = [
    (["pet1451", "t1w"], True, 180),
    (["t1w", "pet1451"], False, 180),
    (["pet1451", "t1w", "tabular"], False, 180),
    (["t1w", "tabular"], True, 90),
    (["pet1451"], False, 180),
    (["tabular", "pet1451", "t1w"], 3, 365),
    (["pet1451", "t1w"], 2, 0),
    (["t1w", "pet1451", "tabular"], True, 180),
]
FEATURES = ["Ventricles", "Hippocampus", "WholeBrain", "Entorhinal", "Fusiform", "MidTemp",
            "ICV", "AGE", "PTEDUCAT"]


def make_table(seed=2024, n_subjects=36):
    rng = np.random.RandomState(seed)
    rows = []
    base_day = pd.Timestamp("2016-01-01")
    labels = ["CN", "MCI", "Dementia"]
    for s in range(n_subjects):
        sid = f"sub-{s * 7 + 3:04d}"
        lab = labels[rng.randint(3)]
        visits = np.cumsum(rng.choice([0, 45, 90, 150, 179, 180, 181, 200, 364, 365, 366],
                                      size=rng.randint(1, 4)))
        for v in visits:
            vlab = lab if rng.rand() > 0.2 else labels[rng.randint(3)]   # label changes
            day = base_day + pd.Timedelta(days=int(v + rng.randint(0, 30)))
            if rng.rand() < 0.8:
                rows.append({"ID": sid, "ses": day + pd.Timedelta(days=int(rng.randint(-20, 20))),
                             "path_pet1451": f"/data/{sid}/pet/{v}_MNI_2mm.nii.gz", "label": vlab})
            for k in range(rng.randint(0, 3)):
                r = {"ID": sid, "ses": day + pd.Timedelta(days=int(rng.choice([-181, -90, 0, 30, 179, 180]))),
                     "path_anat": f"/data/{sid}/anat/{v}_{k}_reg_ants2_MNI_2mm.nii.gz",
                     "path_anat_mask": f"/data/{sid}/anat/{v}_{k}_mask.nii.gz",
                     "label": vlab if rng.rand() > 0.1 else labels[rng.randint(3)]}
                if rng.rand() < 0.1:               # a scan row that also carries a visit
                    r.update({f: float(np.round(rng.rand() * 1000, 3)) for f in FEATURES})
                rows.append(r)
            if rng.rand() < 0.7:
                r = {"ID": sid, "ses": day + pd.Timedelta(days=int(rng.randint(-200, 200))),
                     "label": vlab}
                r.update({f: float(np.round(rng.rand() * 1000, 3)) for f in FEATURES})
                r["AGE"] = float(np.round(60 + rng.rand() * 30, 4))
                r["PTEDUCAT"] = float(rng.randint(8, 21))
                if rng.rand() < 0.2:
                    r["Ventricles"] = np.nan
                rows.append(r)
    df = pd.DataFrame(rows)
    df["ses"] = df["ses"].dt.strftime("%Y-%m-%d")
    cols = ["ID", "ses", "path_pet1451", "label", "path_anat", "path_anat_mask"] + FEATURES
    return df[cols]


def install_stubs():
    nib = types.ModuleType("nibabel")
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")

    class _T:
        def __init__(self, *a, **k):
            raise RuntimeError("not used while building the table")

    tvt.ToTensor, tvt.Normalize = _T, _T
    tv.transforms = tvt
    sys.modules.update({"nibabel": nib, "torchvision": tv, "torchvision.transforms": tvt,
                        "seaborn": types.ModuleType("seaborn")})
    sys.path[:] = [p for p in sys.path
                   if os.path.abspath(p or ".") != os.path.dirname(os.path.dirname(HERE))]
    for name in [m for m in sys.modules if m == "pkg" or m.startswith("pkg.")]:
        del sys.modules[name]
    sys.path.insert(0, REF)


def record(ds):
    """the merged table as JSON-able rows: None for missing, ISO dates, floats as floats"""
    def val(v):
        if v is None or (isinstance(v, float) and np.isnan(v)):
            return None
        if isinstance(v, pd.Timestamp):
            return v.strftime("%Y-%m-%d")
        if isinstance(v, (np.integer, int)) and not isinstance(v, bool):
            return float(v)
        if isinstance(v, (np.floating, float)):
            return float(v)
        return str(v)
    return {"columns": [str(c) for c in ds.columns],
            "rows": [[val(v) for v in row] for row in ds.itertuples(index=False, name=None)]}


def main():
    table = make_table()
    table.to_csv(CSV)                       # with the index column, as data_labels.py:274
    install_stubs()
    from pkg.utils.dataloader import MultiModalDataset
    assert MultiModalDataset.__module__ == "pkg.utils.dataloader"
    out = {"settings": [], "csv": os.path.basename(CSV)}
    for mods, binary, days in SETTINGS:
        d = MultiModalDataset(CSV, binary_classification=binary, modalities=mods,
                              days_threshold=days)
        rec = {"modalities": mods, "binary_classification": binary, "days_threshold": days,
               "len": len(d), "table": record(d.ds)}
        try:
            counts, counts_n = d.get_label_distribution()
            rec["counts"] = [None if np.isnan(c) else float(c) for c in counts.double().tolist()]
            rec["counts_normalized"] = [None if np.isnan(c) else float(c)
                                        for c in counts_n.double().tolist()]
        except KeyError as e:            # an empty merged table has no 'label' column
            rec["label_distribution_error"] = f"KeyError: {e}"
        out["settings"].append(rec)
        print(mods, binary, days, "->", len(d), "samples")
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)


if __name__ == "__main__":
    main()
