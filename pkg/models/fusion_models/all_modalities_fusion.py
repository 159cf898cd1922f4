from multimodal_alzheimer_amd.classifiers import All_Modalities_Fusion, Tabular_MLP  # noqa: F401
