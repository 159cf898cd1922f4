from multimodal_alzheimer_amd.classifiers import FocalLoss  # noqa: F401
