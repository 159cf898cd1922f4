from multimodal_alzheimer_amd.classifiers import Anat_CNN  # noqa: F401
