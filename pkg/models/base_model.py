from multimodal_alzheimer_amd.classifiers import Base_Model  # noqa: F401
