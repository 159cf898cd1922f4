from multimodal_alzheimer_amd.classifiers import PET_CNN_ResNet  # noqa: F401
