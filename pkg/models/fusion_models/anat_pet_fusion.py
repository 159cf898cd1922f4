from multimodal_alzheimer_amd.classifiers import Anat_PET_CNN, PET_MRI_ResNet_Fusion  # noqa: F401
