"""MI355X-native (gfx950) 3D-volume training hot path of Liz490/multimodal_alzheimer.

MedicalNet 3D-ResNet forward/backward over MRI and PET volumes + the focal /
weighted-CE loss, as hand-written HIP kernels behind the C ABI in include/mmad.h
(libmmad_hip.so), exposed through drop-in replacements of the reference's ``pkg.models``
LightningModule classes (see classifiers.py) and the MedicalNet API (medicalnet.py).
"""
from . import _lib, head_ops, layers, medicalnet, preprocess, tabular, volume_ops  # noqa: F401
from .classifiers import (All_Modalities_Fusion, Anat_CNN, Anat_PET_CNN, Base_Model,  # noqa
                          FocalLoss, PET_CNN_ResNet, PET_MRI_EF, PET_MRI_FMF,
                          PET_MRI_ResNet_Fusion, PET_TABULAR_CNN,
                          Random_Benchmark_All_CN, Small_PET_CNN, Tabular_MLP, Tabular_MRT_Model,
                          Tri_ResNet_Tabular_Fusion)

__version__ = "0.1.0"


def library_path():
    return _lib.LIB_PATH
