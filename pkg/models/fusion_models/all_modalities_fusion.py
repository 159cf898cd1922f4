from multimodal_alzheimer_amd.classifiers import (All_Modalities_Fusion, PET_TABULAR_CNN,  # noqa: F401
                                                  Tabular_MRT_Model)
