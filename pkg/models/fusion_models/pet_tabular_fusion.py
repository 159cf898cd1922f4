from multimodal_alzheimer_amd.classifiers import PET_TABULAR_CNN  # noqa: F401
from multimodal_alzheimer_amd.tabular import TRAINPATH, get_avg_activation, load_model  # noqa: F401
