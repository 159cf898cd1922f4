from multimodal_alzheimer_amd.classifiers import Tabular_MRT_Model  # noqa: F401
from multimodal_alzheimer_amd.tabular import TRAINPATH, get_avg_activation, load_model  # noqa: F401
