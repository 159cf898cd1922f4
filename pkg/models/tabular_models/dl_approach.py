from multimodal_alzheimer_amd.tabular import get_avg_activation, get_data, load_model  # noqa: F401
