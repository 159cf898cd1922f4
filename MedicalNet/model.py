from multimodal_alzheimer_amd.medicalnet import generate_model  # noqa: F401
