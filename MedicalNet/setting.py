from multimodal_alzheimer_amd.medicalnet import parse_opts  # noqa: F401
