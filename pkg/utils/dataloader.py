"""pkg.utils.dataloader (pkg/utils/dataloader.py:21-436) -> the MI355X drop-in."""
from multimodal_alzheimer_amd.dataset import MultiModalDataset  # noqa: F401
