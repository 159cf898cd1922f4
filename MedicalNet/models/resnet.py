from multimodal_alzheimer_amd.medicalnet import ResNet, BasicBlock, Bottleneck, resnet  # noqa: F401
