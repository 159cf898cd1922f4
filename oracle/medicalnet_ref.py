"""torch-CPU restatement of Tencent/MedicalNet's 3D-ResNet (TEST INFRASTRUCTURE ONLY).

The reference imports ``from MedicalNet.model import generate_model`` and
``from MedicalNet.setting import parse_opts`` (pkg/models/mri_models/anat_cnn.py:4-5,
pkg/models/pet_models/pet_resnet_cnn.py:4-5) but the package is git-ignored
(.gitignore:5), un-vendored and has no pinned version or commit anywhere in the
reference (README.md:38 only links the GitHub project).  This module restates the
published architecture so the reference ``pkg`` code can run here:

* stem  ``conv1`` 7^3 / stride 2 / pad 3, no bias -> ``bn1`` -> ReLU ->
  ``maxpool`` 3^3 / stride 2 / pad 1;
* ``layer1`` (64), ``layer2`` (128, stride 2), ``layer3`` (256, dilation 2),
  ``layer4`` (512, dilation 4) with padding == dilation in every 3^3 conv;
* shortcut "B" (the MedicalNet default; the reference never overrides it,
  anat_cnn.py:18-28): a 1^3 conv(stride) + BN whenever stride != 1 or the channel
  count changes;
* depth table 10/18/34 -> BasicBlock x (1,1,1,1)/(2,2,2,2)/(3,4,6,3); 50 ->
  Bottleneck x (3,4,6,3);
* total stride 8 -- the one in-repo pin: pkg/utils/outdated/inspect_model.py:105 sizes
  a Linear as 12*14*12 after a 91x109x91 input.

Parity against genuine MedicalNet is UNPINNED (no reference test or fixture holds its
numbers); everything downstream is pinned against "reference pkg code + this module".
"""
import argparse

import torch
import torch.nn as nn
import torch.nn.functional as F

DEPTHS = {10: ("basic", (1, 1, 1, 1)), 18: ("basic", (2, 2, 2, 2)),
          34: ("basic", (3, 4, 6, 3)), 50: ("bottleneck", (3, 4, 6, 3))}


class BasicBlockRef(nn.Module):
    expansion = 1

    def __init__(self, cin, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv3d(cin, planes, 3, stride=stride, padding=dilation,
                               dilation=dilation, bias=False)
        self.bn1 = nn.BatchNorm3d(planes)
        self.conv2 = nn.Conv3d(planes, planes, 3, stride=1, padding=dilation,
                               dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm3d(planes)
        self.downsample = downsample

    def forward(self, x):
        h = F.relu(self.bn1(self.conv1(x)))
        h = self.bn2(self.conv2(h))
        r = x if self.downsample is None else self.downsample(x)
        return F.relu(h + r)


class BottleneckRef(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv3d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm3d(planes)
        self.conv2 = nn.Conv3d(planes, planes, 3, stride=stride, padding=dilation,
                               dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm3d(planes)
        self.conv3 = nn.Conv3d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm3d(planes * 4)
        self.downsample = downsample

    def forward(self, x):
        h = F.relu(self.bn1(self.conv1(x)))
        h = F.relu(self.bn2(self.conv2(h)))
        h = self.bn3(self.conv3(h))
        r = x if self.downsample is None else self.downsample(x)
        return F.relu(h + r)


class ResNetRef(nn.Module):
    def __init__(self, depth, n_seg_classes=2):
        super().__init__()
        kind, counts = DEPTHS[depth]
        block = BasicBlockRef if kind == "basic" else BottleneckRef
        self._cin = 64
        self.conv1 = nn.Conv3d(1, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm3d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool3d(3, stride=2, padding=1)
        self.layer1 = self._stage(block, 64, counts[0], 1, 1)
        self.layer2 = self._stage(block, 128, counts[1], 2, 1)
        self.layer3 = self._stage(block, 256, counts[2], 1, 2)
        self.layer4 = self._stage(block, 512, counts[3], 1, 4)
        # MedicalNet's own segmentation head; every reference caller replaces it.
        self.conv_seg = nn.Sequential(
            nn.ConvTranspose3d(512 * block.expansion, 32, 2, stride=2),
            nn.BatchNorm3d(32), nn.ReLU(inplace=True),
            nn.Conv3d(32, 32, 3, padding=1, bias=False), nn.BatchNorm3d(32),
            nn.ReLU(inplace=True), nn.Conv3d(32, n_seg_classes, 1, bias=False))
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
            elif isinstance(m, nn.BatchNorm3d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _stage(self, block, planes, count, stride, dilation):
        ds = None
        if stride != 1 or self._cin != planes * block.expansion:
            ds = nn.Sequential(
                nn.Conv3d(self._cin, planes * block.expansion, 1, stride=stride, bias=False),
                nn.BatchNorm3d(planes * block.expansion))
        blocks = [block(self._cin, planes, stride, dilation, ds)]
        self._cin = planes * block.expansion
        blocks += [block(self._cin, planes, 1, dilation) for _ in range(1, count)]
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.conv_seg(x)


# --- MedicalNet module-level API used by the reference (anat_cnn.py:18-31) -------------

def parse_opts():
    """Namespace with the MedicalNet option names the reference reads or mutates."""
    return argparse.Namespace(
        model="resnet", model_depth=10, resnet_shortcut="B", input_D=56, input_H=448,
        input_W=448, n_seg_classes=2, no_cuda=True, gpu_id=[0], pretrain_path="",
        new_layer_names=["conv_seg"], phase="train")


def generate_model(opts):
    """(DataParallel-like wrapper exposing ``.module``, parameter list)."""
    net = ResNetRef(int(opts.model_depth), getattr(opts, "n_seg_classes", 2))

    class _Wrapped(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.module = m

        def forward(self, *a):
            return self.module(*a)

    return _Wrapped(net), net.parameters()
