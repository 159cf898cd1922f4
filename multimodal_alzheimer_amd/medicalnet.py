"""MedicalNet-compatible 3D-ResNet running on the MI355X kernels.

The reference builds its backbone with the third-party, un-vendored Tencent/MedicalNet
(``generate_model(opts)`` / ``parse_opts()``, pkg/models/mri_models/anat_cnn.py:4-5,
:18-31).  This module provides the same architecture, module names and state_dict keys
(``conv1``, ``bn1``, ``layer{1..4}.{i}.{conv1,bn1,conv2,bn2[,conv3,bn3]}``,
``layer{2,3,4}.0.downsample.{0,1}``, ``conv_seg``) so MedicalNet checkpoints and the
reference's Lightning checkpoints load unchanged:

* stem: conv 7^3 / s2 / p3 (no bias) -> BN -> ReLU -> max-pool 3^3 / s2 / p1;
* stages 64 / 128 (s2) / 256 (dilation 2) / 512 (dilation 4), padding = dilation;
* shortcut "B": 1^3 conv(stride) + BN when the shape changes;
* depth 10/18/34 (BasicBlock 1111 / 2222 / 3463) and 50 (Bottleneck 3463).

The forward is fused per block: each conv also emits the BN partial sums of its output
from the MFMA epilogue, and BN + residual add + ReLU is one elementwise pass.
"""
import argparse
import os

import torch
import torch.nn as nn

from . import layers as Lyr
from . import volume_ops as V

DEPTHS = {10: ("basic", (1, 1, 1, 1)), 18: ("basic", (2, 2, 2, 2)),
          34: ("basic", (3, 4, 6, 3)), 50: ("bottleneck", (3, 4, 6, 3))}
FEATURES = {10: 512, 18: 512, 34: 512, 50: 2048}


def _conv(cin, cout, k, stride=1, dilation=1):
    return Lyr.Conv3d(cin, cout, k, stride=stride, padding=dilation * (k // 2),
                      dilation=dilation, bias=False)


# Eval-mode (inference, running statistics, no autograd) blocks run each conv+BN(+res)+ReLU
# as one kernel (volume_ops.conv_bn_act_eval); False forces the training-style ops.
EVAL_FUSED = True


def _eval_fused_ok(block, x):
    return (EVAL_FUSED and not block.training and not torch.is_grad_enabled() and x.is_cuda
            and x.dim() == 5)


def _conv_bn_act(conv, bn, x, relu=True, res=None, res_conv=None, res_bn=None, res_x=None,
                 twin=False):
    y, parts = conv.forward_stats(x)
    if res_conv is not None:
        r, rparts = res_conv.forward_stats(res_x)
        return V.batchnorm_act(y, bn, parts, relu=relu, res=r, res_bn=res_bn, res_parts=rparts,
                               twin=twin)
    return V.batchnorm_act(y, bn, parts, relu=relu, res=res, twin=twin)


# A block's input feeds conv1 and the shortcut: the shortcut reads the producer's twin alias
# (volume_ops "twin outputs"), so the two gradients meet inside the producer's BN backward
# instead of in a separate add.  ResNet sets twin_out on every block whose output feeds
# another block.


class BasicBlock(nn.Module):
    expansion = 1
    twin_out = False

    def __init__(self, cin, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(cin, planes, 3, stride, dilation)
        self.bn1 = Lyr.BatchNorm3d(planes)
        self.relu = Lyr.ReLU(inplace=True)
        self.conv2 = _conv(planes, planes, 3, 1, dilation)
        self.bn2 = Lyr.BatchNorm3d(planes)
        self.downsample = downsample
        self.stride = stride
        self.dilation = dilation

    def forward(self, x):
        if _eval_fused_ok(self, x):
            y = self._eval_fused(x)
            if y is not None:
                return y
        h = _conv_bn_act(self.conv1, self.bn1, x)
        xr = V.take_twin(x)
        if self.downsample is None:
            return _conv_bn_act(self.conv2, self.bn2, h, res=xr, twin=self.twin_out)
        return _conv_bn_act(self.conv2, self.bn2, h, res_conv=self.downsample[0],
                            res_bn=self.downsample[1], res_x=xr, twin=self.twin_out)

    def _eval_fused(self, x):
        """3 (or 2) kernels per block instead of 4-5 conv / BN / add passes: BN folded into
        the conv weights, residual add + ReLU in the conv epilogue."""
        h = V.conv_bn_act_eval(x, self.conv1, self.bn1, relu=True)
        if h is None:
            return None
        if self.downsample is None:
            res = x if x.dtype == h.dtype else None
        else:
            res = V.conv_bn_act_eval(x, self.downsample[0], self.downsample[1], relu=False)
        if res is None:
            return None
        return V.conv_bn_act_eval(h, self.conv2, self.bn2, relu=True, res=res)


class Bottleneck(nn.Module):
    expansion = 4
    twin_out = False

    def __init__(self, cin, planes, stride=1, dilation=1, downsample=None):
        super().__init__()
        self.conv1 = _conv(cin, planes, 1)
        self.bn1 = Lyr.BatchNorm3d(planes)
        self.conv2 = _conv(planes, planes, 3, stride, dilation)
        self.bn2 = Lyr.BatchNorm3d(planes)
        self.conv3 = _conv(planes, planes * 4, 1)
        self.bn3 = Lyr.BatchNorm3d(planes * 4)
        self.relu = Lyr.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride
        self.dilation = dilation

    def forward(self, x):
        h = _conv_bn_act(self.conv1, self.bn1, x)
        xr = V.take_twin(x)
        h = _conv_bn_act(self.conv2, self.bn2, h)
        if self.downsample is None:
            return _conv_bn_act(self.conv3, self.bn3, h, res=xr, twin=self.twin_out)
        return _conv_bn_act(self.conv3, self.bn3, h, res_conv=self.downsample[0],
                            res_bn=self.downsample[1], res_x=xr, twin=self.twin_out)


class ResNet(nn.Module):
    def __init__(self, depth=10, n_seg_classes=2, shortcut_type="B"):
        super().__init__()
        if depth not in DEPTHS:
            raise ValueError(f"resnet depth {depth} not in {sorted(DEPTHS)}")
        if shortcut_type != "B":
            raise NotImplementedError("only MedicalNet shortcut 'B' (the reference default)")
        kind, counts = DEPTHS[depth]
        block = BasicBlock if kind == "basic" else Bottleneck
        self.depth = depth
        self._cin = 64
        self.conv1 = Lyr.Conv3d(1, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = Lyr.BatchNorm3d(64)
        self.relu = Lyr.ReLU(inplace=True)
        self.maxpool = Lyr.MaxPool3d(3, stride=2, padding=1)
        self.layer1 = self._stage(block, 64, counts[0], 1, 1)
        self.layer2 = self._stage(block, 128, counts[1], 2, 1)
        self.layer3 = self._stage(block, 256, counts[2], 1, 2)
        self.layer4 = self._stage(block, 512, counts[3], 1, 4)
        blocks = [b for s in (self.layer1, self.layer2, self.layer3, self.layer4) for b in s]
        for b in blocks[:-1]:
            b.twin_out = True        # feeds the next block (conv1 + shortcut)
        # MedicalNet's segmentation head; every reference caller replaces it
        # (anat_cnn.py:79).  Kept so MedicalNet state_dicts load without surprises.
        self.conv_seg = nn.Sequential(
            nn.ConvTranspose3d(512 * block.expansion, 32, 2, stride=2), nn.BatchNorm3d(32),
            nn.ReLU(inplace=True), nn.Conv3d(32, 32, 3, padding=1, bias=False),
            nn.BatchNorm3d(32), nn.ReLU(inplace=True),
            nn.Conv3d(32, n_seg_classes, 1, bias=False))
        for m in self.modules():
            if isinstance(m, nn.Conv3d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
            elif isinstance(m, nn.BatchNorm3d):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def _stage(self, block, planes, count, stride, dilation):
        ds = None
        if stride != 1 or self._cin != planes * block.expansion:
            ds = nn.Sequential(Lyr.Conv3d(self._cin, planes * block.expansion, 1, stride=stride,
                                          bias=False),
                               Lyr.BatchNorm3d(planes * block.expansion))
        blocks = [block(self._cin, planes, stride, dilation, ds)]
        self._cin = planes * block.expansion
        blocks += [block(self._cin, planes, 1, dilation) for _ in range(1, count)]
        return nn.Sequential(*blocks)

    def forward_features(self, x):
        """stem + 4 stages: (N,1,D,H,W) raw volume (f64/f32) -> (N,C,D/8,H/8,W/8) NDHWC."""
        # conv1 -> bn1 -> relu -> maxpool: BN, ReLU and the pool run as one pass over the
        # conv output (volume_ops.batchnorm_relu_maxpool)
        if self.conv1.weight.is_cuda and not _eval_fused_ok(self, x):
            V.prepack(self)          # every conv weight repacked in one launch per step
        V.clear_twins()
        y, parts = self.conv1.forward_stats(x)
        mp = self.maxpool
        x = V.batchnorm_relu_maxpool(y, self.bn1, parts, mp.kernel_size, mp.stride, mp.padding,
                                     twin=True)
        return self.layer4(self.layer3(self.layer2(self.layer1(x))))

    def forward(self, x):
        return self.conv_seg(self.forward_features(x))


def resnet(depth, **kw):
    return ResNet(depth, **kw)


# --- MedicalNet module-level API (MedicalNet.setting.parse_opts / model.generate_model) --
def parse_opts(argv=()):
    """MedicalNet option namespace (only the fields the reference reads or sets).

    Unlike MedicalNet's argparse-on-sys.argv, this never reads the process command line.
    """
    p = argparse.ArgumentParser(add_help=False)
    p.add_argument("--model", default="resnet")
    p.add_argument("--model_depth", type=int, default=10)
    p.add_argument("--resnet_shortcut", default="B")
    p.add_argument("--input_D", type=int, default=56)
    p.add_argument("--input_H", type=int, default=448)
    p.add_argument("--input_W", type=int, default=448)
    p.add_argument("--n_seg_classes", type=int, default=2)
    p.add_argument("--no_cuda", action="store_true")
    p.add_argument("--gpu_id", nargs="+", default=[0])
    p.add_argument("--pretrain_path", default="")
    p.add_argument("--phase", default="train")
    p.add_argument("--new_layer_names", default=["conv_seg"])
    return p.parse_args(list(argv))


def load_pretrained(net, path):
    """Load a MedicalNet ``resnet_{d}_23dataset.pth`` (keys may carry 'module.')."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck.get("state_dict", ck)
    own = net.state_dict()
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    own.update({k: v for k, v in sd.items() if k in own and own[k].shape == v.shape})
    net.load_state_dict(own)


class _Wrapped(nn.Module):
    """Stands in for MedicalNet's nn.DataParallel wrapper: the reference only reads
    ``.module`` (anat_cnn.py:31)."""

    def __init__(self, m):
        super().__init__()
        self.module = m

    def forward(self, *a):
        return self.module(*a)


def generate_model(opts):
    net = ResNet(int(opts.model_depth), int(getattr(opts, "n_seg_classes", 2)),
                 getattr(opts, "resnet_shortcut", "B"))
    path = getattr(opts, "pretrain_path", "")
    if path and os.path.exists(path) and getattr(opts, "phase", "train") != "test":
        load_pretrained(net, path)
    return _Wrapped(net), net.parameters()
