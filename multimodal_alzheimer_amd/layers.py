"""nn.Module drop-ins whose forward runs the MI355X kernels.

Each class subclasses the torch module it replaces and keeps its constructor, parameters
and buffers, so state_dict keys, checkpoint files, ``load_state_dict`` and slicing of
``nn.Sequential`` heads (anat_pet_fusion.py:28-32) behave exactly as in the reference.
Only ``forward`` changes.  Volumes flow as channels_last_3d tensors (NDHWC); the compute
dtype of a conv is its ``compute_dtype`` attribute (float32 parity mode by default,
bfloat16 throughput mode), and every downstream op follows the dtype of its input.
"""
import os

import torch
import torch.nn as nn

from . import head_ops, volume_ops

_SUPPORTED_DTYPES = (torch.float32, torch.bfloat16)


def _triple(v):
    if isinstance(v, int):
        return (v, v, v)
    return tuple(int(a) for a in v)


class Conv3d(nn.Conv3d):
    """nn.Conv3d (groups=1, zero padding, symmetric 'same') -> MFMA implicit GEMM."""

    compute_dtype = torch.float32

    def _pads(self):
        if isinstance(self.padding, str):
            if self.padding == "valid":
                return (0, 0, 0)
            pads = []
            for k, d in zip(self.kernel_size, self.dilation):
                if (d * (k - 1)) % 2:
                    raise NotImplementedError("padding='same' with an even kernel extent")
                pads.append(d * (k - 1) // 2)
            return tuple(pads)
        return _triple(self.padding)

    _prepacked = None     # (fwd, dgrad) packed weights from volume_ops.PackPlan.run

    def _stride3(self):
        return _triple(self.stride)

    def _dilation3(self):
        return _triple(self.dilation)

    def forward_stats(self, x):
        """(y, bn partial sums): the conv epilogue also reduces the output per channel."""
        return self._run(x, True)

    def _run(self, x, want_stats):
        if self.groups != 1 or self.padding_mode != "zeros":
            raise NotImplementedError("groups != 1 / non-zero padding_mode")
        cd = self.compute_dtype
        # raw inputs (Cin = 1, or a channel stack of Cin < 8) are cast by the conv's own
        # unfold / gather pass
        if isinstance(x, torch.Tensor) and x.shape[1] % 8 == 0 and x.dtype != cd:
            x = volume_ops.cast(x, cd)
        packed, self._prepacked = self._prepacked, None     # valid for one forward only
        return volume_ops.conv3d(x, self.weight, self.bias, _triple(self.stride), self._pads(),
                                 _triple(self.dilation), cd, want_stats, packed)

    def forward(self, x):
        return self._run(x, False)


class BatchNorm3d(nn.BatchNorm3d):
    def forward(self, x):
        return volume_ops.batchnorm_act(x, self)


class BatchNorm1d(nn.BatchNorm1d):
    def forward(self, x):
        if x.dim() != 2:
            raise NotImplementedError("BatchNorm1d over (B, C, L) inputs")
        return volume_ops.batchnorm_act(x.contiguous(), self)


class ReLU(nn.ReLU):
    def forward(self, x):
        return volume_ops.relu(x)


class MaxPool3d(nn.MaxPool3d):
    def forward(self, x):
        k, s, p = _triple(self.kernel_size), _triple(self.stride or self.kernel_size), \
            _triple(self.padding)
        if len(set(k)) != 1 or len(set(s)) != 1 or len(set(p)) != 1 or \
                _triple(self.dilation) != (1, 1, 1) or self.ceil_mode or self.return_indices:
            raise NotImplementedError("MaxPool3d: cubic windows, dilation 1, floor mode only")
        return volume_ops.max_pool3d(x, k[0], s[0], p[0])


class AdaptiveAvgPool3d(nn.AdaptiveAvgPool3d):
    def forward(self, x):
        if _triple(self.output_size) != (1, 1, 1):
            raise NotImplementedError("AdaptiveAvgPool3d only to 1x1x1 (global average)")
        return volume_ops.global_avg_pool(x)


class Linear(nn.Linear):
    def forward(self, x):
        return head_ops.linear(x, self.weight, self.bias)


class Sequential(nn.Sequential):
    """nn.Sequential (same modules, indices, state_dict keys and slicing) whose
    ``Linear -> ReLU`` pairs run as one fused launch each way (head_ops.linear(relu=True):
    the ReLU in the dot-product epilogue, its mask in the linear backward).  A pair with
    module hooks runs unfused."""

    def forward(self, x):
        mods = list(self._modules.values())
        i = 0
        while i < len(mods):
            m = mods[i]
            nxt = mods[i + 1] if i + 1 < len(mods) else None
            # AdaptiveAvgPool3d(1) -> Flatten -> Linear (-> ReLU): head_ops.gap_linear
            k = _gap_linear_run(mods, i, x)
            if k:
                lin = mods[i + 2]
                x = head_ops.gap_linear(x, lin.weight, lin.bias, relu=k == 4)
                i += k
                continue
            if (type(m) is Linear and type(nxt) is ReLU and x.dim() == 2 and
                    not (m._forward_hooks or m._forward_pre_hooks or nxt._forward_hooks or
                         nxt._forward_pre_hooks)):
                x = head_ops.linear(x, m.weight, m.bias, relu=True)
                i += 2
                continue
            x = m(x)
            i += 1
        return x


# MMAD_GAP_LINEAR=0: conv_seg's pool -> flatten -> linear run module by module (A/B)
GAP_LINEAR = os.environ.get("MMAD_GAP_LINEAR", "1") != "0"


def _gap_linear_run(mods, i, x):
    """modules fused by head_ops.gap_linear at position i (4 with a trailing ReLU, 3
    without), else 0"""
    if not (GAP_LINEAR and volume_ops.GAP_BCAST) or i + 2 >= len(mods):
        return 0
    m, f, lin = mods[i], mods[i + 1], mods[i + 2]
    if not (type(m) is AdaptiveAvgPool3d and type(f) is nn.Flatten and type(lin) is Linear):
        return 0
    if lin.in_features > 4096:                  # mmad_gap_linear_fwd's pooled-row buffer
        return 0
    if _triple(m.output_size) != (1, 1, 1) or f.start_dim != 1 or f.end_dim != -1:
        return 0
    if not (isinstance(x, torch.Tensor) and x.dim() == 5 and x.is_cuda and
            x.dtype in (torch.float32, torch.bfloat16)):
        return 0
    if x.shape[1] != lin.in_features:           # unfused: the Linear raises its shape error
        return 0
    relu =i + 3 < len(mods) and type(mods[i + 3]) is ReLU
    used = mods[i:i + (4 if relu else 3)]
    if any(u._forward_hooks or u._forward_pre_hooks for u in used):
        return 0
    return 4 if relu else 3


class Dropout(nn.Dropout):
    def forward(self, x):
        return head_ops.dropout(x, self.p, self.training)


class CrossEntropyLoss(nn.CrossEntropyLoss):
    """nn.CrossEntropyLoss(weight) (registers ``weight`` -> state_dict 'criterion.weight')."""

    def forward(self, input, target):
        if self.ignore_index != -100 or self.label_smoothing != 0.0 or self.reduction != "mean":
            raise NotImplementedError("only weighted 'mean' cross entropy")
        return head_ops.weighted_cross_entropy(input, target, self.weight)

    def fused_spec(self):
        """(weight, gamma, mode) for head_ops.logits_and_loss"""
        if self.ignore_index != -100 or self.label_smoothing != 0.0 or self.reduction != "mean":
            return None
        return self.weight, 0.0, 0


_TORCH_TO_HIP = {
    nn.Conv3d: Conv3d, nn.BatchNorm3d: BatchNorm3d, nn.BatchNorm1d: BatchNorm1d,
    nn.ReLU: ReLU, nn.MaxPool3d: MaxPool3d, nn.AdaptiveAvgPool3d: AdaptiveAvgPool3d,
    nn.Linear: Linear, nn.Dropout: Dropout,
}


def set_compute_dtype(module, dtype):
    """Select float32 (parity) or bfloat16 (throughput) compute for every conv below."""
    if dtype not in _SUPPORTED_DTYPES:
        raise ValueError(f"compute dtype must be one of {_SUPPORTED_DTYPES}")
    for m in module.modules():
        if isinstance(m, Conv3d):
            m.compute_dtype = dtype
    return module


def precision_dtype(hparams):
    """hparams['precision'] -> torch dtype; the reference trains fp32 (no precision key)."""
    p = str((hparams or {}).get("precision", "32")).lower()
    if p in ("32", "fp32", "float32", "32-true"):
        return torch.float32
    if p in ("bf16", "bfloat16", "bf16-mixed", "bf16-true"):
        return torch.bfloat16
    raise ValueError(f"unsupported precision {p!r}")
