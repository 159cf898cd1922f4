import sys; sys.path.insert(0, '.')
import torch
from tests.test_fullsize_gpu import _ref_conv, _gen, DEV, BF, CL
from multimodal_alzheimer_amd import volume_ops as V, layers as Lyr
torch.manual_seed(21)
conv = Lyr.Conv3d(512, 512, 3, padding=4, dilation=4, bias=False).to(DEV)
conv.compute_dtype = BF
bn = torch.nn.BatchNorm3d(512).to(DEV)
with torch.no_grad():
    bn.running_mean.uniform_(-0.2, 0.2); bn.running_var.uniform_(0.5, 2.0)
    bn.weight.uniform_(0.5, 1.5); bn.bias.uniform_(-0.3, 0.3)
bn.eval()
g = _gen(22)
x = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
res = (torch.rand((8, 512, 16, 16, 16), generator=g, device=DEV) * 2 - 1).to(BF).contiguous(memory_format=CL)
with torch.no_grad():
    y = V.conv_bn_act_eval(x, conv, bn, relu=True, res=res)
    y0 = V.conv_bn_act_eval(x, conv, bn, relu=False, res=None)
    inv = (1.0 / (bn.running_var.double() + bn.eps).sqrt()).float()
    scale = bn.weight * inv
    shift = bn.bias - bn.running_mean * bn.weight * inv
    wf = (conv.weight * scale.view(-1, 1, 1, 1, 1)).to(BF).float()
    pre = _ref_conv(x.float(), wf, 1, 4, 4) + shift.view(1, -1, 1, 1, 1)
    ref = torch.relu(pre + res.float())
err = (y.float() - ref).abs()
e0 = (y0.float() - pre).abs()
print("no-res/relu path max err", e0.max().item(), "max|pre|", pre.abs().max().item())
idx = torch.nonzero(err > 2 ** -8 * (pre.abs() + res.float().abs()) + 1e-3 * ref.abs().max())
print(len(idx))
for t in idx[:12].tolist():
    n, c, z, yy, xx = t
    print(t, "y", y[n, c, z, yy, xx].item(), "ref", ref[n, c, z, yy, xx].item(), "pre", pre[n, c, z, yy, xx].item(),
          "res", res[n, c, z, yy, xx].item(), "y0", y0[n, c, z, yy, xx].item())
