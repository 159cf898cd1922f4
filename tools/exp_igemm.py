"""A/B helper for implicit-GEMM tile configurations: run the layer3/layer4 convs (fwd and
stride-1 dgrad) on fixed seeded inputs with the configuration chosen by MMAD_IGEMM_BIG and
save the outputs, so two runs with different settings can be compared bit for bit.
    MMAD_IGEMM_BIG=5 python tools/exp_igemm.py out5.pt ; python tools/exp_igemm.py --cmp a b"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodal_alzheimer_amd import _lib as L  # noqa: E402
from multimodal_alzheimer_amd import volume_ops as V  # noqa: E402

CL = torch.channels_last_3d
LAYERS = [("l3c2", 256, 256, 2), ("l4c1", 256, 512, 4), ("l4c2", 512, 512, 4)]


def main():
    if sys.argv[1] == "--cmp":
        a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
        for k in a:
            same = torch.equal(a[k], b[k])
            err = (a[k].float() - b[k].float()).abs().max().item()
            print(f"{k}: bit-identical={same} max|diff|={err:.3e}")
            assert err <= 1e-2 * a[k].float().abs().max().item(), k
        return
    out = {}
    g = torch.Generator(device="cuda").manual_seed(1)
    code = L.BF16
    for name, ci, co, dl in LAYERS:
        x = torch.randn((8, ci, 16, 16, 16), device="cuda", generator=g).to(torch.bfloat16)
        x = x.contiguous(memory_format=CL)
        w = torch.randn((co, ci, 3, 3, 3), device="cuda", generator=g) * 0.02
        d = V.conv_desc(tuple(x.shape), tuple(w.shape), (1,) * 3, (dl,) * 3, (dl,) * 3)
        wp = V.pack_weight(d, code, w, torch.bfloat16, False)
        y = torch.empty((8, co, 16, 16, 16), dtype=torch.bfloat16, device="cuda",
                        memory_format=CL)
        L.call("mmad_conv3d_fwd", d, code, L.ptr(x), L.ptr(wp), None, L.ptr(y), None, L.stream())
        wpt = V.pack_weight(d, code, w, torch.bfloat16, True)
        dx = torch.empty_like(x)
        L.call("mmad_conv3d_dgrad", d, code, L.ptr(y), L.ptr(wpt), L.ptr(dx), L.stream())
        torch.cuda.synchronize()
        out[name + "_fwd"], out[name + "_dgrad"] = y.cpu(), dx.cpu()
    torch.save(out, sys.argv[1])
    print("saved", sys.argv[1])


if __name__ == "__main__":
    main()
