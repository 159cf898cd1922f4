"""Diagnostic: for one golden case and one BN layer, the channels whose bias gradient
differs from an f64 evaluation, and the smallest |pre-ReLU activation| (f64) in each:
a value within fp32 rounding of 0 means a ReLU mask flip, not an arithmetic error.
    python tools/diag_maskflip.py anat_r50 model.layer4.1.bn2"""
import sys
import numpy as np
import torch
sys.path.insert(0, '.')
from tests import _golden as G
from tests.test_model_parity_gpu import _f64_oracle_grads, run_product

name, bn_name = sys.argv[1], sys.argv[2]
g, f64 = _f64_oracle_grads(name)
_, m, _ = run_product(name)
ours = dict(m.named_parameters())[bn_name + ".bias"].grad.double().cpu().numpy()
exact = f64[bn_name + ".bias"]
ref32 = g.get(f"grad/full/{bn_name}.bias")
diff = np.abs(ours - exact)
print("max|err| ours", diff.max(), "ref32", None if ref32 is None else np.abs(ref32 - exact).max())
ref = G.build_oracle(name)
G.load_prng_weights(ref, int(g["seed"]))
ref = ref.double()
bn = dict(ref.named_modules())[bn_name]
acts = {}
bn.register_forward_hook(lambda mod, i, o: acts.__setitem__("out", o.detach()))
batch = G.batch_of(name, g)
ref.train()
ref(batch[ref.batch_key].unsqueeze(1).double())
pre = acts["out"]                                     # BN output (before ReLU / residual)
for c in np.argsort(-diff)[:5]:
    v = pre[:, c].abs()
    print(f"channel {c}: |err| {diff[c]:.3e}  min|bn out| {v.min().item():.3e}  "
          f"grad {exact[c]:.3e}")
