"""Diagnostic: per-parameter gradient error of the HIP path and of the reference fp32
(golden) against a float64 oracle evaluation, for one golden case."""
import sys
import numpy as np
sys.path.insert(0, '.')
from tests.test_model_parity_gpu import _f64_oracle_grads, run_product

name = sys.argv[1]
g, f64 = _f64_oracle_grads(name)
_, m, _ = run_product(name)
params = dict(m.named_parameters())
for key in g:
    if not key.startswith("grad/") or "/stats/" in key:
        continue
    pname = key.split("/", 2)[2]
    ref32 = g[key]
    exact = f64[pname][: ref32.size]
    ours = params[pname].grad.detach().double().cpu().numpy().ravel()[: ref32.size]
    print(f"{pname:50s} max|g|={np.abs(exact).max():.3e} ref32={np.abs(ref32-exact).max():.2e} ours={np.abs(ours-exact).max():.2e}")
