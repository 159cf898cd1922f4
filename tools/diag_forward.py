"""Diagnostic: forward activations of the HIP fp32 path and of the torch fp32 CPU oracle
against a float64 oracle, per ResNet stage (train-mode BN), for one golden case."""
import sys
import torch
sys.path.insert(0, '.')
from tests import _golden as G
from tests.test_model_parity_gpu import build_product

name = sys.argv[1]
g = G.load(name)
batch = G.batch_of(name, g)
acts = {}

def hook(tag):
    def f(mod, inp, out):
        acts[tag] = out.detach().double().cpu()
    return f

def run(model, tag, x, dev):
    hs = [getattr(model.model, n).register_forward_hook(hook(f"{tag}.{n}"))
          for n in ("maxpool", "layer1", "layer2", "layer3", "layer4")]
    model.train()
    y = model(x.to(dev))
    for h in hs:
        h.remove()
    acts[f"{tag}.logits"] = y.detach().double().cpu()

ref64 = G.build_oracle(name); G.load_prng_weights(ref64, int(g["seed"])); ref64 = ref64.double()
ref32 = G.build_oracle(name); G.load_prng_weights(ref32, int(g["seed"]))
ours = build_product(name); G.load_prng_weights(ours, int(g["seed"])); ours = ours.cuda()
x = batch["mri"].unsqueeze(1)
run(ref64, "f64", x.double(), "cpu")
run(ref32, "r32", x.float(), "cpu")
run(ours, "hip", x, "cuda")
for n in ("maxpool", "layer1", "layer2", "layer3", "layer4", "logits"):
    e = acts[f"f64.{n}"]
    for t in ("r32", "hip"):
        a = acts[f"{t}.{n}"]
        err = (a - e).abs().max().item()
        flips = ((a > 0) != (e > 0)).sum().item()
        print(f"{n:8s} {t}: max|err| {err:.3e}  (scale {e.abs().max().item():.3e})  sign flips {flips}")
