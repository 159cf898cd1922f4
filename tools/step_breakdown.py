"""Per-category time of one step from a prof_summary 'step' table.
    python tools/step_breakdown.py profiles/r01_step_kernels.txt"""
import collections
import re
import sys

RULES = [("igemm", "igemm fwd/dgrad"), ("lattice_wgrad", "lattice wgrad"),
         ("lattice", "lattice conv fwd/dgrad"), ("patch_conv", "patch conv"), ("wgrad_kernel", "wgrad"),
         ("reduce", "wgrad reduce"), ("slab", "wgrad reduce"), ("stem_fwd", "stem fwd"),
         ("stem_wgrad", "stem wgrad"), ("bnpool", "bnpool fused"), ("scale_shift", "bn apply"),
         ("colsum", "bn bwd reduce"), ("bn_bwd_apply", "bn bwd apply"),
         ("unfold", "stem input unfold"), ("finalize", "bn finalize"), ("fold", "bn finalize"),
         ("pack", "weight pack"), ("pwgrad", "wgrad"), ("Cijk", "1x1 dgrad (hipBLASLt)"), ("FusedOpt", "adam"), ("TensorListMetadata", "adam"),
         ("CUDAFunctor_add", "residual add (torch)"), ("gap", "gap")]


def main(path):
    cat = collections.Counter()
    for line in open(path):
        m = re.match(r"\s*([\d.]+)\s+g=\s*\S+\s+(.*)", line)
        if not m:
            continue
        us, name = float(m.group(1)), m.group(2)
        key = next((k for pat, k in RULES if pat in name), "other (head/loss/casts)")
        cat[key] += us
    tot = sum(cat.values())
    for k, v in cat.most_common():
        print(f"{k:26s} {v:8.1f} us {100 * v / tot:5.1f}%")
    print(f"{'total':26s} {tot:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
