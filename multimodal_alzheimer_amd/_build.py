"""Build libmmad_hip.so in-tree with hipcc for gfx950 (no torch / cmake involved).

    python -m multimodal_alzheimer_amd._build [--force]

Each .hip translation unit compiles to an object in ``build/`` (parallel), then one
link produces ``multimodal_alzheimer_amd/libmmad_hip.so``.  Objects are rebuilt when
their source or any header is newer.
"""
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(REPO, "build", "obj")
LIB = os.path.join(PKG, "libmmad_hip.so")
ARCH = os.environ.get("MMAD_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++20", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(REPO, "include", "*.h"))
    return max(os.path.getmtime(h) for h in hs)


def _compile(src, force, obj_dir=OBJ, defines=()):
    obj = os.path.join(obj_dir, os.path.basename(src).replace(".hip", ".o"))
    if not force and os.path.exists(obj) and os.path.getmtime(obj) >= max(
            os.path.getmtime(src), _headers_mtime()):
        return obj, None
    cmd = [HIPCC, *FLAGS, *defines, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}"
    return obj, None


def build(force=False, verbose=False, defines=(), lib=None):
    """defines: extra -D flags for an A/B variant build (objects in build/obj-<tag>, the
    library at ``lib``; load it with MMAD_LIB_PATH)."""
    obj_dir = OBJ if not defines else OBJ + "-" + "_".join(
        d.replace("=", "").replace("-D", "") for d in defines)
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        results = list(ex.map(lambda s: _compile(s, force, obj_dir, defines), srcs))
    errs = [e for _, e in results if e]
    if errs:
        raise RuntimeError("hipcc failed:\n" + "\n".join(errs))
    objs = [o for o, _ in results]
    out = lib or LIB
    if out != LIB:
        os.makedirs(os.path.dirname(out), exist_ok=True)
    if force or not os.path.exists(out) or os.path.getmtime(out) < max(map(os.path.getmtime, objs)):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out, *objs,
               "-L/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if verbose:
        print(f"built {out}")
    return out


if __name__ == "__main__":
    # python -m multimodal_alzheimer_amd._build [--force] [--variant NAME -DFLAG=V ...]
    args = sys.argv[1:]
    if "--variant" in args:
        i = args.index("--variant")
        name = args[i + 1]
        defs = [a for a in args[i + 2:] if a.startswith("-D")]
        build(force="--force" in args, verbose=True, defines=defs,
              lib=os.path.join(REPO, "variants", name, "libmmad_hip.so"))
    else:
        build(force="--force" in args, verbose=True)
