"""CPU-side checks of the C ABI: the library loads (no GPU needed) and exports exactly the
functions include/mmad.h declares, with the ctypes table in _lib.py covering all of them.
No kernel is launched here."""
import os
import re
import subprocess

import pytest

from multimodal_alzheimer_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "mmad.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mmad_\w+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        from multimodal_alzheimer_amd import _build
        _build.build()
    return _lib.load()


def test_header_matches_binding_table():
    assert header_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_header_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mmad_\w+)", out))
    missing = set(header_functions()) - exported
    assert not missing, f"not exported: {sorted(missing)}"
    for name in header_functions():
        assert hasattr(lib, name)


def test_abi_version_and_errors(lib):
    assert lib.mmad_abi_version() == 1
    assert lib.mmad_strerror(0) == b"ok"
    assert b"shape" in lib.mmad_strerror(1001)


def test_host_side_shape_queries(lib):
    from multimodal_alzheimer_amd.volume_ops import conv_desc
    d = conv_desc((8, 64, 32, 32, 32), (128, 64, 3, 3, 3), (2, 2, 2), (1, 1, 1), (1, 1, 1))
    assert (d.do_, d.ho, d.wo) == (16, 16, 16)
    assert lib.mmad_conv_packed_elems(d, _lib.BF16, 0) == 128 * 27 * 64
    assert lib.mmad_conv_packed_elems(d, _lib.BF16, 1) == 64 * 27 * 128
    # one BN partial row per output tile: the stride-2 sub-patch kernel's 2 x 8 x 8 boxes in
    # bf16; the implicit GEMM's 64-voxel tiles (grids under 512 tiles of 128) in fp32
    assert lib.mmad_conv3d_stats_rows(d, _lib.BF16) == 8 * 16 ** 3 // 128
    assert lib.mmad_conv3d_stats_rows(d, _lib.F32) == 8 * 16 ** 3 // 64
    assert lib.mmad_conv3d_wgrad_workspace(d, _lib.BF16) > 0
    stem = conv_desc((8, 1, 128, 128, 128), (64, 1, 7, 7, 7), (2, 2, 2), (3, 3, 3), (1, 1, 1))
    assert lib.mmad_conv_unfolded_elems(stem) == 8 * 128 * 128 * 64 * 8
    # bf16 stem runs on the dedicated stem kernel: one BN partial row per (n, y-pair) block
    assert lib.mmad_conv3d_stats_rows(stem, _lib.BF16) == 8 * 64 // 2
    assert lib.mmad_conv3d_stats_rows(stem, _lib.F32) == 8 * 64 ** 3 // 128
    # 49 (kd, kh) taps x 8 unfolded kw "channels" = 392, padded to a 128-byte K slice
    assert lib.mmad_conv_packed_elems(stem, _lib.BF16, 0) == 64 * 448
    bad = conv_desc((1, 64, 8, 8, 8), (64, 64, 3, 3, 3), (1, 1, 1), (1, 1, 1), (1, 1, 1))
    bad.wo = 9   # inconsistent with the torch output-extent formula
    assert lib.mmad_conv_packed_elems(bad, _lib.F32, 0) == -1


def test_wide_stem_routes_by_wgrad_offsets(lib):
    """Column-tiled stems (wo > 64) take the stem kernels only when the hoisted weight
    gradient's 32-bit buffer offsets hold (csrc/stem.hip wg2_small): a 400^3 sample (200^3
    outputs x 64 ch x 2 B < 2^30) stays on the stem (one BN row per block), a 416^3 one
    (208^3 outputs) goes to the implicit GEMM from the forward on (one row per 128-voxel
    tile) -- so its backward never meets a stem wgrad that cannot run."""
    from multimodal_alzheimer_amd.volume_ops import conv_desc
    w = (64, 1, 7, 7, 7)
    on = conv_desc((1, 1, 400, 400, 400), w, (2, 2, 2), (3, 3, 3), (1, 1, 1))
    off = conv_desc((1, 1, 416, 416, 416), w, (2, 2, 2), (3, 3, 3), (1, 1, 1))
    assert on.wo > 64 and off.wo > 64
    assert lib.mmad_conv3d_stats_rows(on, _lib.BF16) == 400
    assert lib.mmad_conv3d_stats_rows(off, _lib.BF16) == 208 ** 3 // 128


def test_bad_arguments_are_rejected_without_launching(lib):
    from multimodal_alzheimer_amd.volume_ops import conv_desc
    d = conv_desc((1, 64, 8, 8, 8), (64, 64, 3, 3, 3), (1, 1, 1), (1, 1, 1), (1, 1, 1))
    assert lib.mmad_conv3d_fwd(d, 7, None, None, None, None, None, None) == 1002
    assert lib.mmad_conv3d_fwd(d, _lib.F32, None, None, None, None, None, None) == 1003
    assert lib.mmad_loss_fwd(0, 2, None, None, None, 0.0, 0, None, None, None) == 1001
    # a misaligned operand is refused before anything is launched (16-byte vector moves);
    # the pointer values are never dereferenced here
    assert lib.mmad_conv3d_fwd(d, _lib.BF16, 0x1008, 0x2000, None, 0x3000, None, None) == 1001
    assert lib.mmad_conv3d_dgrad(d, _lib.BF16, 0x1000, 0x2004, 0x3000, None) == 1001
    assert lib.mmad_conv3d_wgrad(d, _lib.BF16, 0x1000, 0x2000, 0x3000, None, 0x4002,
                                 None) == 1001
    assert b"alignment" in lib.mmad_strerror(1001)
