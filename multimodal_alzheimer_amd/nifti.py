"""Minimal NIfTI-1 reader for the sample table's volumes (``nib.load(path).get_fdata()``,
pkg/utils/dataloader.py:206-207, 228-229, 240-241).

nibabel is not part of this image; the reference only ever reads single-file NIfTI-1
images (``.nii`` / ``.nii.gz``, the MNI-registered 2 mm scans and brain masks) and takes
``get_fdata()``: the voxel array in float64, in the file's axis order (NIfTI stores x
fastest: a Fortran-ordered array of shape ``dim[1:ndim+1]``), scaled by ``scl_slope`` /
``scl_inter`` when the slope is finite and non-zero.  That is what :func:`load` returns.
Parity with nibabel itself is unpinned (nibabel is absent here); tests/test_dataset_cpu.py
checks the reader against files written to the NIfTI-1 layout.
"""
import gzip
import struct

import numpy as np

_DTYPES = {2: "u1", 4: "i2", 8: "i4", 16: "f4", 64: "f8", 256: "i1", 512: "u2", 768: "u4",
           1024: "i8", 1280: "u8"}
HEADER_BYTES = 348


def _read(path):
    with open(path, "rb") as f:
        raw = f.read()
    if raw[:2] == b"\x1f\x8b":
        raw = gzip.decompress(raw)
    return raw


def parse_header(raw):
    """(endian, shape, numpy dtype, vox_offset, slope, inter) of a NIfTI-1 image."""
    if len(raw) < HEADER_BYTES:
        raise ValueError("not a NIfTI-1 file: shorter than its header")
    for endian in ("<", ">"):
        if struct.unpack(endian + "i", raw[:4])[0] == HEADER_BYTES:
            break
    else:
        raise ValueError("not a NIfTI-1 file: sizeof_hdr != 348")
    magic = raw[344:348]
    if magic not in (b"n+1\x00", b"ni1\x00"):
        raise ValueError(f"not a NIfTI-1 file: magic {magic!r}")
    if magic == b"ni1\x00":
        raise ValueError("two-file NIfTI (.hdr/.img) is not supported")
    dim = struct.unpack(endian + "8h", raw[40:56])
    ndim = dim[0]
    if not 1 <= ndim <= 7:
        raise ValueError(f"bad dim[0] = {ndim}")
    shape = tuple(int(d) for d in dim[1:ndim + 1])
    code = struct.unpack(endian + "h", raw[70:72])[0]
    if code not in _DTYPES:
        raise ValueError(f"unsupported NIfTI datatype {code}")
    dtype = np.dtype(endian + _DTYPES[code])
    vox_offset = int(struct.unpack(endian + "f", raw[108:112])[0])
    slope, inter = struct.unpack(endian + "2f", raw[112:120])
    return endian, shape, dtype, max(vox_offset, HEADER_BYTES), slope, inter


def load(path):
    """``nib.load(path).get_fdata()``: float64 voxel array (Fortran-ordered view)."""
    raw = _read(path)
    _, shape, dtype, off, slope, inter = parse_header(raw)
    n = int(np.prod(shape))
    if len(raw) < off + n * dtype.itemsize:
        raise ValueError("NIfTI file truncated")
    data = np.frombuffer(raw, dtype=dtype, count=n, offset=off).reshape(shape, order="F")
    out = data.astype(np.float64)
    if np.isfinite(slope) and slope != 0 and (slope != 1 or inter != 0):
        if not np.isfinite(inter):
            raise ValueError("non-finite scl_inter")
        out = out * float(slope) + float(inter)
    return out


def save(path, data, slope=1.0, inter=0.0):
    """Write ``data`` as a single-file NIfTI-1 image (test fixtures; .gz by extension)."""
    data = np.asarray(data)
    code = {v: k for k, v in _DTYPES.items()}[data.dtype.newbyteorder("=").str[1:]]
    hdr = bytearray(HEADER_BYTES)
    struct.pack_into("<i", hdr, 0, HEADER_BYTES)
    dim = [data.ndim] + list(data.shape) + [1] * (7 - data.ndim)
    struct.pack_into("<8h", hdr, 40, *dim)
    struct.pack_into("<hh", hdr, 70, code, data.dtype.itemsize * 8)
    struct.pack_into("<8f", hdr, 76, *([1.0] * 8))             # pixdim
    struct.pack_into("<f", hdr, 108, 352.0)                    # vox_offset
    struct.pack_into("<2f", hdr, 112, slope, inter)
    hdr[344:348] = b"n+1\x00"
    body = bytes(hdr) + b"\x00" * 4 + np.asarray(data, dtype=data.dtype.newbyteorder("<")) \
        .tobytes(order="F")
    if str(path).endswith(".gz"):
        body = gzip.compress(body)
    with open(path, "wb") as f:
        f.write(body)
