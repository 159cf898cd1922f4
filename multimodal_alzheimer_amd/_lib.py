"""ctypes binding of libmmad_hip.so (the C ABI declared in include/mmad.h).

torch is imported first on purpose: it loads its bundled HIP runtime
(``libamdhip64.so.7``), and the library's own dependency on that soname then resolves to
the same runtime, so torch's streams and allocations are valid handles for our kernels.

There is no fallback: if the library is missing or a call is made on tensors that are not
on a HIP device, the call raises.
"""
import ctypes as C
import os

import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
# MMAD_LIB_PATH: an alternative build of the same library (A/B experiments, tools/)
LIB_PATH = os.environ.get("MMAD_LIB_PATH") or os.path.join(_PKG, "libmmad_hip.so")

F32, BF16, F64 = 0, 1, 2
EUNSUPPORTED = 1004
EHIP = 2000
_HIP_OOM = 2   # hipErrorOutOfMemory

_vp, _i32, _i64, _f32, _f64, _u64 = C.c_void_p, C.c_int, C.c_int64, C.c_float, C.c_double, C.c_uint64


class ConvDesc(C.Structure):
    _fields_ = [(n, C.c_int32) for n in (
        "n", "ci", "di", "hi", "wi", "co", "do_", "ho", "wo", "kd", "kh", "kw",
        "sd", "sh", "sw", "pd", "ph", "pw", "dd", "dh", "dw")]


class PackJob(C.Structure):
    """mirror of mmad_pack_job (include/mmad.h)"""
    _fields_ = ([("w", C.c_void_p), ("w_packed", C.c_void_p)] +
                [(n, C.c_int32) for n in ("rows", "cols", "batch", "jdiv", "ostride_j2",
                                          "tiles_x", "tiles_y", "pad_", "rdiv")] +
                [(n, C.c_int64) for n in ("ostride_b", "ostride_j1", "tile0")])


class PackDual(C.Structure):
    """mirror of mmad_pack_dual (include/mmad.h)"""
    _fields_ = ([("w", C.c_void_p), ("w_fwd", C.c_void_p), ("w_dgrad", C.c_void_p)] +
                [(n, C.c_int32) for n in ("co", "ci", "taps", "flip")] + [("tile0", C.c_int64)])


class AdamJob(C.Structure):
    """mirror of mmad_adam_job (include/mmad.h)"""
    _fields_ = ([(n, C.c_void_p) for n in ("param", "grad", "exp_avg", "exp_avg_sq", "step",
                                           "lr")] +
                [(n, C.c_double) for n in ("beta1", "beta2", "eps", "weight_decay")] +
                [("w_fwd", C.c_void_p), ("w_dgrad", C.c_void_p)] +
                [(n, C.c_int32) for n in ("co", "ci", "taps", "flip", "unf_kw", "kpad")] +
                [(n, C.c_int64) for n in ("numel", "tile0", "ntiles")])


class BnFin(C.Structure):
    """mirror of mmad_bn_fin (include/mmad.h)"""
    _fields_ = ([("nparts", C.c_int32)] +
                [(n, C.c_void_p) for n in ("parts", "gamma", "beta", "running_mean",
                                           "running_var")] +
                [("momentum", C.c_float), ("eps", C.c_float), ("training", C.c_int32)] +
                [(n, C.c_void_p) for n in ("mean", "invstd", "scale", "shift",
                                           "num_batches_tracked")])


class WgradJob(C.Structure):
    """mirror of mmad_wgrad_job (include/mmad.h): one deferred slab reduction"""
    _fields_ = ([("ws", C.c_void_p), ("dw", C.c_void_p)] +
                [(n, C.c_int32) for n in ("splits", "nd", "k", "cs", "taps", "tper", "kind",
                                          "gx", "gy", "gz")])


_P = C.POINTER(ConvDesc)
_PJ = C.POINTER(PackJob)
_PD = C.POINTER(PackDual)
_PA = C.POINTER(AdamJob)
_SIGS = {
    "mmad_abi_version": (_i32, []),
    "mmad_strerror": (C.c_char_p, [_i32]),
    "mmad_set_kernel_variant": (_i32, [C.c_char_p, _i32]),
    "mmad_conv_packed_elems": (_i64, [_P, _i32, _i32]),
    "mmad_conv_pack_weight": (_i32, [_P, _i32, _vp, _vp, _i32, _vp]),
    "mmad_conv_pack_job": (_i32, [_P, _i32, _i32, _vp, _vp, _i64, _PJ]),
    "mmad_pack_job_tiles": (_i64, [_PJ]),
    "mmad_conv_pack_batch": (_i32, [_i32, _i32, _vp, _i64, _vp]),
    "mmad_conv_pack_dual_job": (_i32, [_P, _i32, _vp, _vp, _vp, _i64, _PD]),
    "mmad_pack_dual_tiles": (_i64, [_PD]),
    "mmad_conv_pack_dual_batch": (_i32, [_i32, _i32, _vp, _i64, _vp]),
    "mmad_adam_job_tiles": (_i64, [_PA]),
    "mmad_adam_repack": (_i32, [_i32, _vp, _vp, _i64, _vp, _vp]),
    "mmad_conv_unfolded_elems": (_i64, [_P]),
    "mmad_conv_unfold_input": (_i32, [_P, _i32, _vp, _i32, _vp, _vp]),
    "mmad_conv3d_stats_rows": (_i64, [_P, _i32]),
    "mmad_conv3d_fwd": (_i32, [_P, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_conv3d_dgrad": (_i32, [_P, _i32, _vp, _vp, _vp, _vp]),
    "mmad_conv3d_dgrad_bnsum_rows": (_i64, [_P, _i32]),
    "mmad_conv3d_dgrad_bnsum": (_i32, [_P, _i32] + [_vp] * 10),
    "mmad_conv3d_wgrad_workspace": (_i64, [_P, _i32]),
    "mmad_conv3d_wgrad": (_i32, [_P, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_conv3d_wgrad_split": (_i32, [_P, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_conv3d_wgrad_deferred": (_i32, [_P, _i32, _vp, _vp, _vp, _vp,
                                          C.POINTER(WgradJob), _vp]),
    "mmad_conv3d_wgrad_raw_deferred": (_i32, [_P, _i32, _vp, _i32, _vp, _vp, _vp,
                                              C.POINTER(WgradJob), _vp]),
    "mmad_wgrad_reduce_batch": (_i32, [_i32, C.POINTER(WgradJob), _vp]),
    "mmad_stem_raw_ok": (_i32, [_P, _i32, _i32]),
    "mmad_conv3d_fwd_raw": (_i32, [_P, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "mmad_conv3d_wgrad_raw": (_i32, [_P, _i32, _vp, _i32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_bn_stats_parts": (_i64, [_i64, _i32]),
    "mmad_bn_stats": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp]),
    "mmad_bn_parts_fold": (_i32, [_i32, _i32, _vp, _i32, _vp, _vp]),
    "mmad_bn_finalize": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _f32, _f32, _i32,
                                _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_bn_finalize2": (_i32, [_i32, _i64, C.POINTER(BnFin), C.POINTER(BnFin), _vp]),
    "mmad_scale_shift_act": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _vp,
                                    _vp]),
    "mmad_bn_bwd_parts": (_i64, [_i64, _i32]),
    "mmad_bn_bwd_reduce": (_i32, [_i32, _i64, _i32] + [_vp] * 8),
    "mmad_bn_bwd_finalize": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "mmad_bn_bwd_apply": (_i32, [_i32, _i64, _i32] + [_vp] * 10),
    "mmad_bn_bwd_reduce2": (_i32, [_i32, _i64, _i32, _vp, _vp, _i64] + [_vp] * 10),
    "mmad_bn_bwd_finalize2": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp,
                                     _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "mmad_bn_bwd_apply2": (_i32, [_i32, _i64, _i32, _vp, _vp, _i64] + [_vp] * 12),
    "mmad_relu_fwd": (_i32, [_i32, _i64, _vp, _vp, _vp]),
    "mmad_relu_bwd": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp]),
    "mmad_colsum_ws": (_i32, [_i32, _i64, _i32, _vp, _vp, _vp, _vp]),
    "mmad_add": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp]),
    "mmad_maxpool3d_fwd": (_i32, [_i32] * 12 + [_vp, _vp, _vp, _vp]),
    "mmad_maxpool3d_bwd": (_i32, [_i32] * 12 + [_vp, _vp, _vp, _vp]),
    "mmad_bnpool_fwd": (_i32, [_i32] * 12 + [_vp] * 7),
    "mmad_bnpool_bwd_reduce": (_i32, [_i32, _i64, _i32] + [_vp] * 9),
    "mmad_bnpool_bwd_apply": (_i32, [_i32] * 12 + [_vp] * 8),
    "mmad_gap_fwd": (_i32, [_i32, _i32, _i64, _i32, _vp, _vp, _vp]),
    "mmad_gap_fwd_ws_elems": (_i64, [_i32, _i64, _i32]),
    "mmad_conv3d_fwd_ex": (_i32, [_P, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp]),
    "mmad_conv_pack_weight_scaled": (_i32, [_P, _i32, _vp, _vp, _vp, _i32, _vp]),
    "mmad_bn_fold": (_i32, [_i32, _vp, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp]),
    "mmad_norm_ws_bytes": (_i64, [_i32, _i64]),
    "mmad_mri_minmax_norm": (_i32, [_i32, _i64, _vp, _vp, _f64, _vp, _vp, _vp, _vp]),
    "mmad_mri_zscore_norm": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "mmad_affine_norm": (_i32, [_i64, _vp, _f64, _f64, _vp, _vp]),
    "mmad_gap_fwd_ws": (_i32, [_i32, _i32, _i64, _i32, _vp, _vp, _vp, _vp]),
    "mmad_gap_bwd": (_i32, [_i32, _i32, _i64, _i32, _vp, _vp, _vp]),
    "mmad_gap_bwd_compact": (_i32, [_i32, _i32, _i64, _i32, _vp, _vp, _vp]),
    "mmad_gap_parts": (_i32, [_i32, _i64, _i32]),
    "mmad_gap_partial": (_i32, [_i32, _i32, _i64, _i32, _vp, _vp, _vp]),
    "mmad_gap_linear_fwd": (_i32, [_i32, _i32, _i32, _i32, _i64, _vp, _vp, _vp, _i32, _vp,
                                   _vp, _vp]),
    "mmad_linear_gap_bwd": (_i32, [_i32, _i32, _i32, _i64, _vp, _vp, _vp, _vp, _i32, _vp, _vp,
                                   _vp, _vp]),
    "mmad_linear_fwd": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _vp]),
    "mmad_linear_bwd": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mmad_linear_bwd_ex": (_i32, [_i32, _i32, _i32] + [_vp] * 8),
    "mmad_concat_cols": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp]),
    "mmad_split_cols": (_i32, [_i32, _i32, _vp, _vp, _vp, _vp]),
    "mmad_cast": (_i32, [_i32, _i32, _i64, _vp, _vp, _vp]),
    "mmad_dropout_fwd": (_i32, [_i32, _i64, _f32, _u64, _vp, _vp, _vp, _vp]),
    "mmad_dropout_fwd_dev": (_i32, [_i32, _i64, _f32, _vp, _vp, _vp, _vp, _vp]),
    "mmad_dropout_bwd": (_i32, [_i32, _i64, _f32, _vp, _vp, _vp, _vp]),
    "mmad_loss_fwd": (_i32, [_i32, _i32, _vp, _vp, _vp, _f64, _i32, _vp, _vp, _vp]),
    "mmad_loss_fwd_ex": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp, _f64, _i32, _vp, _vp, _vp,
                                _vp]),
    "mmad_loss_bwd": (_i32, [_i64, _vp, _vp, _vp, _i32, _vp, _vp]),
    "mmad_gather_channels": (_i32, [_i32, _i32, _vp, _i64, _i64, _i32, _i64, _i32, _i32, _vp,
                                    _vp]),
    "mmad_pad_rows": (_i32, [_i32, _i32, _i32, _vp, _vp, _vp]),
    "mmad_concat_channels": (_i32, [_i32, _i64, _i32, _vp, _i32, _vp, _vp, _vp]),
    "mmad_split_channels": (_i32, [_i32, _i64, _i32, _i32, _vp, _vp, _vp, _vp]),
    "mmad_max2_fwd": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "mmad_max2_bwd": (_i32, [_i32, _i64, _vp, _vp, _vp, _vp, _vp]),
    "mmad_bootstrap_cls_metrics": (_i32, [_i32, _i32, _vp, _vp, _i32, _vp, _vp, _vp, _vp]),
    "mmad_mean_std": (_i32, [_i32, _vp, _vp, _vp]),
    "mmad_bn_relu_bwd_reduce": (_i32, [_i32, _i64, _i32] + [_vp] * 8),
    "mmad_bn_relu_bwd_apply": (_i32, [_i32, _i64, _i32] + [_vp] * 9),
}
EXPORTS = tuple(_SIGS)

_lib = None


class MMADError(RuntimeError):
    pass


def load():
    """Load (once) and return the CDLL; raises if the library has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MMADError(f"{LIB_PATH} is missing: build it with "
                            "`python -m multimodal_alzheimer_amd._build` (hipcc, gfx950)")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        if lib.mmad_abi_version() != 1:
            raise MMADError("libmmad_hip.so ABI version mismatch")
        _lib = lib
    return _lib


def check(rc, what=""):
    if rc == 0:
        return
    msg = load().mmad_strerror(rc).decode()
    if rc == EHIP + _HIP_OOM:
        raise torch.OutOfMemoryError(f"{what}: {msg}")
    raise MMADError(f"{what} failed ({rc}): {msg}")


def call(name, *args):
    check(getattr(load(), name)(*args), name)


_cur_dev = torch._C._cuda_getDevice
_raw_stream = torch._C._cuda_getCurrentRawStream


def stream():
    """the current HIP stream of the current device, as an address (the per-call cost of
    torch.cuda.current_stream()'s Stream object was a visible share of the step's host time)"""
    return _raw_stream(_cur_dev())


def ptr(t):
    if t is None:
        return None
    return t.data_ptr()


def dtype_code(dt):
    if dt == torch.float32:
        return F32
    if dt == torch.bfloat16:
        return BF16
    if dt == torch.float64:
        return F64
    raise MMADError(f"unsupported dtype {dt}")


def require_device(*tensors):
    for t in tensors:
        if t is not None and t.device.type != "cuda":
            raise MMADError("the MI355X hot path runs on HIP devices only "
                            f"(got a tensor on {t.device}); move the model and batch to "
                            "'cuda' -- there is no CPU fallback")

