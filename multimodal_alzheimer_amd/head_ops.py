"""Autograd ops of the classifier / late-fusion head and the losses (libmmad_hip.so).

Reference ops replaced:
  linear          nn.Linear            anat_cnn.py:68-76; anat_pet_fusion.py:42-51
  concat_features torch.cat(dim=1)     anat_pet_fusion.py:76; all_modalities_fusion.py:77
  dropout         nn.Dropout           pet_cnn.py:27-29, :38-39
  focal / CE loss FocalLoss, nn.CrossEntropyLoss(weight)   focalloss.py:19-39; anat_cnn.py:81-85
"""
import ctypes as C

import torch

from . import _lib as L
from . import volume_ops as V
from .volume_ops import cast, grad_slot


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        L.require_device(x, weight)
        if x.dtype != torch.float32:
            x = cast(x, torch.float32)
        x = x.contiguous()
        b, n_in = x.shape
        n_out = weight.shape[0]
        w = weight.detach().contiguous()
        bb = None if bias is None else bias.detach().contiguous()
        y = torch.empty((b, n_out), dtype=torch.float32, device=x.device)
        L.call("mmad_linear_fwd", b, n_in, n_out, L.ptr(x), L.ptr(w), L.ptr(bb), int(relu),
               L.ptr(y), L.stream())
        ctx.save_for_backward(x, weight, y if relu else None)
        ctx.has_bias = bias is not None
        ctx.relu = relu
        ctx.params = (weight, bias)        # gradient-slot lookup (volume_ops.grad_slot)
        return y

    @staticmethod
    def backward(ctx, g):
        x, weight, y = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = cast(g, torch.float32)
        b, n_in = x.shape
        n_out = weight.shape[0]
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
        need_w = ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2])
        if need_w:
            dw = grad_slot(ctx.params[0], tuple(weight.shape), g.device)
            if ctx.has_bias:
                db = grad_slot(ctx.params[1], (n_out,), g.device)
        # one launch: dx and dW / dbias, the fused ReLU's mask taken from the saved output
        L.call("mmad_linear_bwd_ex", b, n_in, n_out, L.ptr(x), L.ptr(weight.detach()), L.ptr(g),
               L.ptr(y if ctx.relu else None), L.ptr(dx), L.ptr(dw), L.ptr(db), L.stream())
        return dx, (dw if ctx.needs_input_grad[1] else None), db, None


def linear(x, weight, bias=None, relu=False):
    return _LinearFn.apply(x, weight, bias, bool(relu))


class _GapLinearFn(torch.autograd.Function):
    """conv_seg's AdaptiveAvgPool3d(1) -> Flatten -> Linear (-> ReLU) (anat_cnn.py:66-76):
    forward = the GAP's partial sums + one launch folding them into the pooled rows and
    applying the linear (mmad_gap_linear_fwd); backward = one launch for dW, dbias and the
    input gradient as the GAP's compact broadcast rows (mmad_linear_gap_bwd).  Same values
    as volume_ops.global_avg_pool + flatten + linear, two launches fewer."""

    @staticmethod
    def forward(ctx, x, weight, bias, relu):
        V._check_vol(x)
        lib = L.load()
        n, c = x.shape[:2]
        s = x.numel() // (n * c)
        parts = lib.mmad_gap_parts(n, s, c)
        ws = torch.empty(lib.mmad_gap_fwd_ws_elems(n, s, c), dtype=torch.float32,
                         device=x.device)
        L.call("mmad_gap_partial", L.dtype_code(x.dtype), n, s, c, L.ptr(x), L.ptr(ws),
               L.stream())
        n_out = weight.shape[0]
        w = weight.detach().contiguous()
        bb = None if bias is None else bias.detach().contiguous()
        xs = torch.empty((n, c), dtype=torch.float32, device=x.device)
        y = torch.empty((n, n_out), dtype=torch.float32, device=x.device)
        L.call("mmad_gap_linear_fwd", n, c, n_out, parts, s, L.ptr(ws), L.ptr(w), L.ptr(bb),
               int(relu), L.ptr(xs), L.ptr(y), L.stream())
        ctx.save_for_backward(xs, weight, y if relu else None)
        ctx.has_bias = bias is not None
        ctx.relu = relu
        ctx.params = (weight, bias)
        ctx.shape, ctx.dtype, ctx.s = tuple(x.shape), x.dtype, s
        return y

    @staticmethod
    def backward(ctx, g):
        xs, weight, y = ctx.saved_tensors
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = cast(g, torch.float32)
        n, c = xs.shape
        n_out = weight.shape[0]
        rows = dw = db = None
        if ctx.needs_input_grad[0]:
            rows = torch.empty((n, c), dtype=ctx.dtype, device=g.device)
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            dw = grad_slot(ctx.params[0], tuple(weight.shape), g.device)
            if ctx.has_bias:
                db = grad_slot(ctx.params[1], (n_out,), g.device)
        L.call("mmad_linear_gap_bwd", n, c, n_out, ctx.s, L.ptr(xs), L.ptr(weight.detach()),
               L.ptr(g), L.ptr(y if ctx.relu else None), L.dtype_code(ctx.dtype), L.ptr(rows),
               L.ptr(dw), L.ptr(db), L.stream())
        dx = None if rows is None else rows.view(n, c, 1, 1, 1).expand(ctx.shape)
        return dx, (dw if ctx.needs_input_grad[1] else None), db, None


def gap_linear(x, weight, bias=None, relu=False):
    """linear(flatten(global_avg_pool(x)), weight, bias, relu) for an NDHWC volume x whose
    GAP gradient may be handed on as broadcast rows (volume_ops.GAP_BCAST)."""
    return _GapLinearFn.apply(x, weight, bias, bool(relu))


class _ConcatFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, *xs):
        L.require_device(*xs)
        xs = [x if x.dtype == torch.float32 else cast(x, torch.float32) for x in xs]
        xs = [x.contiguous() for x in xs]
        b = xs[0].shape[0]
        widths = [int(x.shape[1]) for x in xs]
        y = torch.empty((b, sum(widths)), dtype=torch.float32, device=xs[0].device)
        srcs = (C.c_void_p * len(xs))(*[x.data_ptr() for x in xs])
        ws = (C.c_int * len(xs))(*widths)
        L.call("mmad_concat_cols", b, len(xs), srcs, ws, L.ptr(y), L.stream())
        ctx.widths = widths
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        b = g.shape[0]
        outs = [torch.empty((b, w), dtype=torch.float32, device=g.device) for w in ctx.widths]
        dsts = (C.c_void_p * len(outs))(*[o.data_ptr() for o in outs])
        ws = (C.c_int * len(outs))(*ctx.widths)
        L.call("mmad_split_cols", b, len(outs), L.ptr(g), dsts, ws, L.stream())
        return tuple(outs)


def concat_features(*xs):
    """torch.cat(xs, dim=1) for (B, w_k) float32 feature rows."""
    if len(xs) > 8:
        raise L.MMADError("concat_features supports at most 8 inputs")
    return _ConcatFn.apply(*xs)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p):
        L.require_device(x)
        dense = x.is_contiguous() or (x.dim() == 5 and
                                      x.is_contiguous(memory_format=torch.channels_last_3d))
        if not dense:
            x = x.contiguous()
        y = torch.empty_like(x)
        keep = torch.empty(x.numel(), dtype=torch.uint8, device=x.device)
        # the seed is drawn on the device from torch's CUDA generator and read by the kernel
        # when it runs: reproducible under torch.manual_seed, never synchronises, and graph
        # safe (a captured draw advances the generator's Philox offset on every replay, so a
        # replayed step gets a fresh mask instead of the one baked in at capture)
        seed = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64, device=x.device)
        L.call("mmad_dropout_fwd_dev", L.dtype_code(x.dtype), x.numel(), float(p), L.ptr(seed),
               L.ptr(x), L.ptr(y), L.ptr(keep), L.stream())
        ctx.save_for_backward(keep)
        ctx.p = p
        ctx.like = y
        return y

    @staticmethod
    def backward(ctx, g):
        (keep,) = ctx.saved_tensors
        g = g.contiguous(memory_format=torch.channels_last_3d) if g.dim() == 5 and \
            ctx.like.is_contiguous(memory_format=torch.channels_last_3d) else g.contiguous()
        dx = torch.empty_like(g)
        L.call("mmad_dropout_bwd", L.dtype_code(g.dtype), g.numel(), float(ctx.p), L.ptr(g),
               L.ptr(keep), L.ptr(dx), L.stream())
        return dx, None


def dropout(x, p, training):
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        raise L.MMADError("dropout p must be < 1")
    return _DropoutFn.apply(x, float(p))


class _LossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, weight, gamma, mode):
        L.require_device(logits, target)
        x = logits.contiguous()
        if x.dtype != torch.float64:
            x = cast(x, torch.float64)
        t = target.contiguous().to(torch.int64) if target.dtype != torch.int64 else \
            target.contiguous()
        b, c = x.shape
        w = None if weight is None else weight.detach().to(torch.float64).contiguous()
        loss = torch.empty((), dtype=torch.float64, device=x.device)
        dx = torch.empty_like(x)
        L.call("mmad_loss_fwd", b, c, L.ptr(x), L.ptr(t), L.ptr(w), float(gamma), int(mode),
               L.ptr(loss), L.ptr(dx), L.stream())
        ctx.save_for_backward(dx)
        ctx.in_dtype = logits.dtype
        return loss

    @staticmethod
    def backward(ctx, g):
        (dx,) = ctx.saved_tensors
        grad = dx * g          # (B, C) x 0-d scale: trivial glue, stays on device
        if ctx.in_dtype != torch.float64:
            grad = cast(grad, ctx.in_dtype)
        return grad, None, None, None, None


class _LogitsLossFn(torch.autograd.Function):
    """(logits as f64, loss(f64 logits, target)): general_step's f64 cast of the model output
    (anat_cnn.py:102-104) and the loss in one launch (mmad_loss_fwd_ex); backward: the loss
    gradient times the incoming scalar, plus the f64 logits' own gradient if any, cast back
    to the logits' dtype in one launch (mmad_loss_bwd).  Same values as cast + _LossFn."""

    @staticmethod
    def forward(ctx, logits, target, weight, gamma, mode):
        L.require_device(logits, target)
        x = logits.contiguous()
        t = target.contiguous().to(torch.int64) if target.dtype != torch.int64 else \
            target.contiguous()
        b, c = x.shape
        w = None if weight is None else weight.detach().to(torch.float64).contiguous()
        y64 = torch.empty((b, c), dtype=torch.float64, device=x.device)
        loss = torch.empty((), dtype=torch.float64, device=x.device)
        dx = torch.empty_like(y64)
        L.call("mmad_loss_fwd_ex", b, c, L.dtype_code(x.dtype), L.ptr(x), L.ptr(t), L.ptr(w),
               float(gamma), int(mode), L.ptr(y64), L.ptr(loss), L.ptr(dx), L.stream())
        ctx.save_for_backward(dx)
        ctx.in_dtype = logits.dtype
        ctx.set_materialize_grads(False)
        return y64, loss

    @staticmethod
    def backward(ctx, g_y64, g_loss):
        if g_loss is None:
            return (None if g_y64 is None else cast(g_y64.contiguous(), ctx.in_dtype),
                    None, None, None, None)
        (dx,) = ctx.saved_tensors
        gl = g_loss.detach().to(torch.float64).contiguous()
        go = None if g_y64 is None else g_y64.detach().to(torch.float64).contiguous()
        out = torch.empty(dx.shape, dtype=ctx.in_dtype, device=dx.device)
        L.call("mmad_loss_bwd", dx.numel(), L.ptr(dx), L.ptr(gl), L.ptr(go),
               L.dtype_code(ctx.in_dtype), L.ptr(out), L.stream())
        return out, None, None, None, None


def logits_and_loss(logits, target, weight, gamma, mode):
    """(logits.to(float64), loss) for (B, C) fp32 / f64 logits: mode 0 weighted CE with
    ``weight``, mode 1 focal with ``gamma`` (see _LogitsLossFn)."""
    if logits.dim() != 2 or logits.dtype not in (torch.float32, torch.float64):
        raise L.MMADError("logits_and_loss expects (B, C) fp32 / f64 logits")
    return _LogitsLossFn.apply(logits, target.reshape(-1), weight, float(gamma), int(mode))


def weighted_cross_entropy(logits, target, weight=None):
    """nn.CrossEntropyLoss(weight)(logits, target), 'mean' reduction (anat_cnn.py:84-85)."""
    if logits.dim() != 2:
        raise L.MMADError("cross entropy expects (B, C) logits")
    return _LossFn.apply(logits, target, weight, 0.0, 0)


def focal_loss(logits, target, gamma):
    """FocalLoss(gamma)(logits, target): alpha None, mean, pt detached (focalloss.py:19-39)."""
    if logits.dim() > 2:
        n, c = logits.shape[:2]
        logits = logits.reshape(n, c, -1).transpose(1, 2).reshape(-1, c)
    return _LossFn.apply(logits, target.reshape(-1), None, float(gamma), 1)


def bootstrap_cls_metrics(logits, labels, idx):
    """Per-drawing (macro F1, MCC) of argmax(logits[idx[d]]) vs labels[idx[d]] for every
    drawing d (Base_Model.bootstrap_metric, base_model.py:219-239), one block per drawing.
    Returns two float32 device tensors of length idx.shape[0]."""
    L.require_device(logits, labels)
    x = logits.detach()
    if x.dtype != torch.float64:
        x = cast(x, torch.float64)
    x = x.contiguous()
    y = labels.contiguous().to(torch.int64)
    ix = idx.to(device=x.device, dtype=torch.int64).contiguous()
    nd, n = ix.shape
    f1 = torch.empty(nd, dtype=torch.float32, device=x.device)
    mcc = torch.empty_like(f1)
    L.call("mmad_bootstrap_cls_metrics", n, x.shape[1], L.ptr(x), L.ptr(y), nd, L.ptr(ix),
           L.ptr(f1), L.ptr(mcc), L.stream())
    return f1, mcc


def mean_std(v):
    """(mean, unbiased std) of a float32 device vector, f64 accumulation."""
    out = torch.empty(2, dtype=torch.float64, device=v.device)
    L.call("mmad_mean_std", v.numel(), L.ptr(v.contiguous()), L.ptr(out), L.stream())
    return out
