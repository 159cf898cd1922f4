"""Autograd ops over NDHWC volumes, each a thin call into libmmad_hip.so.

A volume tensor is a logical (N, C, D, H, W) torch tensor in ``torch.channels_last_3d``
memory format -- exactly the NDHWC layout the kernels use -- so any torch code that
inspects shapes sees the reference's NCDHW semantics.  Compute dtype is float32
(parity mode, exact-f32 MFMA) or bfloat16 (throughput mode, f32 accumulation).

Reference ops replaced (file:line in the reference tree):
  conv3d          nn.Conv3d            MedicalNet convs via anat_cnn.py:29-31; pet_cnn.py:20-22
  batchnorm_act   nn.BatchNorm3d/1d + nn.ReLU (+ residual add)  MedicalNet BasicBlock;
                                       anat_cnn.py:50-51, :69-70; pet_cnn.py:23-25
  max_pool3d      nn.MaxPool3d         MedicalNet stem; anat_cnn.py:62; pet_cnn.py:26
  global_avg_pool nn.AdaptiveAvgPool3d(1)  anat_cnn.py:66; pet_cnn.py:33
"""
import ctypes as C
import os
import weakref

import torch

from . import _lib as L

CL = torch.channels_last_3d


def _cl(t):
    """dense NDHWC view of a volume gradient (no copy when already channels-last)."""
    if t.dim() == 5:
        return t.contiguous(memory_format=CL)
    return t.contiguous()


def _empty_vol(n, c, d, h, w, dtype, device):
    return torch.empty((n, c, d, h, w), dtype=dtype, device=device, memory_format=CL)


def _check_vol(x, dtype=None):
    L.require_device(x)
    if x.dim() != 5 or not x.is_contiguous(memory_format=CL):
        raise L.MMADError("volume tensors must be 5-D channels_last_3d (NDHWC)")
    if dtype is not None and x.dtype != dtype:
        raise L.MMADError(f"expected {dtype}, got {x.dtype}")
    if x.data_ptr() % 16:
        raise L.MMADError("volume tensors must be 16-byte aligned")


# ---------------------------------------------------------------------------------- conv
def out_extent(i, k, s, p, d):
    return (i + 2 * p - d * (k - 1) - 1) // s + 1


def conv_desc(xshape, wshape, stride, padding, dilation):
    n, ci, di, hi, wi = xshape
    co, ci_w, kd, kh, kw = wshape
    if ci_w != ci:
        raise L.MMADError(f"conv3d: input has {ci} channels, weight expects {ci_w}")
    sd, sh, sw = stride
    pd, ph, pw = padding
    dd, dh, dw = dilation
    return L.ConvDesc(n, ci, di, hi, wi, co, out_extent(di, kd, sd, pd, dd),
                      out_extent(hi, kh, sh, ph, dh), out_extent(wi, kw, sw, pw, dw),
                      kd, kh, kw, sd, sh, sw, pd, ph, pw, dd, dh, dw)


def _desc_tuple(d):
    return tuple(getattr(d, f) for f, _ in L.ConvDesc._fields_)


# Live kernel timing: map a conv descriptor tuple to a list; every forward launch with that
# geometry appends a (start, end) HIP event pair recorded on the launch stream around it.
FWD_PROBES = {}
# the same for the weight gradient (the event pair brackets the whole mmad_conv3d_wgrad call:
# the MFMA kernel and its slab reduce)
WGRAD_PROBES = {}

# Deferred weight-gradient slab reductions (round 5).  Inside ``deferred_wgrad_reduce()`` a
# conv weight gradient whose dW autograd adopts as-is (no existing .grad, no bias, no channel
# padding) runs only its split-K kernel (mmad_conv3d_wgrad_deferred) and queues its slab
# reduction; ``flush_wgrad_reduce()`` then runs every queued reduction as ONE launch
# (mmad_wgrad_reduce_batch, bit-identical sums).  graph_step captures the backward this way
# and flushes at its end (per stage when staged), so the replay has one reduction launch
# instead of one per conv.  Nothing may read a queued dW before the flush: eager backward
# hooks that all-reduce buckets keep it off, a weight with tensor / post-accumulate hooks is
# never deferred, and every deferred dW must end up as its parameter's ``.grad`` itself
# (``check_deferred_adoption``: an AccumulateGrad that cloned it, or a second contribution
# summed into it, would have read it before the flush -- that raises).
_WGRAD_DEFER = {"on": False, "jobs": [], "keep": [], "adopt": []}
# MMAD_REDUCE_EACH=1 (diagnostic): the queued reductions run one launch per job, so a kernel
# trace times each conv's share of the batched reduction
_REDUCE_EACH = os.environ.get("MMAD_REDUCE_EACH", "0") == "1"


def _deferrable(wparam):
    """a weight gradient may queue its slab reduction: the weight is a leaf parameter with
    no gradient yet and no hook that would read dW during the backward, and the wgrad runs
    on the main stream (MMAD_WGRAD_STREAM keeps deferral off: the flush runs on the main
    stream, the workspace would belong to the side stream)"""
    if not _WGRAD_DEFER["on"] or WGRAD_STREAM or wparam is None or not wparam.is_leaf:
        return False
    if wparam.grad is not None or getattr(wparam, "_backward_hooks", None):
        return False
    return not getattr(wparam, "_post_accumulate_grad_hooks", None)


def check_deferred_adoption():
    """Every weight whose dW reduction was deferred holds that very tensor as ``.grad`` (host
    side, pointer compare).  Anything else means a copy or a sum read dW before the flush."""
    pending = _WGRAD_DEFER["adopt"]
    bad = [p for p, ptr in pending if p.grad is None or p.grad.data_ptr() != ptr]
    pending.clear()
    if bad:
        raise RuntimeError(
            f"{len(bad)} deferred weight gradient(s) were not adopted as .grad as-is (copied "
            f"or summed before the batched slab reduction ran); shapes "
            f"{[tuple(p.shape) for p in bad[:4]]}.  Run with MMAD_DEFER_WGRAD=0.")


class deferred_wgrad_reduce:
    """context manager: queue the weight-gradient slab reductions (see above)"""

    def __init__(self, on=True):
        self.on = on

    def __enter__(self):
        self.prev = _WGRAD_DEFER["on"]
        _WGRAD_DEFER["on"] = self.on
        return self

    def __exit__(self, *exc):
        flush_wgrad_reduce()
        _WGRAD_DEFER["on"] = self.prev
        if exc[0] is None:
            check_deferred_adoption()
        else:
            _WGRAD_DEFER["adopt"].clear()
        return False


def flush_wgrad_reduce():
    """run every queued weight-gradient slab reduction (one launch per 16) on the current
    stream"""
    jobs = _WGRAD_DEFER["jobs"]
    if not jobs:
        return
    if _REDUCE_EACH:                       # diagnostic: one launch per job (per-job timing)
        for j in jobs:
            one = (L.WgradJob * 1)(j)
            L.call("mmad_wgrad_reduce_batch", 1, one, L.stream())
    else:
        arr = (L.WgradJob * len(jobs))(*jobs)
        L.call("mmad_wgrad_reduce_batch", len(jobs), arr, L.stream())
    # (stream-ordered: the workspaces return to the caching allocator only for work queued
    # after this launch)
    jobs.clear()
    _WGRAD_DEFER["keep"].clear()


# training-mode BN statistic updates so far (the running buffers are written by our kernels,
# which torch's tensor version counters do not see); keys the eval-mode folded-weight caches
_BN_UPDATES = [0]

# Weight gradients run on a second HIP stream: nothing downstream in the backward pass needs
# dW, so each conv's wgrad (+ split-K reduce) overlaps the dgrad -> BN-backward chain that
# is the backward's critical path, filling the machine during its small launches.  The
# main stream joins the side stream once, at the end of the backward pass (an autograd
# engine callback), before anything (optimizer, gradient all-reduce) reads a dW.
# Measured 2 % SLOWER on the ResNet-10 step (1564 vs 1598 vol/s, MI355X): the side-stream
# wgrad blocks take CUs from the one-block-per-CU dgrad tiles on the critical path.  So it
# is off unless MMAD_WGRAD_STREAM=1 (A/B switch); the gradient all-reduce still uses the
# side stream (data_parallel.GradAllReduce).
WGRAD_STREAM = os.environ.get("MMAD_WGRAD_STREAM", "0") == "1"
# MMAD_REDUCE_STREAM=1: only the split-K slab REDUCTION of each weight gradient goes to the
# side stream (the wgrad kernel stays on the main stream), to overlap the latency-bound BN
# backward kernels that follow (mmad_conv3d_wgrad_split).  The same side stream carries the
# data-parallel all-reduce, so it stays ordered after every reduction it reads; the main
# stream joins it at the end of backward.  Measured 2 % SLOWER on the ResNet-10 step
# (2148-2167 vs 2196-2205 vol/s, interleaved on one MI355X): the reduction blocks wait for
# CU slots behind the one-block-per-CU conv kernels and then delay the next one.  Off.
REDUCE_STREAM = os.environ.get("MMAD_REDUCE_STREAM", "0") == "1"
# MMAD_STEM_RAW=0: the Cin-1 stem reads the W-unfolded copy written by
# mmad_conv_unfold_input instead of the raw volume (A/B switch; mmad_conv3d_fwd_raw)
STEM_RAW = os.environ.get("MMAD_STEM_RAW", "1") != "0"
_SIDE = {}
_JOIN_PENDING = set()


def grad_stream(device):
    """The side stream weight gradients are produced on (one per device)."""
    s = _SIDE.get(device)
    if s is None:
        s = _SIDE[device] = torch.cuda.Stream(device=device)
    return s


def _queue_join(main, side):
    key = (main.cuda_stream, side.cuda_stream)
    if key in _JOIN_PENDING:
        return
    _JOIN_PENDING.add(key)

    def join():
        _JOIN_PENDING.discard(key)
        main.wait_stream(side)

    torch.autograd.Variable._execution_engine.queue_callback(join)


def grad_slot(param, shape, device):
    """Destination for a parameter's gradient: a fresh alias of its data-parallel bucket
    slice (``_mmad_grad_view``, set by data_parallel.GradAllReduce) while the parameter has
    no gradient yet -- autograd then adopts it as ``.grad`` and the all-reduce needs no
    gather -- else a new fp32 tensor."""
    slot = getattr(param, "_mmad_grad_view", None) if param is not None else None
    if slot is not None and param.grad is None and tuple(slot.shape) == tuple(shape):
        return slot.view(slot.shape)
    return torch.empty(shape, dtype=torch.float32, device=device)


def pack_weight(d, dt_code, weight, cdtype, for_dgrad):
    lib = L.load()
    n = lib.mmad_conv_packed_elems(d, dt_code, int(for_dgrad))
    if n < 0:
        raise L.MMADError("conv3d: unsupported geometry")
    wp = torch.empty(n, dtype=cdtype, device=weight.device)
    L.call("mmad_conv_pack_weight", d, dt_code, L.ptr(weight.detach().contiguous()), L.ptr(wp),
           int(for_dgrad), L.stream())
    return wp


def _weight_desc(weight, stride, padding, dilation):
    """a descriptor for packing only: the packed layouts depend on the weight shape and the
    conv's stride/padding/dilation, not on the volume extent, so any consistent extent does."""
    co, ci, kd, kh, kw = weight.shape
    ext = [max(16, (k - 1) * d + 1) for k, d in zip((kd, kh, kw), dilation)]
    return conv_desc((1, ci, *ext), tuple(weight.shape), stride, padding, dilation)


class PackPlan:
    """Repack a set of conv weights (forward layout, and the dgrad layout when gradients
    are on) with one or two kernel launches per step instead of one or two per conv: bf16
    convs needing both layouts get them from a single read (mmad_conv_pack_dual_batch),
    the rest go through the generic job batch.

    ``convs``: layers.Conv3d modules sharing one compute dtype.  ``run()`` refreshes every
    packed copy from the current fp32 master weights and hands each conv its buffers for
    its next forward (``conv._prepacked``).  Convs the batched kernel does not cover (a
    ci == 1 stem, padded K rows) keep packing per call."""

    def __init__(self, convs, cdtype, with_dgrad):
        lib = L.load()
        dt = L.dtype_code(cdtype)
        self.cdtype, self.dt = cdtype, dt
        self.entries = []
        jobs = []
        tiles = 0
        duals = []
        dtiles = 0
        self.unfolds = []        # (weight, desc, forward buffer) of Cin = 1 stems
        for conv in convs:
            w = conv.weight
            d = _weight_desc(w, conv._stride3(), conv._pads(), conv._dilation3())
            if d.ci == 1 and cdtype == torch.bfloat16:
                # the stem's unfolded forward layout: packed here (one launch, as per call
                # before) so a fused optimizer step can produce it instead (fused_optim)
                wp = torch.empty(lib.mmad_conv_packed_elems(d, dt, 0), dtype=cdtype,
                                 device=w.device)
                self.unfolds.append((w, d, wp))
                self.entries.append((conv, w.data_ptr(), wp, None))
                continue
            if with_dgrad and cdtype == torch.bfloat16:
                # both layouts from one read of the fp32 weight when the shapes allow it
                nf = lib.mmad_conv_packed_elems(d, dt, 0)
                nd = lib.mmad_conv_packed_elems(d, dt, 1)
                if nf > 0 and nd > 0:
                    wp = torch.empty(nf, dtype=cdtype, device=w.device)
                    wpt = torch.empty(nd, dtype=cdtype, device=w.device)
                    job = L.PackDual()
                    if lib.mmad_conv_pack_dual_job(d, dt, L.ptr(w), L.ptr(wp), L.ptr(wpt),
                                                   dtiles, job) == 0:
                        dtiles += lib.mmad_pack_dual_tiles(job)
                        duals.append(job)
                        self.entries.append((conv, w.data_ptr(), wp, wpt))
                        continue
            bufs = []
            for fd in ((0, 1) if with_dgrad else (0,)):
                n = lib.mmad_conv_packed_elems(d, dt, fd)
                wp = torch.empty(max(n, 0), dtype=cdtype, device=w.device)
                job = L.PackJob()
                rc = lib.mmad_conv_pack_job(d, dt, fd, L.ptr(w), L.ptr(wp), tiles, job)
                if rc != 0:
                    bufs.append(None)
                    continue
                tiles += lib.mmad_pack_job_tiles(job)
                jobs.append(job)
                bufs.append(wp)
            if not with_dgrad:
                bufs.append(None)
            self.entries.append((conv, w.data_ptr(), bufs[0], bufs[1]))
        self.njobs, self.tiles = len(jobs), tiles
        if jobs:
            raw = (L.PackJob * len(jobs))(*jobs)
            host = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
            self.table = host.to(convs[0].weight.device)
        self.nduals, self.dtiles = len(duals), dtiles
        self.duals = duals
        # external: the dual repack is produced elsewhere (fused_optim.AdamRepack writes it
        # at the end of the previous captured step), so run() skips that launch
        self.external = False
        if duals:
            raw = (L.PackDual * len(duals))(*duals)
            host = torch.frombuffer(bytearray(bytes(raw)), dtype=torch.uint8)
            self.dtable = host.to(convs[0].weight.device)
        self.with_dgrad = with_dgrad

    def valid_for(self, convs, cdtype, with_dgrad):
        return (cdtype == self.cdtype and with_dgrad == self.with_dgrad and
                len(convs) == len(self.entries) and
                all(c is e[0] and c.weight.data_ptr() == e[1]
                    for c, e in zip(convs, self.entries)))

    def run(self):
        if self.njobs:
            L.call("mmad_conv_pack_batch", self.dt, self.njobs, L.ptr(self.table), self.tiles,
                   L.stream())
        if not self.external:
            self.run_duals()
        for conv, _, wp, wpt in self.entries:
            conv._prepacked = (wp, wpt) if wp is not None or wpt is not None else None


    def run_duals(self):
        """the repacks a fused optimizer step can take over (dual layouts, unfolded stems)"""
        if self.nduals:
            L.call("mmad_conv_pack_dual_batch", self.dt, self.nduals, L.ptr(self.dtable),
                   self.dtiles, L.stream())
        for w, d, wp in self.unfolds:
            L.call("mmad_conv_pack_weight", d, self.dt, L.ptr(w.detach()), L.ptr(wp), 0,
                   L.stream())


def prepack(module, convs=None):
    """Batched weight repack for every layers.Conv3d under ``module`` (see PackPlan)."""
    from .layers import Conv3d
    if convs is None:
        convs = [m for m in module.modules() if isinstance(m, Conv3d) and m.weight.is_cuda]
    if not convs:
        return
    cdtype = convs[0].compute_dtype
    convs = [c for c in convs if c.compute_dtype == cdtype and
             (c.weight.shape[1] == 1 or c.weight.shape[1] % 8 == 0)]  # Cin 2..7: padded per call
    with_dgrad = torch.is_grad_enabled()
    plan = getattr(module, "_mmad_pack_plan", None)
    if plan is None or not plan.valid_for(convs, cdtype, with_dgrad):
        plan = PackPlan(convs, cdtype, with_dgrad)
        module._mmad_pack_plan = plan
    plan.run()


class StackedVolumes:
    """``torch.stack(srcs, dim=1)`` of raw single-channel volumes, not materialised.

    PET_MRI_EF stacks the PET and MRI volumes into a 2-channel input
    (pkg/models/fusion_models/early_fusion.py:77-80); the first conv gathers the planes
    straight into its channel-padded NDHWC operand (mmad_gather_channels), so the stacked
    f64 tensor and its f32 copy never exist.  Also accepts one (B, C, D, H, W) tensor with
    C < 8 (any layout whose D, H, W collapse to one voxel stride)."""

    def __init__(self, srcs):
        if isinstance(srcs, torch.Tensor):
            x = srcs
            n, c, di, hi, wi = x.shape
            s = x.stride()
            if not (s[3] == wi * s[4] and s[2] == hi * s[3]):
                x = x.contiguous()
                s = x.stride()
            es = x.element_size()
            self.ptrs = [x.data_ptr() + ch * s[1] * es for ch in range(c)]
            self.bstride, self.vstride = s[0], s[4]
            self._keep = [x]
        else:
            srcs = [t.contiguous() for t in srcs]
            x = srcs[0]
            if any(t.shape != x.shape or t.dtype != x.dtype or t.device != x.device
                   for t in srcs):
                raise L.MMADError("stacked volumes must share shape, dtype and device")
            if x.dim() != 4:
                raise L.MMADError("stack sources are (B, D, H, W) volumes")
            n, di, hi, wi = x.shape
            c = len(srcs)
            self.ptrs = [t.data_ptr() for t in srcs]
            self.bstride, self.vstride = di * hi * wi, 1
            self._keep = srcs
        if not 1 <= c <= 8:
            raise L.MMADError("at most 8 stacked channels")
        self.shape = torch.Size((n, c, di, hi, wi))
        self.dtype, self.device = x.dtype, x.device

    def dim(self):
        return 5

    def gather(self, cdtype):
        """The padded NDHWC compute-dtype operand: (N, 8, D, H, W) channels_last_3d."""
        n, c, di, hi, wi = self.shape
        out = _empty_vol(n, 8, di, hi, wi, cdtype, self.device)
        srcs = (C.c_void_p * c)(*self.ptrs)
        L.call("mmad_gather_channels", L.dtype_code(self.dtype), c, srcs, self.bstride,
               self.vstride, n, di * hi * wi, 8, L.dtype_code(cdtype), L.ptr(out), L.stream())
        return out


def _pad_rows(src, rows, cin, cout, shape):
    dst = torch.empty(shape, dtype=torch.float32, device=src.device)
    L.call("mmad_pad_rows", rows, cin, cout, L.ptr(src), L.ptr(dst), L.stream())
    return dst


class _Conv3dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, geom, cdtype, want_stats, packed=None):
        stride, padding, dilation = geom
        L.require_device(x, weight)
        if weight.dtype != torch.float32:
            raise L.MMADError("conv3d master weights must be float32")
        d = conv_desc(tuple(x.shape), tuple(weight.shape), stride, padding, dilation)
        dt = L.dtype_code(cdtype)
        lib = L.load()
        ctx.ci_real = d.ci
        wsrc = weight
        ctx.raw = None
        if isinstance(x, StackedVolumes) or (d.ci > 1 and d.ci % 8):
            # Cin in 2..7 (early fusion): channel-padded operand and weight (fusion.hip);
            # the zero lanes contribute exact zeros
            if ctx.needs_input_grad[0]:
                raise L.MMADError("conv3d: gradient w.r.t. a channel-stacked raw input is "
                                  "not supported (the input never needs one)")
            sv = x if isinstance(x, StackedVolumes) else StackedVolumes(x)
            if sv.shape[1] == 1:
                raise L.MMADError("a single raw volume goes to conv3d as a (B,1,D,H,W) tensor")
            taps = d.kd * d.kh * d.kw
            src = sv.gather(cdtype)
            wsrc = _pad_rows(weight.detach().contiguous(), d.co, d.ci * taps, 8 * taps,
                             (d.co, 8, d.kd, d.kh, d.kw))
            d.ci = 8
            packed = None
        elif d.ci == 1:
            if ctx.needs_input_grad[0]:
                raise L.MMADError("conv3d: gradient w.r.t. a 1-channel raw input volume "
                                  "is not supported (the input never needs one)")
            xc = x.contiguous()
            in_dt = L.dtype_code(xc.dtype)
            if STEM_RAW and lib.mmad_stem_raw_ok(d, in_dt, dt) == 1:
                # the stem kernels unfold the raw volume's rows themselves (no unfolded copy)
                src, ctx.raw = xc, in_dt
            else:
                src = torch.empty(lib.mmad_conv_unfolded_elems(d), dtype=cdtype,
                                  device=x.device)
                L.call("mmad_conv_unfold_input", d, in_dt, L.ptr(xc), dt, L.ptr(src),
                       L.stream())
        else:
            _check_vol(x, cdtype)
            src = x
        ctx.bnsum = None
        if BNSUM and _BNSUM_SRC and ctx.needs_input_grad[0] and cdtype == torch.bfloat16 \
                and isinstance(x, torch.Tensor):
            ctx.bnsum = _bnsum_source(x, d, dt)
        wp, wpt = packed if packed is not None else (None, None)
        if wp is None:
            wp = pack_weight(d, dt, wsrc, cdtype, False)
        y = _empty_vol(d.n, d.co, d.do_, d.ho, d.wo, cdtype, x.device)
        stats = None
        if want_stats:
            rows = lib.mmad_conv3d_stats_rows(d, dt)
            stats = torch.empty((rows, 2, d.co), dtype=torch.float32, device=x.device)
        b = None if bias is None else bias.detach().contiguous()
        probe = FWD_PROBES.get(_desc_tuple(d)) if FWD_PROBES else None
        if probe is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        if ctx.raw is not None:
            L.call("mmad_conv3d_fwd_raw", d, ctx.raw, L.ptr(src), dt, L.ptr(wp), L.ptr(b),
                   L.ptr(y), L.ptr(stats), L.stream())
        else:
            L.call("mmad_conv3d_fwd", d, dt, L.ptr(src), L.ptr(wp), L.ptr(b), L.ptr(y),
                   L.ptr(stats), L.stream())
        if probe is not None:
            e1.record()
            probe.append((e0, e1))
        ctx.save_for_backward(src, weight)
        ctx.wparam = weight                # the Parameter itself (gradient slot lookup)
        ctx.wpt = wpt                      # prepacked dgrad layout (or None: pack in bwd)
        ctx.set_materialize_grads(False)   # the stats output never gets a gradient
        ctx.desc = _desc_tuple(d)
        ctx.cdtype = cdtype
        ctx.has_bias = bias is not None
        ctx.xshape = tuple(x.shape)
        if want_stats:
            ctx.mark_non_differentiable(stats)
            return y, stats
        return y

    @staticmethod
    def backward(ctx, gy, *_):
        if gy is None:
            return None, None, None, None, None, None, None
        src, weight = ctx.saved_tensors
        d = L.ConvDesc(*ctx.desc)
        cdtype = ctx.cdtype
        dt = L.dtype_code(cdtype)
        gy = _cl(gy)
        if gy.dtype != cdtype:
            gy = cast(gy, cdtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            wpt = ctx.wpt if ctx.wpt is not None else pack_weight(d, dt, weight, cdtype, True)
            dx = _empty_vol(d.n, d.ci, d.di, d.hi, d.wi, cdtype, gy.device)
            if ctx.bnsum is not None:
                # the input's BN backward sums from the dgrad epilogue (see BNSUM above)
                yb, mu, ist, sc, sh = ctx.bnsum
                rows = L.load().mmad_conv3d_dgrad_bnsum_rows(d, dt)
                parts = torch.empty((rows, 2, d.ci), dtype=torch.float32, device=gy.device)
                L.call("mmad_conv3d_dgrad_bnsum", d, dt, L.ptr(gy), L.ptr(wpt), L.ptr(dx),
                       L.ptr(yb), L.ptr(sc), L.ptr(sh), L.ptr(mu), L.ptr(ist), L.ptr(parts),
                       L.stream())
                _BNSUM_PARTS[id(dx)] = (weakref.ref(dx), parts)
            else:
                L.call("mmad_conv3d_dgrad", d, dt, L.ptr(gy), L.ptr(wpt), L.ptr(dx),
                       L.stream())
        if ctx.needs_input_grad[1] or (ctx.has_bias and ctx.needs_input_grad[2]):
            main = torch.cuda.current_stream()
            side = grad_stream(gy.device) if WGRAD_STREAM else main
            if side is not main:
                side.wait_stream(main)          # gy (and src) complete
            with torch.cuda.stream(side):
                rside = grad_stream(gy.device) if REDUCE_STREAM and side is main else None
                dw, db = _wgrad(ctx, d, dt, src, gy, weight, ctx.wparam, rside)
            if side is not main:
                # memory first used on the side stream stays reserved until it is done
                for t in (src, gy, dw, db):
                    if t is not None:
                        t.record_stream(side)
                _queue_join(main, side)
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db, None, None, None, None


def _wgrad(ctx, d, dt, src, gy, weight, wparam=None, rside=None):
    """dW (torch layout, fp32) and the bias gradient of one conv, on the current stream
    (its slab reduction on ``rside`` when given: REDUCE_STREAM).
    When the weight parameter carries a gradient slot (``_mmad_grad_view``: its slice of
    a data-parallel bucket, data_parallel.GradAllReduce) and has no gradient yet, dW is
    written straight into it; autograd then adopts that tensor as ``.grad`` as-is."""
    lib = L.load()
    ws = torch.empty((lib.mmad_conv3d_wgrad_workspace(d, dt) + 3) // 4, dtype=torch.float32,
                     device=gy.device)
    padded = ctx.ci_real != d.ci
    slot = getattr(wparam, "_mmad_grad_view", None) if wparam is not None else None
    if slot is not None and not padded and wparam.grad is None and \
            slot.shape == weight.shape and slot.dtype == torch.float32:
        dw = slot.view(slot.shape)     # a fresh alias: autograd adopts it only if unshared
    else:
        dw = torch.empty((d.co, d.ci, d.kd, d.kh, d.kw) if padded else weight.shape,
                         dtype=torch.float32, device=gy.device)
    db = torch.empty(d.co, dtype=torch.float32, device=gy.device) if ctx.has_bias else None
    # a dW that autograd will not adopt as-is (an existing .grad it is added into, or the
    # channel-padded copy cut below) is read on the main stream: no split then
    raw = getattr(ctx, "raw", None)
    defer = not ctx.has_bias and not padded and _deferrable(wparam)
    if raw is not None and defer:
        job = L.WgradJob()
        L.call("mmad_conv3d_wgrad_raw_deferred", d, raw, L.ptr(src), dt, L.ptr(gy), L.ptr(dw),
               L.ptr(ws), C.byref(job), L.stream())
        if job.kind:
            _WGRAD_DEFER["jobs"].append(job)
            _WGRAD_DEFER["keep"].append(ws)
            # the address only: an extra reference to dW would make AccumulateGrad copy it
            _WGRAD_DEFER["adopt"].append((wparam, dw.data_ptr()))
    elif raw is not None:
        # the raw stem input (see _Conv3dFn.forward); slab reduction on rside when given
        split = rside is not None and (wparam is None or wparam.grad is None)
        L.call("mmad_conv3d_wgrad_raw", d, raw, L.ptr(src), dt, L.ptr(gy), L.ptr(dw),
               L.ptr(db), L.ptr(ws), L.stream(), rside.cuda_stream if split else None)
        if split:
            for t in (ws, gy, dw, db):
                if t is not None:
                    t.record_stream(rside)
            _queue_join(torch.cuda.current_stream(), rside)
    elif rside is not None and not padded and (wparam is None or wparam.grad is None):
        L.call("mmad_conv3d_wgrad_split", d, dt, L.ptr(src), L.ptr(gy), L.ptr(dw), L.ptr(db),
               L.ptr(ws), L.stream(), rside.cuda_stream)
        # what the side stream reads or writes stays allocated until it has run; dW (and
        # anything derived from it) is read only after the join
        for t in (ws, gy, dw, db):
            if t is not None:
                t.record_stream(rside)
        _queue_join(torch.cuda.current_stream(), rside)
    elif defer:
        job = L.WgradJob()
        L.call("mmad_conv3d_wgrad_deferred", d, dt, L.ptr(src), L.ptr(gy), L.ptr(dw), L.ptr(ws),
               C.byref(job), L.stream())
        if job.kind:
            _WGRAD_DEFER["jobs"].append(job)
            _WGRAD_DEFER["keep"].append(ws)
            # the address only: an extra reference to dW would make AccumulateGrad copy it
            _WGRAD_DEFER["adopt"].append((wparam, dw.data_ptr()))
    else:
        probe = WGRAD_PROBES.get(_desc_tuple(d)) if WGRAD_PROBES else None
        if probe is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        L.call("mmad_conv3d_wgrad", d, dt, L.ptr(src), L.ptr(gy), L.ptr(dw), L.ptr(db),
               L.ptr(ws), L.stream())
        if probe is not None:
            e1.record()
            probe.append((e0, e1))
    if padded:                             # cut the zero-lane channels back off
        taps = d.kd * d.kh * d.kw
        dw = _pad_rows(dw, d.co, d.ci * taps, ctx.ci_real * taps, weight.shape)
    return dw, db


def conv3d(x, weight, bias=None, stride=(1, 1, 1), padding=(0, 0, 0), dilation=(1, 1, 1),
           cdtype=torch.float32, want_stats=False, packed=None):
    """nn.functional.conv3d on NDHWC volumes; with want_stats also returns the BN partial
    sums ([rows][2][Co] fp32) of the output, produced by the conv epilogue.  ``packed``:
    (forward, dgrad) packed weights refreshed this step by PackPlan.run (either None)."""
    return _Conv3dFn.apply(x, weight, bias, (tuple(stride), tuple(padding), tuple(dilation)),
                           cdtype, want_stats, packed)


def conv_bn_act_eval(x, conv, bn, relu=True, res=None):
    """Eval-mode conv -> BN (running statistics) [-> + res] [-> ReLU] as ONE kernel: the BN
    scale is folded into the packed weights and its shift into the conv bias
    (mmad_bn_fold + mmad_conv_pack_weight_scaled), the residual add and ReLU run in the
    conv epilogue (mmad_conv3d_fwd_ex).  Inference only (no autograd).  Returns None when
    the layer is not eligible (Cin = 1 stem, batch-statistics BN, unsupported packing), so
    the caller falls back to the unfused ops."""
    if bn.training or bn.running_mean is None or torch.is_grad_enabled():
        return None
    cd = conv.compute_dtype
    if x.shape[1] == 1:
        return None
    if x.dtype != cd:
        x = _cast_raw(x, cd)
    _check_vol(x, cd)
    if res is not None:
        _check_vol(res, cd)
    lib = L.load()
    d = conv_desc(tuple(x.shape), tuple(conv.weight.shape), conv._stride3(), conv._pads(),
                  conv._dilation3())
    dt = L.dtype_code(cd)
    # folded weights are cached until a weight / BN tensor changes: in-place optimizer
    # updates and load_state_dict bump tensor versions; the running statistics are
    # rewritten by our BN kernels (invisible to torch), counted in _BN_UPDATES
    key = (cd, conv.weight.data_ptr(), conv.weight._version,
           None if conv.bias is None else conv.bias._version,
           None if bn.weight is None else bn.weight._version,
           None if bn.bias is None else bn.bias._version,
           bn.running_mean._version, bn.running_var._version, _BN_UPDATES[0])
    cached = getattr(conv, "_eval_fold", None)
    if cached is not None and cached[0] == key:
        wp, bias = cached[1], cached[2]
        y = _empty_vol(d.n, d.co, d.do_, d.ho, d.wo, cd, x.device)
        L.call("mmad_conv3d_fwd_ex", d, dt, L.ptr(x), L.ptr(wp), L.ptr(bias), L.ptr(res),
               int(relu), L.ptr(y), None, L.stream())
        return y
    c = d.co
    scale = torch.empty(c, dtype=torch.float32, device=x.device)
    bias = torch.empty_like(scale)
    cb = None if conv.bias is None else conv.bias.detach()
    L.call("mmad_bn_fold", c, L.ptr(None if bn.weight is None else bn.weight.detach()),
           L.ptr(None if bn.bias is None else bn.bias.detach()), L.ptr(bn.running_mean),
           L.ptr(bn.running_var), float(bn.eps), L.ptr(cb), L.ptr(scale), L.ptr(bias),
           L.stream())
    n = lib.mmad_conv_packed_elems(d, dt, 0)
    if n < 0:
        return None
    wp = torch.empty(n, dtype=cd, device=x.device)
    rc = lib.mmad_conv_pack_weight_scaled(d, dt, L.ptr(conv.weight.detach().contiguous()),
                                          L.ptr(scale), L.ptr(wp), 0, L.stream())
    if rc == L.EUNSUPPORTED:
        return None
    L.check(rc, "mmad_conv_pack_weight_scaled")
    conv._eval_fold = (key, wp, bias)
    y = _empty_vol(d.n, d.co, d.do_, d.ho, d.wo, cd, x.device)
    L.call("mmad_conv3d_fwd_ex", d, dt, L.ptr(x), L.ptr(wp), L.ptr(bias), L.ptr(res), int(relu),
           L.ptr(y), None, L.stream())
    return y


# ----------------------------------------------------------------------------- batchnorm
def _rows(t):
    c = t.shape[1]
    return t.numel() // c, c


def _finalize_args(y, parts, bn, training):
    """(mmad_bn_fin for this BN, (mean, invstd, scale, shift, use_batch)); folds very long
    partial-sum lists first and counts the running-statistics update."""
    m, c = _rows(y)
    dev = y.device
    mean = torch.empty(c, dtype=torch.float32, device=dev)
    invstd = torch.empty_like(mean)
    scale = torch.empty_like(mean)
    shift = torch.empty_like(mean)
    gamma = None if bn.weight is None else bn.weight.detach()
    beta = None if bn.bias is None else bn.bias.detach()
    use_batch = training or bn.running_mean is None
    f = L.BnFin()
    f.gamma, f.beta = _addr(gamma), _addr(beta)
    f.eps = float(bn.eps)
    f.mean, f.invstd, f.scale, f.shift = _addr(mean), _addr(invstd), _addr(scale), _addr(shift)
    keep = [gamma, beta]
    if use_batch:
        if parts is None:
            nparts = L.load().mmad_bn_stats_parts(m, c)
            parts = torch.empty((nparts, 2, c), dtype=torch.float32, device=dev)
            L.call("mmad_bn_stats", L.dtype_code(y.dtype), m, c, L.ptr(y), L.ptr(parts),
                   L.stream())
        if parts.shape[0] > 4096:        # conv-epilogue partials: one row per tile
            group = -(-parts.shape[0] // 512)
            folded = torch.empty((-(-parts.shape[0] // group), 2, c), dtype=torch.float32,
                                 device=dev)
            L.call("mmad_bn_parts_fold", c, parts.shape[0], L.ptr(parts), group, L.ptr(folded),
                   L.stream())
            parts = folded
        update = training and bn.track_running_stats and bn.running_mean is not None
        if update:
            _BN_UPDATES[0] += 1
            if bn.momentum is None:
                raise L.MMADError("BatchNorm momentum=None (cumulative average) unsupported")
        nbt = None
        if update and getattr(bn, "num_batches_tracked", None) is not None:
            nbt = bn.num_batches_tracked
            if nbt.dtype != torch.int64 or nbt.device != dev:
                raise L.MMADError("num_batches_tracked must be an int64 tensor on the device")
        f.nparts, f.parts = parts.shape[0], _addr(parts)
        f.running_mean = _addr(bn.running_mean if update else None)
        f.running_var = _addr(bn.running_var if update else None)
        f.momentum = float(bn.momentum or 0.0)
        f.training = 1
        f.num_batches_tracked = _addr(nbt)
        keep.append(parts)
    else:
        f.nparts, f.parts = 0, None
        f.running_mean, f.running_var = _addr(bn.running_mean), _addr(bn.running_var)
        f.momentum, f.training, f.num_batches_tracked = 0.0, 0, None
    f._keep = keep                       # the tensors the struct points at stay alive
    return f, (mean, invstd, scale, shift, use_batch)


def _addr(t):
    return None if t is None else t.data_ptr()


def _finalize(y, parts, bn, training):
    """batch (or running) statistics -> mean, invstd, scale, shift; updates running stats."""
    m, c = _rows(y)
    f, out = _finalize_args(y, parts, bn, training)
    L.call("mmad_bn_finalize", c, m, f.nparts, f.parts, f.gamma, f.beta, f.running_mean,
           f.running_var, f.momentum, f.eps, f.training, f.mean, f.invstd, f.scale, f.shift,
           f.num_batches_tracked, L.stream())
    return out


def _finalize_pair(y, parts, bn, res, res_parts, rbn, training):
    """_finalize for bn(y) and the shortcut rbn(res) of a residual pair in one launch
    (mmad_bn_finalize2; each set computed exactly as by _finalize)."""
    m, c = _rows(y)
    fa, a = _finalize_args(y, parts, bn, training)
    fb, b = _finalize_args(res, res_parts, rbn, training)
    L.call("mmad_bn_finalize2", c, m, C.byref(fa), C.byref(fb), L.stream())
    return a, b


# ---- twin outputs ---------------------------------------------------------------------
# A residual block reads its input twice (conv1 and the shortcut), so autograd would sum
# the two gradients of that tensor in a separate add pass before the producer's BN
# backward.  A producer asked for a twin (batchnorm_act / batchnorm_relu_maxpool with
# twin=True) also returns a second alias of its output; the block routes its shortcut
# through that alias (take_twin), each gradient reaches the producer's backward on its own,
# and the BN backward kernels add them while loading (g2 of mmad_bn_bwd_* /
# mmad_bnpool_bwd_*), rounded as torch's accumulation rounds them: same values, one pass
# fewer.  MMAD_TWIN=0 turns it off.
TWIN = os.environ.get("MMAD_TWIN", "1") != "0"
_TWINS = {}


def _twin_wanted(flag, y):
    return bool(flag) and TWIN and torch.is_grad_enabled() and y.dim() == 5


def _register_twin(out, alias):
    _TWINS[id(out)] = alias


def take_twin(x):
    """the second alias of ``x`` if its producer made one (each alias is handed out once),
    else ``x`` itself"""
    alias = _TWINS.pop(id(x), None)
    return alias if alias is not None and alias._base is x else x


def clear_twins():
    """drop twins nobody took (called at the start of each backbone forward); also the
    BN-backward-sum registrations of the previous step"""
    _TWINS.clear()
    _BNSUM_SRC.clear()
    _BNSUM_PARTS.clear()


# ---- BN-backward sums from the consumer's dgrad epilogue (round 6) --------------------
# MedicalNet's BasicBlock runs bn1 -> relu -> conv2; conv2's input gradient is exactly what
# bn1's backward column-sums.  Where conv2's dgrad route has the epilogue for it
# (mmad_conv3d_dgrad_bnsum_rows > 0; bnsum.h), the dgrad writes those partial rows itself and
# the BN backward skips its column-sum pass over g and y:
#   * _BNActFn.forward (BN+ReLU with the mask taken from y) registers its output;
#   * _Conv3dFn.forward finds its input registered and keeps the BN's (y, mean, invstd,
#     scale, shift);
#   * _Conv3dFn.backward runs mmad_conv3d_dgrad_bnsum and files the parts under the input
#     gradient it returns;
#   * _BNActFn.backward uses them when its incoming gradient IS that tensor (any other
#     gradient -- a sum with a second consumer's, a copy -- takes the column-sum pass).
# Measured (round 6, profiles/r06/r06e_bnsum_ab.txt, same box, replayed config-2 step): the
# three column sums go (14.1 + 8.3 + 6.3 us) but the dgrads grow by 12.9 / 4.3 / 4.1 us --
# their epilogue is the tail of a one-tile-per-CU launch, so the extra read of y (33.5 MB at
# layer4, all CUs at once) is exposed -- and the applies that follow lose the cache hits the
# column-sum pass gave them: kernel sum 2987.4 -> 2986.0 us, no gain; loading y ahead of the
# accumulator staging made it worse (2971.7 -> 2996.7, r06f).  So it is OFF by default;
# MMAD_BNSUM=1 (or volume_ops.BNSUM = True) switches it on (A/B; tests/test_bnsum_gpu.py
# checks the fused path either way).
BNSUM = os.environ.get("MMAD_BNSUM", "0") == "1"
_BNSUM_SRC = {}          # id(out) -> (weakref(out), (y, mean, invstd, scale, shift))
_BNSUM_PARTS = {}        # id(dx) -> (weakref(dx), parts)


def _bnsum_source(x, d, dt):
    """the BN+ReLU constants behind conv input x, if its dgrad can fold that BN's sums"""
    ent = _BNSUM_SRC.get(id(x))
    if ent is None or ent[0]() is not x:
        return None
    return ent[1] if L.load().mmad_conv3d_dgrad_bnsum_rows(d, dt) > 0 else None


def _bnsum_parts(g):
    ent = _BNSUM_PARTS.pop(id(g), None)
    return ent[1] if ent is not None and ent[0]() is g else None


def _sum_grads(g, g2):
    """g + g2 in g's dtype (the value torch's gradient accumulation produces)"""
    out = torch.empty_like(g)
    L.call("mmad_add", L.dtype_code(g.dtype), g.numel(), L.ptr(g), L.ptr(g2), L.ptr(out),
           L.stream())
    return out


def _twin_grads(g, g2, like):
    """(g, g2) as the backward kernels take them: NDHWC / contiguous in like's dtype, g2
    None when absent; g None only when neither exists"""
    if g is None:
        g, g2 = g2, None
    out = []
    for t in (g, g2):
        if t is not None:
            t = _cl(t) if like.dim() == 5 else t.contiguous()
            if t.dtype != like.dtype:
                t = cast(t, like.dtype)
        out.append(t)
    return out


def _mask_from_y_ok(y):
    """the fixed-channel apply kernel (and so the y-mask variant) covers this layout"""
    c = y.shape[1]
    v = 8 if y.dtype == torch.bfloat16 else 4
    return c % v == 0 and (c // v) & (c // v - 1) == 0 and c // v <= 256


def _bn_backward(g, relu_out, y, mean, invstd, gamma, batch_stats, want_gmask,
                 params=(None, None), mask_affine=None, g2=None, pre_parts=None):
    """BN (+ReLU) backward.  ``mask_affine`` = (scale, shift) of a BN+ReLU without residual:
    the ReLU mask is then recomputed from y (mmad_bn_relu_bwd_*) instead of read from
    ``relu_out``.  ``g2``: a twin's gradient, summed into g by the kernels.  ``pre_parts``:
    the column sums already written by the consumer's dgrad epilogue (BNSUM)."""
    m, c = _rows(y)
    dev = y.device
    dt = L.dtype_code(y.dtype)
    if g2 is not None and (mask_affine is not None or not _mask_from_y_ok(y)):
        g, g2 = _sum_grads(g, g2), None
    if pre_parts is not None:
        parts = pre_parts
        nparts = parts.shape[0]
    else:
        nparts = L.load().mmad_bn_bwd_parts(m, c)
        parts = torch.empty((nparts, 2, c), dtype=torch.float32, device=dev)
    if pre_parts is not None:
        pass
    elif mask_affine is not None:
        sc, sh = mask_affine
        L.call("mmad_bn_relu_bwd_reduce", dt, m, c, L.ptr(g), L.ptr(y), L.ptr(mean),
               L.ptr(invstd), L.ptr(sc), L.ptr(sh), L.ptr(parts), L.stream())
    else:
        L.call("mmad_bn_bwd_reduce", dt, m, c, L.ptr(g), L.ptr(g2), L.ptr(relu_out), L.ptr(y),
               L.ptr(mean), L.ptr(invstd), L.ptr(parts), L.stream())
    dgamma = grad_slot(params[0], (c,), dev)
    dbeta = grad_slot(params[1], (c,), dev)
    coef = torch.empty(3 * c, dtype=torch.float32, device=dev)
    L.call("mmad_bn_bwd_finalize", c, m, nparts, L.ptr(parts), L.ptr(gamma), L.ptr(invstd),
           int(batch_stats), L.ptr(dgamma), L.ptr(dbeta), L.ptr(coef), L.stream())
    dy = torch.empty_like(y)
    gmask = torch.empty_like(y) if want_gmask else None
    if mask_affine is not None:
        L.call("mmad_bn_relu_bwd_apply", dt, m, c, L.ptr(g), L.ptr(y), L.ptr(mean),
               L.ptr(invstd), L.ptr(mask_affine[0]), L.ptr(mask_affine[1]), L.ptr(coef),
               L.ptr(dy), L.stream())
    else:
        L.call("mmad_bn_bwd_apply", dt, m, c, L.ptr(g), L.ptr(g2), L.ptr(relu_out), L.ptr(y),
               L.ptr(mean), L.ptr(invstd), L.ptr(coef), L.ptr(dy), L.ptr(gmask), L.stream())
    return dy, dgamma, dbeta, gmask


_BN_DUAL = os.environ.get("MMAD_BN_DUAL", "1") != "0"


def _bn_backward_pair(g, relu_out, y, mean, invstd, gamma, batch_stats, y2, mean2, invstd2,
                      gamma2, batch_stats2, params, params2, g2=None, g_rows=0):
    """Both BNs of relu(bn(y) + bn2(y2)) backward, g and relu_out read once per pass
    (mmad_bn_bwd_reduce2 / _finalize2 / _apply2); equal bit for bit to two _bn_backward
    calls.  Returns (dy, dgamma, dbeta, dy2, dgamma2, dbeta2)."""
    m, c = _rows(y)
    dev = y.device
    dt = L.dtype_code(y.dtype)
    nparts = L.load().mmad_bn_bwd_parts(m, c)
    parts = torch.empty((2, nparts, 2, c), dtype=torch.float32, device=dev)
    L.call("mmad_bn_bwd_reduce2", dt, m, c, L.ptr(g), L.ptr(g2), g_rows, L.ptr(relu_out),
           L.ptr(y), L.ptr(mean), L.ptr(invstd), L.ptr(y2), L.ptr(mean2), L.ptr(invstd2),
           L.ptr(parts[0]), L.ptr(parts[1]), L.stream())
    dgamma = grad_slot(params[0], (c,), dev)
    dbeta = grad_slot(params[1], (c,), dev)
    dgamma2 = grad_slot(params2[0], (c,), dev)
    dbeta2 = grad_slot(params2[1], (c,), dev)
    coef = torch.empty((2, 3 * c), dtype=torch.float32, device=dev)
    L.call("mmad_bn_bwd_finalize2", c, m, nparts, L.ptr(parts[0]), L.ptr(gamma), L.ptr(invstd),
           int(batch_stats), L.ptr(dgamma), L.ptr(dbeta), L.ptr(coef[0]), L.ptr(parts[1]),
           L.ptr(gamma2), L.ptr(invstd2), int(batch_stats2), L.ptr(dgamma2), L.ptr(dbeta2),
           L.ptr(coef[1]), L.stream())
    dy = torch.empty_like(y)
    dy2 = torch.empty_like(y2)
    L.call("mmad_bn_bwd_apply2", dt, m, c, L.ptr(g), L.ptr(g2), g_rows, L.ptr(relu_out),
           L.ptr(y), L.ptr(mean), L.ptr(invstd), L.ptr(coef[0]), L.ptr(dy), L.ptr(y2),
           L.ptr(mean2), L.ptr(invstd2), L.ptr(coef[1]), L.ptr(dy2), L.stream())
    return dy, dgamma, dbeta, dy2, dgamma2, dbeta2


class _BNActFn(torch.autograd.Function):
    """out = act(bn(y) [+ res | + bn_r(res)]) in one pass over y (and res)."""

    @staticmethod
    def forward(ctx, y, parts, gamma, beta, res, res_parts, rgamma, rbeta, cfg):
        bn, relu, training, rbn, twin, bnsum = cfg
        L.require_device(y)
        rscale = rshift = rmean = rinvstd = None
        rbatch = False
        if rbn is not None and _BN_DUAL:
            (mean, invstd, scale, shift, batch), (rmean, rinvstd, rscale, rshift, rbatch) = \
                _finalize_pair(y, parts, bn, res, res_parts, rbn, training)
        else:
            mean, invstd, scale, shift, batch = _finalize(y, parts, bn, training)
            if rbn is not None:
                rmean, rinvstd, rscale, rshift, rbatch = _finalize(res, res_parts, rbn, training)
        out = torch.empty_like(y)
        m, c = _rows(y)
        L.call("mmad_scale_shift_act", L.dtype_code(y.dtype), m, c, L.ptr(y), L.ptr(scale),
               L.ptr(shift), L.ptr(res), L.ptr(rscale), L.ptr(rshift), int(relu), L.ptr(out),
               L.stream())
        masky = relu and res is None and y.dim() == 5 and _mask_from_y_ok(y)
        if masky and bnsum and not twin and y.dtype == torch.bfloat16:
            _BNSUM_SRC[id(out)] = (weakref.ref(out), (y, mean, invstd, scale, shift))
        ctx.save_for_backward(y, out if relu and not masky else None, mean, invstd, gamma,
                              res if rbn is not None else None, rmean, rinvstd, rgamma)
        ctx.mask_affine = (scale, shift) if masky else None
        ctx.cfg = (relu, batch, rbatch, res is not None, rbn is not None)
        ctx.params = ((gamma, beta), (rgamma, rbeta))   # gradient-slot lookup (grad_slot)
        if twin:
            ctx.set_materialize_grads(False)            # an unused twin gets no gradient
            return out, out.view(out.shape)
        return out

    @staticmethod
    def backward(ctx, g, g2=None):
        y, out, mean, invstd, gamma, rres, rmean, rinvstd, rgamma = ctx.saved_tensors
        relu, batch, rbatch, has_res, has_rbn = ctx.cfg
        pair = (has_rbn and _BN_DUAL and out is not None and ctx.mask_affine is None
                and _mask_from_y_ok(y))
        # a global-average-pool gradient arrives as a broadcast view: the pair kernels read
        # its per-sample rows in place; every other path materialises it (_twin_grads)
        g_rows = _gap_rows(g, y) if pair and y.numel() // y.shape[1] < 2 ** 31 else 0
        if g_rows:
            g2 = _twin_grads(g2, None, y)[0]
        else:
            g, g2 = _twin_grads(g, g2, y)
        if g is None:
            return (None,) * 9
        gam = None if gamma is None else gamma.detach()
        if pair:
            rg = None if rgamma is None else rgamma.detach()
            dy, dgamma, dbeta, dres, drg, drb = _bn_backward_pair(
                g, out, y, mean, invstd, gam, batch, rres, rmean, rinvstd, rg, rbatch,
                ctx.params[0], ctx.params[1], g2, g_rows)
            return (dy, None, dgamma if ctx.needs_input_grad[2] else None,
                    dbeta if ctx.needs_input_grad[3] else None, dres, None,
                    drg if ctx.needs_input_grad[6] else None,
                    drb if ctx.needs_input_grad[7] else None, None)
        if g2 is not None and has_rbn:      # per-BN calls below both read g
            g, g2 = _sum_grads(g, g2), None
        pre = _bnsum_parts(g) if ctx.mask_affine is not None and g2 is None and \
            _BNSUM_PARTS else None
        dy, dgamma, dbeta, gmask = _bn_backward(g, out, y, mean, invstd, gam, batch,
                                                has_res and not has_rbn, ctx.params[0],
                                                ctx.mask_affine, g2, pre)
        dres = drg = drb = None
        if has_rbn:
            rg = None if rgamma is None else rgamma.detach()
            dres, drg, drb, _ = _bn_backward(g, out, rres, rmean, rinvstd, rg, rbatch, False,
                                             ctx.params[1])
        elif has_res:
            dres = gmask
        return (dy, None, dgamma if ctx.needs_input_grad[2] else None,
                dbeta if ctx.needs_input_grad[3] else None, dres, None,
                drg if ctx.needs_input_grad[6] else None,
                drb if ctx.needs_input_grad[7] else None, None)


def batchnorm_act(y, bn, parts=None, relu=False, res=None, res_bn=None, res_parts=None,
                  twin=False):
    """bn(y) (+ res or res_bn(res)) then optional ReLU, torch BatchNorm semantics.

    ``bn`` / ``res_bn`` are nn.BatchNorm modules (parameters + running buffers);
    ``parts`` are the conv-epilogue partial sums of y when y came from conv3d.
    ``twin``: the output will be read by two consumers; the second one takes its alias
    with take_twin (see "twin outputs" above).
    """
    if y.dim() == 5:
        _check_vol(y)
    elif not y.is_contiguous():
        raise L.MMADError("batchnorm_act expects a contiguous (B, C) tensor")
    if res is not None:
        if res.shape != y.shape or res.dtype != y.dtype:
            raise L.MMADError("residual must match the BN input in shape and dtype")
        if y.dim() == 5:
            _check_vol(res)
    training = bn.training or not bn.track_running_stats
    twin = _twin_wanted(twin, y)
    out = _BNActFn.apply(y, parts, bn.weight, bn.bias, res, res_parts,
                         None if res_bn is None else res_bn.weight,
                         None if res_bn is None else res_bn.bias,
                         (bn, relu, training, res_bn, twin,
                          BNSUM and torch.is_grad_enabled()))
    if twin:
        out, alias = out
        _register_twin(out, alias)
    return out


class _BNReluPoolFn(torch.autograd.Function):
    """maxpool(relu(bn(y))) in one pass; the full-resolution BN+ReLU output never exists."""

    @staticmethod
    def forward(ctx, y, parts, gamma, beta, cfg):
        bn, training, k, s, p, twin = cfg
        mean, invstd, scale, shift, batch = _finalize(y, parts, bn, training)
        n, c, di, hi, wi = y.shape
        do, ho, wo = ((v + 2 * p - k) // s + 1 for v in (di, hi, wi))
        out = _empty_vol(n, c, do, ho, wo, y.dtype, y.device)
        ymax = torch.empty_like(out)
        am = torch.empty((n, do, ho, wo, c), dtype=torch.uint8, device=y.device)
        L.call("mmad_bnpool_fwd", L.dtype_code(y.dtype), n, c, di, hi, wi, do, ho, wo, k, s, p,
               L.ptr(y), L.ptr(scale), L.ptr(shift), L.ptr(out), L.ptr(am), L.ptr(ymax),
               L.stream())
        ctx.save_for_backward(y, am, ymax, mean, invstd, gamma)
        ctx.params = (gamma, beta)
        ctx.geo = (n, c, di, hi, wi, do, ho, wo, k, s, p)
        ctx.batch = batch
        if twin:
            ctx.set_materialize_grads(False)
            return out, out.view(out.shape)
        return out

    @staticmethod
    def backward(ctx, g, g2=None):
        y, am, ymax, mean, invstd, gamma = ctx.saved_tensors
        n, c, di, hi, wi, do, ho, wo, k, s, p = ctx.geo
        g, g2 = _twin_grads(g, g2, y)
        if g is None:
            return (None,) * 5
        dt = L.dtype_code(y.dtype)
        dev = y.device
        mp = n * do * ho * wo
        nparts = L.load().mmad_bn_bwd_parts(mp, c)
        parts = torch.empty((nparts, 2, c), dtype=torch.float32, device=dev)
        # a twin's gradient: the reduce also writes the summed gradient, which the apply
        # (reading each pooled gradient from up to 8 cells) then takes as its one input
        gsum = torch.empty_like(g) if g2 is not None else None
        L.call("mmad_bnpool_bwd_reduce", dt, mp, c, L.ptr(g), L.ptr(g2), L.ptr(gsum),
               L.ptr(am), L.ptr(ymax), L.ptr(mean), L.ptr(invstd), L.ptr(parts), L.stream())
        if gsum is not None:
            g = gsum
        dgamma = grad_slot(ctx.params[0], (c,), dev)
        dbeta = grad_slot(ctx.params[1], (c,), dev)
        coef = torch.empty(3 * c, dtype=torch.float32, device=dev)
        gam = None if gamma is None else gamma.detach()
        L.call("mmad_bn_bwd_finalize", c, n * di * hi * wi, nparts, L.ptr(parts), L.ptr(gam),
               L.ptr(invstd), int(ctx.batch), L.ptr(dgamma), L.ptr(dbeta), L.ptr(coef),
               L.stream())
        dy = torch.empty_like(y)
        L.call("mmad_bnpool_bwd_apply", dt, n, c, di, hi, wi, do, ho, wo, k, s, p, L.ptr(g),
               L.ptr(am), L.ptr(y), L.ptr(mean), L.ptr(invstd), L.ptr(coef), L.ptr(dy),
               L.stream())
        return (dy, None, dgamma if ctx.needs_input_grad[2] else None,
                dbeta if ctx.needs_input_grad[3] else None, None)


def batchnorm_relu_maxpool(y, bn, parts, kernel_size, stride, padding, twin=False):
    """max_pool3d(relu(bn(y)), k, s, p) fused (MedicalNet stem: bn1 -> relu -> maxpool);
    ``twin`` as in batchnorm_act."""
    _check_vol(y)
    training = bn.training or not bn.track_running_stats
    twin = _twin_wanted(twin, y)
    out = _BNReluPoolFn.apply(y, parts, bn.weight, bn.bias,
                              (bn, training, int(kernel_size), int(stride), int(padding), twin))
    if twin:
        out, alias = out
        _register_twin(out, alias)
    return out


# ------------------------------------------------------------------------------- pooling
class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        _check_vol(x)
        n, c, di, hi, wi = x.shape
        do, ho, wo = ((v + 2 * p - k) // s + 1 for v in (di, hi, wi))
        y = _empty_vol(n, c, do, ho, wo, x.dtype, x.device)
        am = torch.empty((n, do, ho, wo, c), dtype=torch.uint8, device=x.device)
        L.call("mmad_maxpool3d_fwd", L.dtype_code(x.dtype), n, c, di, hi, wi, do, ho, wo, k, s,
               p, L.ptr(x), L.ptr(y), L.ptr(am), L.stream())
        ctx.save_for_backward(am)
        ctx.geo = (n, c, di, hi, wi, do, ho, wo, k, s, p)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        (am,) = ctx.saved_tensors
        n, c, di, hi, wi, do, ho, wo, k, s, p = ctx.geo
        g = _cl(g)
        if g.dtype != ctx.dtype:
            g = cast(g, ctx.dtype)
        dx = _empty_vol(n, c, di, hi, wi, ctx.dtype, g.device)
        L.call("mmad_maxpool3d_bwd", L.dtype_code(ctx.dtype), n, c, di, hi, wi, do, ho, wo, k,
               s, p, L.ptr(g), L.ptr(am), L.ptr(dx), L.stream())
        return dx, None, None, None


def max_pool3d(x, kernel_size, stride=None, padding=0):
    return _MaxPoolFn.apply(x, int(kernel_size), int(stride or kernel_size), int(padding))


# MMAD_GAP_BCAST=0: the GAP backward writes the broadcast gradient out in full (A/B switch)
GAP_BCAST = os.environ.get("MMAD_GAP_BCAST", "1") != "0"


def _gap_rows(g, like):
    """rows per sample when g is _GapFn's stride-0 broadcast gradient for ``like``, else 0"""
    if g is None or g.dim() != 5 or tuple(g.shape) != tuple(like.shape) or \
            g.dtype != like.dtype:
        return 0
    n, c, d, h, w = g.shape
    if g.stride()[1:] != (1, 0, 0, 0) or g.stride(0) != c:
        return 0
    return d * h * w


class _GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        _check_vol(x)
        n, c = x.shape[:2]
        s = x.numel() // (n * c)
        y = torch.empty((n, c, 1, 1, 1), dtype=torch.float32, device=x.device)
        ws = torch.empty(L.load().mmad_gap_fwd_ws_elems(n, s, c), dtype=torch.float32,
                         device=x.device)
        L.call("mmad_gap_fwd_ws", L.dtype_code(x.dtype), n, s, c, L.ptr(x), L.ptr(y), L.ptr(ws),
               L.stream())
        ctx.shape = tuple(x.shape)
        ctx.dtype = x.dtype
        return y

    @staticmethod
    def backward(ctx, g):
        n, c = ctx.shape[:2]
        s = 1
        for v in ctx.shape[2:]:
            s *= v
        g = g.contiguous()
        if g.dtype != torch.float32:
            g = cast(g, torch.float32)
        if GAP_BCAST:
            # the input gradient g/s per (sample, channel), handed on as a stride-0 broadcast
            # view: a BN-pair backward reads its rows in place (g_rows of
            # mmad_bn_bwd_reduce2 / _apply2); any other consumer materialises it
            rows = torch.empty((n, c), dtype=ctx.dtype, device=g.device)
            L.call("mmad_gap_bwd_compact", L.dtype_code(ctx.dtype), n, s, c, L.ptr(g),
                   L.ptr(rows), L.stream())
            return rows.view(n, c, 1, 1, 1).expand(ctx.shape)
        dx = _empty_vol(*ctx.shape, ctx.dtype, g.device)
        L.call("mmad_gap_bwd", L.dtype_code(ctx.dtype), n, s, c, L.ptr(g), L.ptr(dx), L.stream())
        return dx


def global_avg_pool(x):
    """AdaptiveAvgPool3d(1): (N,C,D,H,W) NDHWC -> (N,C,1,1,1) float32."""
    return _GapFn.apply(x)


# ----------------------------------------------------------------- feature-map fusion
class _Max2Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        _check_vol(a)
        _check_vol(b, a.dtype)
        if a.shape != b.shape:
            raise L.MMADError("maxout fusion needs equal volume shapes")
        y = torch.empty_like(a)
        sel = torch.empty(a.numel(), dtype=torch.uint8, device=a.device)
        L.call("mmad_max2_fwd", L.dtype_code(a.dtype), a.numel(), L.ptr(a), L.ptr(b), L.ptr(y),
               L.ptr(sel), L.stream())
        ctx.save_for_backward(sel)
        return y

    @staticmethod
    def backward(ctx, g):
        (sel,) = ctx.saved_tensors
        g = _cl(g)
        ga, gb = torch.empty_like(g), torch.empty_like(g)
        L.call("mmad_max2_bwd", L.dtype_code(g.dtype), g.numel(), L.ptr(g), L.ptr(sel),
               L.ptr(ga), L.ptr(gb), L.stream())
        return ga, gb


def maxout(a, b):
    """torch.max(torch.stack((a, b), dim=0), dim=0)[0] -- the 'maxout' feature-map fusion
    (anat_pet_featuremapfusion.py:115-117): ties go to ``a``, NaN propagates."""
    return _Max2Fn.apply(a, b)


class _CatChannelsFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        _check_vol(a)
        _check_vol(b, a.dtype)
        if a.shape[0] != b.shape[0] or a.shape[2:] != b.shape[2:]:
            raise L.MMADError("channel concat needs equal batch and spatial extents")
        n, ca, di, hi, wi = a.shape
        cb = b.shape[1]
        y = _empty_vol(n, ca + cb, di, hi, wi, a.dtype, a.device)
        L.call("mmad_concat_channels", L.dtype_code(a.dtype), n * di * hi * wi, ca, L.ptr(a),
               cb, L.ptr(b), L.ptr(y), L.stream())
        ctx.cfg = (ca, cb)
        return y

    @staticmethod
    def backward(ctx, g):
        ca, cb = ctx.cfg
        g = _cl(g)
        n, _, di, hi, wi = g.shape
        ga = _empty_vol(n, ca, di, hi, wi, g.dtype, g.device) if ctx.needs_input_grad[0] else None
        gb = _empty_vol(n, cb, di, hi, wi, g.dtype, g.device) if ctx.needs_input_grad[1] else None
        if ga is not None or gb is not None:
            L.call("mmad_split_channels", L.dtype_code(g.dtype), n * di * hi * wi, ca, cb,
                   L.ptr(g), L.ptr(ga), L.ptr(gb), L.stream())
        return ga, gb


def cat_channels(a, b):
    """torch.cat((a, b), dim=1) of two NDHWC volumes -- the 'concatenate' feature-map
    fusion (anat_pet_featuremapfusion.py:112-113)."""
    return _CatChannelsFn.apply(a, b)


# --------------------------------------------------------------------- elementwise / cast
class _ReluFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        L.require_device(x)
        if not (x.is_contiguous() or (x.dim() == 5 and x.is_contiguous(memory_format=CL))):
            raise L.MMADError("relu expects a dense tensor")
        y = torch.empty_like(x)
        L.call("mmad_relu_fwd", L.dtype_code(x.dtype), x.numel(), L.ptr(x), L.ptr(y), L.stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, g):
        (y,) = ctx.saved_tensors
        g = _cl(g) if y.dim() == 5 and y.is_contiguous(memory_format=CL) else g.contiguous()
        if g.dtype != y.dtype:
            g = cast(g, y.dtype)
        dx = torch.empty_like(y)
        L.call("mmad_relu_bwd", L.dtype_code(y.dtype), y.numel(), L.ptr(g), L.ptr(y), L.ptr(dx),
               L.stream())
        return dx


def relu(x):
    return _ReluFn.apply(x)


class _CastFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, dtype):
        ctx.src = x.dtype
        return _cast_raw(x, dtype)

    @staticmethod
    def backward(ctx, g):
        return _cast_raw(g, ctx.src), None


def _cast_raw(x, dtype):
    L.require_device(x)
    if x.dtype == dtype:
        return x
    if x.dim() == 5 and x.is_contiguous(memory_format=CL) and not x.is_contiguous():
        y = torch.empty_like(x, dtype=dtype)
    else:
        x = x.contiguous()
        y = torch.empty(x.shape, dtype=dtype, device=x.device)
    L.call("mmad_cast", L.dtype_code(x.dtype), L.dtype_code(dtype), x.numel(), L.ptr(x),
           L.ptr(y), L.stream())
    return y


def cast(x, dtype):
    """dtype conversion on device (f64 -> f32 -> bf16 rounding order, as torch)."""
    if x.dtype == dtype:
        return x
    return _CastFn.apply(x, dtype)
