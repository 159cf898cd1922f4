"""The captured training step's optimizer: Adam fused with the bf16 weight repack.

``AdamRepack(optimizer, plans)`` replaces ``optimizer.step()`` inside a captured step
(graph_step.GraphedTrainStep) by ONE launch of ``mmad_adam_repack`` (csrc/adam.hip):

* every parameter of every group gets torch's fused Adam update, bit for bit (the
  reference's optimizer: ``torch.optim.Adam`` over anat_cnn.py:111-126's groups, here
  ``classifiers.MergedAdam`` with ``fused=True``), its device ``step`` counter included, so
  the optimizer state stays torch's own (``state_dict`` / resume unchanged);
* each conv weight a ``volume_ops.PackPlan`` repacks every step (the bf16 forward and
  input-gradient layouts, ``mmad_conv_pack_dual_batch``) leaves the update in both layouts
  as well, for the NEXT step's forward: the captured forward then skips that repack
  (``PackPlan.external``), so the fp32 weights are read once per step, not twice, and four
  launches (step counters, two learning-rate groups, the repack) become one.

The packed copies are then only as fresh as the last Adam step: ``refresh()`` repacks them
from the fp32 weights (GraphedTrainStep calls it before the first replay and whenever a
parameter was modified outside the graph, seen through its ``_version``).

Supported: ``torch.optim.Adam`` (and subclasses that keep its ``step``) with fused=True,
amsgrad / maximize / differentiable / decoupled weight decay off, float betas, fp32
parameters and state, no gradient scaler.  ``supported(optimizer)`` says whether it
applies; the caller keeps ``optimizer.step()`` otherwise."""
import ctypes as C
import inspect
import os

import torch

from . import _lib as L

# MMAD_ADAM_REPACK=0: captured steps keep torch's fused Adam and the in-forward repack (A/B)
ENABLED = os.environ.get("MMAD_ADAM_REPACK", "1") != "0"


def supported(optimizer):
    if not ENABLED or not isinstance(optimizer, torch.optim.Adam):
        return False
    # (torch wraps a class's step with its profiling hook on first construction, on the
    # subclass or on Adam itself: compare the functions underneath)
    if isinstance(optimizer, torch.optim.AdamW) or \
            inspect.unwrap(type(optimizer).step) is not inspect.unwrap(torch.optim.Adam.step):
        return False
    if getattr(optimizer, "grad_scale", None) is not None or \
            getattr(optimizer, "found_inf", None) is not None:
        return False
    for g in optimizer.param_groups:
        if not g.get("fused") or g.get("amsgrad") or g.get("maximize") or \
                g.get("differentiable") or g.get("decoupled_weight_decay", False):
            return False
        b1, b2 = g["betas"]
        if torch.is_tensor(b1) or torch.is_tensor(b2) or torch.is_tensor(g["eps"]) or \
                torch.is_tensor(g["weight_decay"]):
            return False
    return True


def state_ready(optimizer):
    """every parameter that will get a gradient has its Adam state (one eager step ran)"""
    return all(all(k in optimizer.state.get(p, {}) for k in ("step", "exp_avg", "exp_avg_sq"))
               for g in optimizer.param_groups for p in g["params"] if p.requires_grad)


def pack_plans(model):
    """the volume_ops.PackPlan objects under ``model`` (built by its forwards)"""
    out = []
    for m in model.modules():
        plan = getattr(m, "_mmad_pack_plan", None)
        if plan is not None and plan not in out:
            out.append(plan)
    return out


class AdamRepack:
    def __init__(self, optimizer, plans=()):
        if not supported(optimizer):
            raise ValueError("AdamRepack: optimizer configuration not supported")
        self.optimizer = optimizer
        self.plans = [p for p in plans if p.nduals or p.unfolds]
        self.table = None
        self.njobs = self.tiles = 0
        self._host = None

    def _jobs(self):
        lib = L.load()
        dual, unf = {}, {}
        for plan in self.plans:
            for job in plan.duals:
                dual[job.w] = job
            for w, d, wp in plan.unfolds:
                unf[w.data_ptr()] = (d, wp)
        jobs, tiles = [], 0
        for g in self.optimizer.param_groups:
            lr = g["lr"]
            if not (torch.is_tensor(lr) and lr.is_cuda and lr.dtype == torch.float32):
                raise ValueError("AdamRepack: the group lr must be a device float32 tensor "
                                 "(graph_step installs one)")
            b1, b2 = g["betas"]
            for p in g["params"]:
                if p.grad is None:
                    continue                 # torch's Adam skips these too
                st = self.optimizer.state.get(p, {})
                need = ("step", "exp_avg", "exp_avg_sq")
                if any(k not in st for k in need):
                    raise ValueError("AdamRepack: optimizer state not initialised (run one "
                                     "eager step first)")
                ts = (p, p.grad, st["exp_avg"], st["exp_avg_sq"], st["step"])
                if any(not t.is_cuda or t.dtype != torch.float32 for t in ts) or \
                        any(not t.is_contiguous() for t in ts[:4]) or st["step"].numel() != 1:
                    raise ValueError("AdamRepack: fp32 contiguous device tensors required")
                j = L.AdamJob()
                j.param, j.grad = p.data_ptr(), p.grad.data_ptr()
                j.exp_avg, j.exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
                j.step, j.lr = st["step"].data_ptr(), lr.data_ptr()
                j.beta1, j.beta2 = float(b1), float(b2)
                j.eps, j.weight_decay = float(g["eps"]), float(g["weight_decay"])
                d = dual.get(p.data_ptr())
                if d is not None:
                    j.w_fwd, j.w_dgrad = d.w_fwd, d.w_dgrad
                    j.co, j.ci, j.taps, j.flip = d.co, d.ci, d.taps, d.flip
                u = unf.get(p.data_ptr())
                if u is not None:
                    desc, wp = u
                    j.w_fwd = wp.data_ptr()
                    j.co, j.ci, j.taps = desc.co, 1, desc.kd * desc.kh
                    j.unf_kw, j.kpad = desc.kw, wp.numel() // desc.co
                j.numel = p.numel()
                j.tile0 = tiles
                j.ntiles = lib.mmad_adam_job_tiles(j)
                tiles += j.ntiles
                jobs.append(j)
        # a repacked weight without an update here (frozen, or outside the optimizer) does
        # not change in the step, so its packed copy from refresh() stays valid
        return jobs, tiles

    def prepare(self, device):
        """allocate the device job table and arrival counters (before capture: nothing may
        be allocated from the host inside one)"""
        n = sum(len(g["params"]) for g in self.optimizer.param_groups)
        self.table = torch.empty(max(n, 1) * C.sizeof(L.AdamJob), dtype=torch.uint8,
                                 device=device)
        self.arrivals = torch.zeros(max(n, 1), dtype=torch.int32, device=device)
        # each block's job index (sized for every parameter as repacked tiles or 4096-element
        # chunks, the most blocks the jobs can need)
        lib = L.load()
        blocks = 0
        for g in self.optimizer.param_groups:
            for p in g["params"]:
                j = L.AdamJob()
                j.numel = p.numel()
                blocks += max(lib.mmad_adam_job_tiles(C.byref(j)), 1)
                if p.dim() == 5:
                    blocks += p.shape[0] // 16 * max(p.shape[1] // 16, 1) + p.shape[0]
        self.block_job = torch.zeros(max(blocks, 1), dtype=torch.int32, device=device)

    def step(self):
        """launch the fused update on the current stream (capturable: the job table is
        written by ``commit()`` once the gradients' addresses are known)"""
        jobs, tiles = self._jobs()
        if self.table is None:
            self.prepare(next(iter(self.optimizer.param_groups))["params"][0].device)
        if len(jobs) * C.sizeof(L.AdamJob) > self.table.numel():
            raise ValueError("AdamRepack: more jobs than prepared")
        if tiles > self.block_job.numel():
            raise ValueError("AdamRepack: more blocks than prepared")
        self.njobs, self.tiles = len(jobs), tiles
        self._host = bytes((L.AdamJob * len(jobs))(*jobs)) if jobs else b""
        self._host_map = torch.repeat_interleave(
            torch.arange(len(jobs), dtype=torch.int32),
            torch.tensor([j.ntiles for j in jobs], dtype=torch.int64)) if jobs else None
        if not torch.cuda.is_current_stream_capturing():
            self.commit()
        L.call("mmad_adam_repack", self.njobs, L.ptr(self.table), L.ptr(self.block_job),
               self.tiles, L.ptr(self.arrivals), L.stream())

    def commit(self):
        """copy the job table built by the last ``step()`` to the device (outside capture)"""
        if self._host:
            host = torch.frombuffer(bytearray(self._host), dtype=torch.uint8)
            self.table[:host.numel()].copy_(host)
            self.block_job[:self._host_map.numel()].copy_(self._host_map)

    def set_external(self, on):
        for plan in self.plans:
            plan.external = bool(on)

    def refresh(self):
        """repack every covered conv weight from its current fp32 values"""
        for plan in self.plans:
            plan.run_duals()

    def params(self):
        return [p for g in self.optimizer.param_groups for p in g["params"]]
