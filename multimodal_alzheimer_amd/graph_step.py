"""One training step captured as HIP graphs and replayed.

The eager step (``general_step`` -> ``loss.backward()`` -> ``optimizer.step()``, what
Lightning's automatic optimisation runs per batch, anat_cnn.py:99-109 + :111-136) issues
~130 kernels from Python; at batch 8 and 128^3 a tenth of them are tiny (BN finalizes, the
head, casts) and every dispatch carries the host launch path and its completion signal.
Captured once with ``torch.cuda.graph`` (our ops launch on torch's current stream, so they
are captured like torch's own kernels), a replay submits the whole step as one graph.

Requirements (the usual whole-step capture rules): static shapes and a fixed batch
buffer (``step(batch)`` copies the new batch into it), no host reads of device values in
the step, the optimizer made capturable (set here), gradients produced inside the graph
(``zero_grad(set_to_none=True)`` before capture).  Warm-up iterations run eagerly on a side
stream first, as torch requires, so the model takes ``warmup`` optimizer steps before the
first replay.

With a data-parallel gradient all-reduce (``reducer``, data_parallel.GradAllReduce) there
are three ways to place the RCCL collectives (``collectives=``):

* ``"staged"`` (one of the three modes bench.py's ``auto`` default probes at N > 1; it
  picks the fastest, ``after`` on one rank): the backward is split at backbone stage
  boundaries (``backward_stages``: head + layer4 | layer3 | layer2 | layer1 + stem of every
  MedicalNet ResNet in the model) and each part is captured as its own graph
  (``StagedBackward``: ``torch.autograd.grad`` from the previous boundary's gradients to
  the next boundary's tensors and this stage's parameters).  Each call replays graph 0
  (forward + first backward stage), starts that stage's bucket all-reduce on the side
  stream (after the main stream's work so far), replays graph 1 on the main stream while
  the collective runs, and so on; then ``finish()`` (main waits for the side stream) and
  the captured Adam.  Only the last stage's ~1 MB bucket is not overlapped.  The ordering
  guarantee is plain stream order: a bucket's collective is enqueued on the side stream
  behind an event recorded on the main stream after the graph that produced it.
* ``"after"``: one graph holds forward + backward; each call replays it, runs
  ``finish()`` eagerly -- every bucket's all-reduce on the side stream, not overlapped with
  the backward -- then replays the captured optimizer step.
* ``"inside"``: the bucket all-reduces (launched from the backward's hooks) and
  ``finish()`` are captured with the step (experimental; bench.py --graph).

What a replay changes without running Python is made visible to the host-side state that
depends on it:
* each group's ``lr`` becomes a 0-d device tensor before capture, so the captured fused Adam
  reads it at replay time and an LR scheduler (``ReduceLROnPlateau`` from
  ``configure_optimizers``, anat_cnn.py:129-134) that updates it in place
  (``param_group['lr'].fill_``) takes effect on the next replay;
* the eval-mode folded-weight cache (``volume_ops.conv_bn_act_eval``) is keyed on tensor
  versions and a BN-update counter, which a replay bumps neither of: every replay advances
  ``volume_ops._BN_UPDATES`` so the next evaluation refolds;
* dropout draws its seed on the device (``head_ops.dropout``), so every replay gets a
  fresh mask.
"""
import os

import torch

from . import fused_optim, volume_ops

COLLECTIVES = ("staged", "after", "inside")
# Captures check only this thread's calls: ProcessGroupNCCL's watchdog thread polls the events
# of collectives issued before a capture (hipEventQuery), which "global" mode turns into a
# capture error that aborts the process (seen when a blocking all-reduce ran just before one)
_CAPTURE_MODE = "thread_local"
# MMAD_DEFER_WGRAD=0: every conv's weight-gradient slab reduction launches right after its
# split-K kernel inside the captured backward (A/B switch for volume_ops'
# deferred_wgrad_reduce)
DEFER_WGRAD = os.environ.get("MMAD_DEFER_WGRAD", "1") != "0"
DEFAULT_CUTS = ("layer4", "layer3", "layer2")


def backward_stages(model, cuts=DEFAULT_CUTS):
    """Split ``model``'s backward at the inputs of the named stages of every MedicalNet
    ResNet inside it (``cuts`` in backward order).  Returns ``(boundaries, params)``:
    ``boundaries[k]`` = the modules whose forward input closes stage k (k < S - 1), and
    ``params[k]`` = the trainable parameters whose gradients stage k completes:
    stage 0 = everything downstream of the first cut (the heads, fusion MLP, any branch
    that is not a ResNet, the cut stage itself), stage k = the k-th cut stage of each
    ResNet, the last stage = what precedes the last cut (stem + earlier stages).
    Returns ``([], [all params])`` when the model has no ResNet."""
    from .medicalnet import ResNet
    nets = [m for m in model.modules() if isinstance(m, ResNet)]
    trainable = [p for p in model.parameters() if p.requires_grad]
    if not nets or not cuts:
        return [], [trainable]
    order = ("conv1", "bn1", "layer1", "layer2", "layer3", "layer4")
    pos = [order.index(c) for c in cuts]
    if pos != sorted(pos, reverse=True) or len(set(pos)) != len(pos):
        raise ValueError(f"cuts must name distinct stages in backward order, got {cuts}")
    stage_of = {}
    for net in nets:
        for i, name in enumerate(order):
            # stage of module ``name``: the number of cuts at or before it, counted from
            # the back (a module at or after cuts[0] is in stage 0)
            k = sum(1 for p in pos if i < p)
            for p in getattr(net, name).parameters():
                stage_of[p] = k
    params = [[] for _ in range(len(cuts) + 1)]
    for p in trainable:
        params[stage_of.get(p, 0)].append(p)
    boundaries = [[getattr(net, c) for net in nets] for c in cuts]
    return boundaries, params


class StagedBackward:
    """The backward of one step as S consecutive parts (``backward_stages``), so that each
    part can be captured as its own graph and the gradients it completes handed to the
    all-reduce while the next part runs.

    ``arm()`` registers forward pre-hooks on the boundary modules that record each
    boundary's input tensor and its twin alias (volume_ops "twin outputs": a residual
    block reads its input through two aliases, both outputs of the producer's autograd
    node).  ``run(k, loss)`` computes stage k with ``torch.autograd.grad`` -- the gradients
    of the next boundary's tensors are CAPTURED at the producer's node (the node itself
    runs in the next stage) -- and assigns this stage's parameter gradients as ``.grad``
    (a weight gradient written into its data-parallel bucket slice stays that slice).
    Same kernels, same order as one ``loss.backward()``."""

    def __init__(self, boundaries, params):
        self.boundaries, self.params = boundaries, params
        self.n = len(params)
        self._rec = [[] for _ in boundaries]
        self._grads = None
        self._hooks = []

    def arm(self):
        self.disarm()
        self._rec = [[] for _ in self.boundaries]
        for k, mods in enumerate(self.boundaries):
            for m in mods:
                self._hooks.append(m.register_forward_pre_hook(self._recorder(k)))

    def disarm(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []

    def _recorder(self, k):
        def hook(_mod, args):
            x = args[0]
            self._rec[k].append(x)
            alias = volume_ops._TWINS.get(id(x))
            if alias is not None and alias._base is x:
                self._rec[k].append(alias)
        return hook

    def run(self, k, loss=None, seed=None):
        if k == 0:
            roots, grads = [loss], (None if seed is None else [seed])
        else:
            roots, grads = self._grads
        nxt = [t for t in self._rec[k] if t.requires_grad] if k < self.n - 1 else []
        ps = self.params[k]
        if not nxt and not ps:
            self._grads = ([], [])
            return
        if not roots:
            raise RuntimeError(f"backward stage {k}: no gradient reached its boundary")
        out = torch.autograd.grad(roots, nxt + ps, grads, allow_unused=True)
        volume_ops.flush_wgrad_reduce()      # this stage's queued dW reductions (if any)
        for p, g in zip(ps, out[len(nxt):]):
            if g is None:
                continue
            if p.grad is None:
                p.grad = g
            else:
                p.grad.add_(g)
        volume_ops.check_deferred_adoption()
        keep = [(t, g) for t, g in zip(nxt, out[:len(nxt)]) if g is not None]
        self._grads = ([t for t, _ in keep], [g for _, g in keep])
        if k == self.n - 1:
            self.release()

    def release(self):
        self._grads = None
        self._rec = [[] for _ in self.boundaries]

    def run_all(self, loss):
        """every stage in order (eager use; ``arm()`` must have been active during the
        forward that produced ``loss``)"""
        for k in range(self.n):
            self.run(k, loss)


class GraphedTrainStep:
    def __init__(self, model, optimizer, batch, warmup=3, reducer=None, collectives="inside",
                 cuts=DEFAULT_CUTS):
        """``reducer``: a data_parallel.GradAllReduce (for ``collectives="staged"`` built
        with ``stages=backward_stages(model, cuts)[1]``).  ``collectives``: see the module
        docstring."""
        self.model, self.optimizer = model, optimizer
        self.reducer = reducer
        if reducer is not None and collectives not in COLLECTIVES:
            raise ValueError(f"collectives must be one of {COLLECTIVES}, not {collectives!r}")
        self.mode = collectives if reducer is not None else None
        self.finish_events = None            # list: (start, end) events around each finish()
        self.static = {k: v.clone() if torch.is_tensor(v) else v for k, v in batch.items()}
        dev = next(model.parameters()).device
        for g in optimizer.param_groups:
            g["capturable"] = True
            if not torch.is_tensor(g["lr"]):
                g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float32, device=dev)
        staged = None
        if self.mode == "staged":
            bounds, params = backward_stages(model, cuts)
            staged = StagedBackward(bounds, params)
            if reducer.stage_buckets is None or len(reducer.stage_buckets) != staged.n:
                raise ValueError("collectives='staged' needs GradAllReduce(stages=...) built "
                                 "from backward_stages(model, cuts)")
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        loss = None
        with torch.cuda.stream(side):
            for _ in range(warmup):
                loss = self._eager()
        torch.cuda.current_stream().wait_stream(side)
        # the backward's seed gradient (d loss / d loss = 1) made before capture, so the
        # captured step has no fill kernel for it
        self._one = None if loss is None else torch.ones_like(loss)
        optimizer.zero_grad(set_to_none=True)
        self.graphs = []
        self.opt_graph = None
        # Adam fused with the weight repack (fused_optim): the captured forwards skip the
        # dual-layout repack, which the captured optimizer step writes for the next replay
        self.fused = None
        if fused_optim.supported(optimizer) and fused_optim.state_ready(optimizer):
            self.fused = fused_optim.AdamRepack(optimizer, fused_optim.pack_plans(model))
            self.fused.prepare(dev)
            self.fused.set_external(True)
        try:
            self._capture(model, optimizer, reducer, staged)
        finally:
            if self.fused is not None:
                self.fused.set_external(False)
        if self.fused is not None:
            self.fused.commit()              # the job table (gradient addresses from capture)
            self.fused.refresh()             # packed weights of the current fp32 weights
        self._versions = self._param_versions()
        self.graph = self.graphs[0]
        # keep the graph-owned output buffers, not their autograd graph: a live grad_fn chain
        # would keep every parameter's AccumulateGrad node (created on the capture stream)
        # alive, and later eager steps would reuse those nodes across streams
        self.out = {k: v.detach() if torch.is_tensor(v) else v for k, v in self.out.items()}

    def _opt_step(self):
        if self.fused is not None:
            self.fused.step()
        else:
            self.optimizer.step()

    def refresh(self):
        """Repack the bf16 weight layouts from the current fp32 weights.  Replays do this by
        themselves when a parameter's ``_version`` moved (an in-place op, or a helper that
        bumps it, as data_parallel.broadcast_module_state does); call it after editing
        weights through ``.data``, which the version counter does not see."""
        if self.fused is not None:
            self.fused.refresh()
            self._versions = self._param_versions()

    def _param_versions(self):
        if self.fused is None:
            return None
        return tuple(p._version for p in self.fused.params())

    def _capture(self, model, optimizer, reducer, staged):
        # the weight-gradient slab reductions queue up and run as one launch at the end of
        # the backward (each stage's, when staged) -- not with collectives captured inside,
        # whose bucket hooks would read the queued gradients
        with volume_ops.deferred_wgrad_reduce(DEFER_WGRAD and self.mode != "inside"):
            self._capture_body(model, optimizer, reducer, staged)

    def _capture_body(self, model, optimizer, reducer, staged):
        if self.mode in ("staged", "after"):
            reducer.defer = True             # the capture's hooks (if any) only count
            try:
                if self.mode == "after":
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                        self.out = model.general_step(self.static, 0, "train")
                        self.out["loss"].backward(self._one)
                        volume_ops.flush_wgrad_reduce()
                    self.graphs.append(g)
                else:
                    staged.arm()
                    try:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                            self.out = model.general_step(self.static, 0, "train")
                            staged.run(0, self.out["loss"], self._one)
                    finally:
                        staged.disarm()
                    self.graphs.append(g)
                    for k in range(1, staged.n):
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, pool=self.graphs[0].pool(),
                                              capture_error_mode=_CAPTURE_MODE):
                            staged.run(k)
                        self.graphs.append(g)
            finally:
                reducer.defer = False
            reducer.reset()
            reducer.finish()                 # eager: gradients now averaged in place
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=self.graphs[0].pool(),
                                  capture_error_mode=_CAPTURE_MODE):
                self._opt_step()
        else:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode=_CAPTURE_MODE):
                self.out = model.general_step(self.static, 0, "train")
                self.out["loss"].backward(self._one)
                volume_ops.flush_wgrad_reduce()
                if reducer is not None:
                    reducer.finish()
                self._opt_step()
            self.graphs.append(g)

    def _eager(self):
        self.optimizer.zero_grad(set_to_none=True)
        loss = self.model.general_step(self.static, 0, "train")["loss"]
        loss.backward()
        if self.reducer is not None:
            self.reducer.finish()
        self.optimizer.step()
        return loss.detach()

    def __call__(self, batch=None):
        """Replay one step; ``batch`` (same keys / shapes) is copied into the graph's input
        buffers first.  Returns the step's {'loss', 'outputs', 'labels'} (graph-owned
        tensors, overwritten by the next replay)."""
        if batch is not None:
            for k, v in batch.items():
                if torch.is_tensor(v):
                    self.static[k].copy_(v, non_blocking=True)
        if self.fused is not None:
            v = self._param_versions()
            if v != self._versions:          # weights changed outside the graph: repack
                self.fused.refresh()
                self._versions = v
        if self.mode is None or self.mode == "inside":
            self.graph.replay()
        else:
            last = len(self.graphs) - 1
            for k, g in enumerate(self.graphs):
                g.replay()
                if self.mode == "staged" and k < last:
                    self.reducer.launch_stage(k)   # overlaps the next graph's replay
            if self.finish_events is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            # the last stage's buckets (nothing left to overlap them with) are reduced by
            # finish() on the main stream; then main waits for the side stream, copies back
            self.reducer.finish()
            if self.finish_events is not None:
                e1.record()
                self.finish_events.append((e0, e1))
            self.opt_graph.replay()
        volume_ops._BN_UPDATES[0] += 1     # weights / running stats changed on the device
        return self.out
