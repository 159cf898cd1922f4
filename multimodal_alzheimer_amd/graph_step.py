"""One training step captured as a HIP graph and replayed.

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
first replay.  Not combined with the RCCL gradient all-reduce (data_parallel) here.

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

from . import volume_ops


class GraphedTrainStep:
    def __init__(self, model, optimizer, batch, warmup=3, reducer=None, collectives="inside"):
        """``reducer``: a data_parallel.GradAllReduce.  ``collectives``:
        * "inside": its bucket all-reduces (launched from the backward's hooks) and
          ``finish()`` are captured with the step (experimental: bench.py --graph under
          torchrun; checked at one rank only);
        * "after": the graph holds forward + backward only (gradients land in the bucket
          slices); each call replays it, then runs ``finish()`` eagerly -- every bucket's
          RCCL all-reduce on the side stream, not overlapped with the backward -- then
          replays the captured optimizer step.  No collective inside a graph; the host
          issues a handful of calls per step (bench.py's default at N > 1)."""
        self.model, self.optimizer = model, optimizer
        self.reducer = reducer
        self.after = reducer is not None and collectives == "after"
        self.finish_events = None            # list: (start, end) events around each finish()
        if reducer is not None and collectives not in ("inside", "after"):
            raise ValueError(f"collectives must be 'inside' or 'after', not {collectives!r}")
        self.static = {k: v.clone() if torch.is_tensor(v) else v for k, v in batch.items()}
        dev = next(model.parameters()).device
        for g in optimizer.param_groups:
            g["capturable"] = True
            if not torch.is_tensor(g["lr"]):
                g["lr"] = torch.tensor(float(g["lr"]), dtype=torch.float32, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        self.opt_graph = None
        if self.after:
            reducer.defer = os.environ.get("MMAD_GRAPH_DEBUG", "") != "nodefer"
            try:
                with torch.cuda.graph(self.graph):
                    self.out = model.general_step(self.static, 0, "train")
                    self.out["loss"].backward()
                    dbg = os.environ.get("MMAD_GRAPH_DEBUG", "")
                    if dbg == "join":
                        torch.cuda.current_stream().wait_stream(
                            volume_ops.grad_stream(self.static_device()))
                    elif dbg == "tail":
                        self._tail = torch.zeros(1, device=self.static_device()).add_(1)
            finally:
                reducer.defer = False
            reducer.reset()                  # the capture's hooks only counted
            reducer.finish()                 # eager: gradients now averaged in place
            self.opt_graph = torch.cuda.CUDAGraph()
            pool = self.graph.pool() if os.environ.get("MMAD_GRAPH_SHARE_POOL", "1") != "0" else None
            with torch.cuda.graph(self.opt_graph, pool=pool):
                optimizer.step()
        else:
            with torch.cuda.graph(self.graph):
                self.out = model.general_step(self.static, 0, "train")
                self.out["loss"].backward()
                if reducer is not None:
                    reducer.finish()
                if os.environ.get("MMAD_GRAPH_DEBUG", "") != "noopt":
                    optimizer.step()
        # keep the graph-owned output buffers, not their autograd graph: a live grad_fn chain
        # would keep every parameter's AccumulateGrad node (created on the capture stream)
        # alive, and later eager steps would reuse those nodes across streams
        self.out = {k: v.detach() if torch.is_tensor(v) else v for k, v in self.out.items()}

    def static_device(self):
        return next(self.model.parameters()).device

    def _eager(self):
        self.optimizer.zero_grad(set_to_none=True)
        if self.reducer is not None:
            self.reducer.defer = self.after
        try:
            self.model.general_step(self.static, 0, "train")["loss"].backward()
            if self.reducer is not None:
                self.reducer.finish()
        finally:
            if self.reducer is not None:
                self.reducer.defer = False
        self.optimizer.step()

    def __call__(self, batch=None):
        """Replay one step; ``batch`` (same keys / shapes) is copied into the graph's input
        buffers first.  Returns the step's {'loss', 'outputs', 'labels'} (graph-owned
        tensors, overwritten by the next replay)."""
        if batch is not None:
            for k, v in batch.items():
                if torch.is_tensor(v):
                    self.static[k].copy_(v, non_blocking=True)
        self.graph.replay()
        if self.after:
            if self.finish_events is not None:
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
            self.reducer.finish()            # no hook ran in the replay: launches every bucket
            if self.finish_events is not None:
                e1.record()
                self.finish_events.append((e0, e1))
            self.opt_graph.replay()
        volume_ops._BN_UPDATES[0] += 1     # weights / running stats changed on the device
        return self.out
