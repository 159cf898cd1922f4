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
"""
import torch


class GraphedTrainStep:
    def __init__(self, model, optimizer, batch, warmup=3):
        self.model, self.optimizer = model, optimizer
        self.static = {k: v.clone() if torch.is_tensor(v) else v for k, v in batch.items()}
        for g in optimizer.param_groups:
            g["capturable"] = True
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._eager()
        torch.cuda.current_stream().wait_stream(side)
        optimizer.zero_grad(set_to_none=True)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = model.general_step(self.static, 0, "train")
            self.out["loss"].backward()
            optimizer.step()

    def _eager(self):
        self.optimizer.zero_grad(set_to_none=True)
        self.model.general_step(self.static, 0, "train")["loss"].backward()
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
        return self.out
