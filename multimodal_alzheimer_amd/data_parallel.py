"""Data parallelism for the 3D-volume training step: one process per GPU, RCCL over xGMI.

The reference trains on one GPU (``pl.Trainer(devices=1)``, train_anat_cnn.py) and has no
collective at all; this is new work.  Samples (single volumes or PET-MRI pairs / triples
merged by MultiModalDataset, pkg/utils/dataloader.py:124-156) are independent, so the
only exchange per step is the gradient all-reduce:

* ``shard_indices`` -- DistributedSampler-style sharding of the sample-pair index list
  (seeded shuffle per epoch, equal shard sizes by padding with wrap-around samples);
* ``GradAllReduce`` -- gradient buckets (``bucket_mb``, reverse registration order so the
  last layers' gradients, ready first in backward, go first; or one bucket per backward
  stage, ``stages=``) all-reduced asynchronously -- from post-accumulate-grad hooks while an
  eager backward continues, or per stage between the replayed backward graphs
  (graph_step ``collectives="staged"``); ``finish()`` reduces what is left on the current
  stream (synchronous collective: no cross-stream hop), waits for the rest, averages and
  writes the reduced gradients back.

BN batch statistics are per replica (each rank normalises its own shard, as DDP without
SyncBatchNorm).  The running statistics: DDP's default ``broadcast_buffers=True`` copies
rank 0's buffers to every rank before each forward; ``broadcast_module_state(model,
buffers_only=True)`` once per step does the same here (bench.py does not call it: ranks'
running statistics then drift apart, which changes nothing in training mode and only
matters for evaluating on a rank other than 0).

Backend "nccl" is RCCL on ROCm; "gloo" runs the same code on CPU for the tests.
"""
import os

import torch
import torch.distributed as dist
from torch.autograd.graph import increment_version


def shard_indices(n_samples, rank, world, epoch=0, shuffle=True, seed=15):
    """Indices of this rank's shard (torch DistributedSampler semantics, drop_last=False)."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        order = torch.randperm(n_samples, generator=g).tolist()
    else:
        order = list(range(n_samples))
    per = -(-n_samples // world)
    total = per * world
    order += order[: total - n_samples] if total > n_samples else []
    return order[rank:total:world]


class ShardSampler(torch.utils.data.Sampler):
    """This rank's shard of a dataset's samples -- for ``dataset.MultiModalDataset`` the
    merged PET/MRI/tabular pairs and triples -- as a DataLoader sampler
    (DistributedSampler semantics via ``shard_indices``); ``set_epoch`` reshuffles."""

    def __init__(self, dataset, rank=None, world=None, shuffle=True, seed=15):
        self.n = len(dataset)
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        self.shuffle, self.seed, self.epoch = shuffle, seed, 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        return iter(shard_indices(self.n, self.rank, self.world, self.epoch, self.shuffle,
                                  self.seed))

    def __len__(self):
        return -(-self.n // self.world)


def broadcast_module_state(module, src=0, group=None, buffers_only=False):
    """Every rank takes rank ``src``'s parameters and buffers (BN running statistics,
    num_batches_tracked), as DDP does at construction; ``buffers_only`` re-syncs just the
    buffers, as DDP's ``broadcast_buffers=True`` does before every forward."""
    ts = list(module.buffers()) if buffers_only else \
        list(module.parameters()) + list(module.buffers())
    with torch.no_grad():
        for t in ts:
            dist.broadcast(t.data, src=src, group=group)
            # a write through .data leaves the version counter alone; bump it so consumers
            # that cache derived layouts (graph_step's packed bf16 weights) see the change
            increment_version(t)


# MMAD_DP_GRAD_SLOTS=0: conv weight gradients go to fresh tensors and are copied into the
# buckets like the BN / head gradients (A/B switch for the in-place bucket slots)
_GRAD_SLOTS = os.environ.get("MMAD_DP_GRAD_SLOTS", "1") != "0"


_SLICE_ALIGN = 256   # bytes


def _aligned(numel, elsize):
    step = max(1, _SLICE_ALIGN // elsize)
    return -(-numel // step) * step


def _split(params, cap):
    out, cur, size = [], [], 0
    for p in params:
        cur.append(p)
        size += p.numel() * p.element_size()
        if size >= cap:
            out.append(cur)
            cur, size = [], 0
    if cur:
        out.append(cur)
    return out


class GradAllReduce:
    def __init__(self, params, bucket_mb=32.0, group=None, stages=None):
        """``stages``: optional list of parameter lists in the order backward completes them
        (graph_step.backward_stages); each stage is cut into buckets of ``bucket_mb``
        (``None``: one bucket per stage) and ``launch_stage(k)`` starts stage k's buckets.
        Without it the parameters are bucketed in reverse registration order."""
        self.group = group
        self.world = dist.get_world_size(group)
        # RCCL averages in the collective itself (ncclAvg); gloo has no AVG: sum, then scale
        self._avg = dist.get_backend(group) == "nccl"
        self._op = dist.ReduceOp.AVG if self._avg else dist.ReduceOp.SUM
        self.params = [p for p in params if p.requires_grad]
        cap = float("inf") if bucket_mb is None else int(bucket_mb * (1 << 20))
        self.stage_buckets = None
        if stages is None:
            # backward produces the last layers first
            self.buckets = _split(list(reversed(self.params)), cap)
        else:
            mine = set(self.params)
            staged = [[p for p in st if p in mine] for st in stages]
            seen = [p for st in staged for p in st]
            if len(seen) != len(set(seen)) or set(seen) != mine:
                raise ValueError("stages must partition the trainable parameters")
            self.buckets, self.stage_buckets = [], []
            for st in staged:
                bs = _split(st, cap) if st else []
                self.stage_buckets.append(list(range(len(self.buckets),
                                                     len(self.buckets) + len(bs))))
                self.buckets += bs
        self._owner = {}
        for bi, b in enumerate(self.buckets):
            for p in b:
                self._owner[p] = bi
        # Persistent flat buffer per bucket; each parameter's slice is offered to the conv
        # backward as its weight-gradient destination (``p._mmad_grad_view``), so the big
        # conv gradients are produced in place: no gather before the collective and no
        # copy back after it.  Gradients produced elsewhere (BN, head) are copied in/out.
        # Every slice starts on a 256-byte boundary: an odd-sized tensor (the head's 2-float
        # bias) must not shift the slices behind it, or torch's fused Adam sees one
        # unaligned gradient and drops to its scalar path for all of them (measured 118 vs
        # 64 us per step on MI355X), and the collective runs on unaligned rows.  The pad
        # lanes are zeros and stay zeros (sum / mean of zeros).
        self.flats = []
        self._views = {}
        for b in self.buckets:
            offs, off = [], 0
            for p in b:
                offs.append(off)
                off += _aligned(p.numel(), p.element_size())
            flat = torch.zeros(off, dtype=b[0].dtype, device=b[0].device)
            for p, o in zip(b, offs):
                self._views[p] = flat[o:o + p.numel()].view_as(p)
                if _GRAD_SLOTS:
                    p._mmad_grad_view = self._views[p]
            self.flats.append(flat)
        self._hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        # defer: the hooks only count; finish() launches every bucket.  Set while a step's
        # forward + backward is captured without its collectives (graph_step
        # collectives="after"): a replay runs no Python hooks, so finish() does it all.
        self.defer = False
        # buckets still unlaunched when finish() runs (the last backward stage's; every
        # bucket in collectives="after") are all-reduced synchronously on the current stream:
        # a blocking ProcessGroupNCCL collective runs on the caller's stream, an async one on
        # the group's internal stream behind two cross-stream waits (tools/ar_latency.py, one
        # RCCL rank: 17 vs 37 us per critical-path all-reduce)
        self.inline_tail = True
        self.reset()

    def reset(self):
        self._pending = [len(b) for b in self.buckets]
        self._inflight = {}

    def _ready(self, p):
        bi = self._owner[p]
        self._pending[bi] -= 1
        if self._pending[bi] == 0 and not self.defer:
            self._launch(bi)

    def _foreign(self, bi):
        """(grads, views) of the bucket's parameters whose .grad is not their slice."""
        pairs = [(p.grad, self._views[p]) for p in self.buckets[bi]
                 if p.grad.data_ptr() != self._views[p].data_ptr()]
        return [g for g, _ in pairs], [v for _, v in pairs]

    def _launch(self, bi, inline=False):
        flat = self.flats[bi]
        for p in self.buckets[bi]:
            if p.grad is None:                   # unused this step: contributes zeros
                p.grad = torch.zeros_like(p)
        grads, views = self._foreign(bi)
        if inline:
            if grads:
                torch._foreach_copy_(views, grads)
            dist.all_reduce(flat, op=self._op, group=self.group)
            if not self._avg:
                flat.div_(self.world)
            self._inflight[bi] = None            # done (on the current stream)
            return
        if flat.is_cuda:
            # conv weight gradients may come from volume_ops' side stream (the backward
            # pass joins it only at its end): gather and reduce there, after the main
            # stream's gradients (BN, head) too, so the collective overlaps the rest of
            # the backward without waiting for it
            from .volume_ops import grad_stream
            main = torch.cuda.current_stream()
            side = grad_stream(flat.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                if grads:
                    torch._foreach_copy_(views, grads)
                work = dist.all_reduce(flat, op=self._op, group=self.group, async_op=True)
        else:
            if grads:
                torch._foreach_copy_(views, grads)
            work = dist.all_reduce(flat, op=self._op, group=self.group, async_op=True)
        self._inflight[bi] = work

    def launch_stage(self, k):
        """Start the all-reduce of backward stage k's buckets (their gradients are complete
        on the current stream): on the side stream, overlapping whatever the current stream
        runs next."""
        for bi in self.stage_buckets[k]:
            if bi not in self._inflight:
                self._launch(bi)

    def finish(self):
        """Wait for every bucket (launching any whose grads never all arrived), then
        make every parameter's grad the mean over ranks."""
        cuda = bool(self.params) and self.params[0].is_cuda
        inline = self.inline_tail and not (cuda and torch.cuda.is_current_stream_capturing())
        for bi, b in enumerate(self.buckets):
            if bi not in self._inflight:
                self._launch(bi, inline=inline)
        if cuda and any(w is not None for w in self._inflight.values()):
            from .volume_ops import grad_stream
            torch.cuda.current_stream().wait_stream(grad_stream(self.params[0].device))
        for bi, work in sorted(self._inflight.items()):
            if work is not None:
                work.wait()
                if not self._avg:
                    self.flats[bi].div_(self.world)
            grads, views = self._foreign(bi)
            if grads:
                # one multi-tensor launch per bucket, not one copy kernel per parameter
                torch._foreach_copy_(grads, views)
        self.reset()

    def remove(self):
        for h in self._hooks:
            h.remove()
