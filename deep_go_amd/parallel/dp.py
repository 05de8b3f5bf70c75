"""Data parallelism: one process per GPU, RCCL (torch.distributed "nccl") over xGMI.

Reference: ``makeDataParallel`` wraps the model in a single-process
``nn.DataParallelTable`` that scatters the batch, gathers outputs to GPU 1, reduces
gradients into GPU 1 and broadcasts parameters back (``experiments.lua:155-168``; never
enabled by a committed config).  Here instead:

* every rank holds a full replica and its own ``batch / world`` slice;
* parameters are broadcast once from rank 0 at start (identical init everywhere);
* gradients are all-reduced (SUM; the head kernel already scales by 1/global_batch, so the
  sum IS the global-batch mean) in **buckets** of contiguous layer ranges of the flat
  gradient buffer, last layer first, each launched as soon as that layer's wgrad has
  finished, so communication of late layers overlaps the backward of earlier ones;
* the per-step launch sequence between collectives is captured into hipGraphs
  ("segments"), and the collectives are issued between segment replays — RCCL runs on
  its own stream, ordered against the compute stream by events.

Bucket sizing for xGMI: each MI355X has 7 point-to-point links (~153 GB/s each); a ring
all-reduce of S bytes costs about 2(n-1)/n * S / link_bw, so 4 MB buckets are ~50 us on
8 GPUs — small enough to overlap 2-3 layers' backward, large enough to stay off the
latency floor.  ``grad_dtype="bf16"`` halves the bytes (rounding documented in tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_info() -> DistInfo:
    return DistInfo(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                    int(os.environ.get("LOCAL_RANK", 0)))


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> DistInfo:
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT.

    backend "nccl" is RCCL on ROCm.  No-op (world=1) when WORLD_SIZE is unset/1."""
    import datetime
    info = env_info()
    if info.world <= 1:
        return info
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(info.local_rank)
            kw["device_id"] = torch.device("cuda", info.local_rank)
        dist.init_process_group(backend=backend, rank=info.rank, world_size=info.world,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return info


def make_buckets(layer_ranges: Sequence[Tuple[int, int]], bucket_bytes: int,
                 elem_size: int = 4,
                 groups: Optional[Sequence[Sequence[int]]] = None) -> List[Tuple[int, int, int]]:
    """Group layers (given as [start, end) element ranges in flat order) into buckets,
    walking from the LAST layer backwards (the order gradients become final).

    ``groups``: layers whose gradients become final together (HipGoNet.wgroups: one
    grouped weight-gradient launch, listed top layer first); a group is never split
    across buckets and is ready at its top layer.

    Returns a list of (start, end, ready_layer) in firing order: the bucket's gradients
    are final after ``backward_layer(ready_layer)`` (without groups: its lowest layer)."""
    top_of = {}
    for g in groups or ():
        for i in g:
            top_of[i] = max(g)
    buckets = []
    cur_start = cur_end = None
    cur_ready = None
    i = len(layer_ranges) - 1
    while i >= 0:
        # one unit: a whole group (contiguous layers lo..top) or a single layer
        top = i
        lo = i
        if i in top_of:
            lo = min(j for j, t in top_of.items() if t == top_of[i])
        s, e = layer_ranges[lo][0], layer_ranges[top][1]
        if cur_end is None:
            cur_start, cur_end = s, e
        else:
            cur_start = s
        cur_ready = top_of.get(lo, lo)
        if (cur_end - cur_start) * elem_size >= bucket_bytes:
            buckets.append((cur_start, cur_end, cur_ready))
            cur_start = cur_end = None
        i = lo - 1
    if cur_end is not None:
        buckets.append((cur_start, cur_end, cur_ready))
    return buckets


class GradBucketer:
    """Issues async all-reduces of flat-gradient buckets; ``wait()`` joins them all."""

    def __init__(self, grads: torch.Tensor, buckets: List[Tuple[int, int, int]],
                 group=None, grad_dtype: str = "fp32"):
        self.grads = grads
        self.buckets = buckets
        self.group = group
        self.grad_dtype = grad_dtype
        self.works = []
        self._shadow = None
        if grad_dtype == "bf16":
            self._shadow = torch.empty(grads.numel(), dtype=torch.bfloat16, device=grads.device)

    def fire(self, b: int):
        s, e, _ = self.buckets[b]
        if self._shadow is not None:
            sh = self._shadow[s:e]
            sh.copy_(self.grads[s:e])
            self.works.append((dist.all_reduce(sh, group=self.group, async_op=True), b))
        else:
            self.works.append((dist.all_reduce(self.grads[s:e], group=self.group,
                                               async_op=True), b))

    def wait(self):
        for w, b in self.works:
            w.wait()
            if self._shadow is not None:
                s, e, _ = self.buckets[b]
                self.grads[s:e].copy_(self._shadow[s:e])
        self.works = []


def all_reduce_scalars(vals: Sequence[float], device=None, op=None) -> List[float]:
    """Sum a few scalars across ranks (validation cost / errors / count)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return list(vals)
    t = torch.tensor(list(vals), dtype=torch.float64, device=device)
    dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t.tolist()


def broadcast_(t: torch.Tensor, src: int = 0):
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast(t, src)
    return t


def barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()
