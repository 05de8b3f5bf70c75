"""Prefetching batch loader: Python face of the C++ ring loader (csrc/engine/loader.cpp).

Replaces the reference's 32 Lua worker threads + ``threads.sharedserialize`` hand-off
(``data.lua:11-27,82-96``).  Workers fill a ring of pinned host slots with compact uint8
batches (3.2 KB/board instead of the reference's 106 KB float64); the consumer copies a
slot to the GPU asynchronously and releases it once that copy has completed (tracked with a
HIP event, so a slot is never refilled while its DMA is in flight).
"""
from __future__ import annotations

import time
from typing import Optional

import numpy as np
import torch

from ..ops.native import cpu
from .batch import packed_batch_bytes, unpack_views
from .dataset import GameIndex, PackedDataset


class BatchLoader:
    def __init__(self, source, batch: int, threads: int = 8, prefetch: int = 4, seed: int = 0,
                 sampling: str = "game", pin: Optional[bool] = None, start_seq: int = 0):
        if prefetch < 2:
            raise ValueError("prefetch must be >= 2")
        self.batch = batch
        self.prefetch = prefetch
        pin = torch.cuda.is_available() if pin is None else pin
        B = batch
        # ring slots in the packed layout (data/batch.py): a slot goes to the GPU in ONE
        # async copy (next_packed_to); the named views are what the C++ workers fill
        self.packed = torch.zeros((prefetch, packed_batch_bytes(B)), dtype=torch.uint8,
                                  pin_memory=pin)
        views = [unpack_views(self.packed[i], B) for i in range(prefetch)]
        self.planes = [v[0] for v in views]
        self.player = [v[1] for v in views]
        self.rank = [v[2] for v in views]
        self.label = [v[3] for v in views]
        slots = [(v[0].data_ptr(), v[1].data_ptr(), v[2].data_ptr(), v[3].data_ptr())
                 for v in views]
        self._keep = None
        if isinstance(source, PackedDataset):
            self._keep = source  # arrays must outlive the C++ loader
            games = source.game_refs()
            pk = (source.planes.ctypes.data, source.player.ctypes.data, source.rank.ctypes.data,
                  source.label.ctypes.data)
        elif isinstance(source, GameIndex):
            games = [(d, 0, n) for d, n in source.games]
            pk = (0, 0, 0, 0)
        else:
            raise TypeError("source must be a GameIndex or PackedDataset")
        self._impl = cpu().Loader(games, B, threads, slots, int(seed) & (2 ** 64 - 1),
                                  sampling == "position", *pk, int(start_seq))
        self.consumed = int(start_seq)
        self._pending = []  # (slot, event) awaiting release
        self.wait_s = 0.0   # host time spent blocked on the workers (next_host)

    def next_host(self):
        """Blocks until the next batch is ready; returns (slot, seq) — caller releases."""
        t0 = time.perf_counter()
        slot, seq = self._impl.next()
        self.wait_s += time.perf_counter() - t0
        if slot < 0:
            raise RuntimeError("loader stopped")
        self.consumed = seq + 1
        return slot, seq

    def release(self, slot: int):
        self._impl.release(slot)

    def _reap(self, block: bool = False):
        keep = []
        for slot, ev in self._pending:
            if ev is None or block or ev.query():
                if ev is not None and block:
                    ev.synchronize()
                self._impl.release(slot)
            else:
                keep.append((slot, ev))
        # slots held by in-flight copies cannot be refilled: bound them (oldest first) so the
        # workers always have free slots and next_host() cannot wait on a slot only we hold
        while len(keep) > max(1, self.prefetch - 2):
            slot, ev = keep.pop(0)
            ev.synchronize()
            self._impl.release(slot)
        self._pending = keep

    def next_to(self, planes: torch.Tensor, player: torch.Tensor, rank: torch.Tensor,
                labels: torch.Tensor):
        """Asynchronously copy the next batch into (device) tensors on the current stream."""
        self._reap()
        slot, seq = self.next_host()
        planes.copy_(self.planes[slot].reshape(planes.shape), non_blocking=True)
        player.copy_(self.player[slot], non_blocking=True)
        rank.copy_(self.rank[slot], non_blocking=True)
        labels.copy_(self.label[slot].to(labels.dtype) if labels.dtype != torch.int32
                     else self.label[slot], non_blocking=True)
        ev = None
        if planes.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        else:
            self._impl.release(slot)
            return seq
        self._pending.append((slot, ev))
        return seq

    def next_packed_to(self, dst: torch.Tensor) -> int:
        """One asynchronous copy of the next packed batch into ``dst`` (e.g. HipGoNet.inbuf)
        on the current stream; the slot is released once that copy has completed."""
        self._reap()
        slot, seq = self.next_host()
        dst.copy_(self.packed[slot], non_blocking=True)
        if dst.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self._pending.append((slot, ev))
        else:
            self._impl.release(slot)
        return seq

    def next_numpy(self):
        """Copy the next batch out as numpy arrays (CPU path / tools)."""
        slot, seq = self.next_host()
        B = self.batch
        out = (self.planes[slot].numpy().reshape(B, 9, 19, 19).copy(),
               self.player[slot].numpy().copy(), self.rank[slot].numpy().copy(),
               self.label[slot].numpy().copy())
        self._impl.release(slot)
        return out

    def errors(self) -> int:
        return self._impl.errors()

    def close(self):
        self._reap(block=True)
        self._impl.stop()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
