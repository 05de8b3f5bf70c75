"""Packed single-copy batch layout shared by the loader's pinned ring slots and HipGoNet's
input buffer: [planes B*9*361 u8 | player B u8 | rank B u8 | pad to 4 | labels B i32].
One batch is then ONE host-to-device (or device-to-device) copy."""
from __future__ import annotations

import torch

from ..config import NUM_POINTS


def packed_batch_bytes(B: int) -> int:
    n = B * 9 * NUM_POINTS + 2 * B
    return n + (-n % 4) + 4 * B


def unpack_views(buf: torch.Tensor, B: int):
    """(planes [B,9,361] u8, player [B] u8, rank [B] u8, labels [B] i32) views of a packed
    batch buffer (labels 4-byte aligned)."""
    n = B * 9 * NUM_POINTS
    planes = buf[:n].view(B, 9, NUM_POINTS)
    player = buf[n:n + B]
    rank = buf[n + B:n + 2 * B]
    lo = n + 2 * B
    lo += -lo % 4
    labels = buf[lo:lo + 4 * B].view(torch.int32)
    return planes, player, rank, labels


def pack_batch(planes, player, rank, labels, device=None) -> torch.Tensor:
    """Pack one batch (numpy arrays or tensors) into the HipGoNet input layout."""
    def t(x, dt):
        x = torch.as_tensor(x)
        return x.to(dt)
    planes = t(planes, torch.uint8)
    B = planes.shape[0]
    buf = torch.zeros(packed_batch_bytes(B), dtype=torch.uint8, device=device or planes.device)
    p, pl, rk, lb = unpack_views(buf, B)
    p.copy_(planes.reshape(B, 9, NUM_POINTS))
    pl.copy_(t(player, torch.uint8))
    rk.copy_(t(rank, torch.uint8))
    lb.copy_(t(labels, torch.int32))
    return buf
