"""Feature-plane specification: 9 stored uint8 planes -> 37 network input planes (38 with
the optional simple-ko plane).

Stored planes (``dataloader.lua:20-27``, written by ``flatten_data`` ``:30-39``), index
``[plane][x][y]`` with x = first SGF coordinate:
  0 stones (0 empty / 1 black / 2 white), 1 group liberties, 2-3 liberties_after[black,
  white], 4-5 kills[black, white], 6 age, 7-8 ladders[black, white].

Network planes (``preprocess``, ``dataloader.lua:50-92``), relative to the player p to move:
  0 empty, 1 stone of p, 2 opponent stone, 3-5 liberties == 1..3, 6 liberties >= 4,
  7 empty & liberties_after[p] == 0, 8-12 liberties_after[p] == 1..5, 13 >= 6,
  14-19 kills[p] == 1..6, 20 kills[p] >= 7, 21-25 age == 1..5, 26 ladder[p] >= 1,
  27 always zero (the reference's off-by-one rank offset), 28-36 rank of p == 1..9 dan.
  37 (optional, ``ExperimentConfig.ko_plane``): the simple-ko point — an addition, the
  reference tracks no ko.  It rides in stored plane 1 as ``KO_MARK`` at an EMPTY point (plane 1
  is 0 at empty points otherwise; ``makedata --ko`` writes it), so the liberty planes 3-6 are
  gated on a stone (identical on files without the mark).
Label = 19*x0 + y0 (``dataloader.lua:89``).

This numpy version is the CPU oracle; the GPU path is ``expand_features_kernel``
(csrc/kernels/elementwise.hip) and the threaded loader uses the C++ version
(csrc/engine/features.cpp).
"""
from __future__ import annotations

import numpy as np

NUM_PLANES = 37
NUM_PLANES_KO = 38
KO_MARK = 255     # csrc/engine/go_engine.h
BOARD = 19


def expand(planes: np.ndarray, player: int, rank: int, out: np.ndarray | None = None,
           ko: bool = False) -> np.ndarray:
    """planes uint8 [9,19,19] -> float32 [37,19,19] ([38,19,19] with ko)."""
    p = int(player)
    st = planes[0]
    lib = np.where(planes[0] != 0, planes[1], 0)
    la = planes[2 + (p - 1)]
    kill = planes[4 + (p - 1)]
    age = planes[6]
    lad = planes[7 + (p - 1)]
    n = NUM_PLANES_KO if ko else NUM_PLANES
    x = out if out is not None else np.zeros((n, BOARD, BOARD), np.float32)
    x[:] = 0
    x[0] = st == 0
    x[1] = st == p
    x[2] = st == 3 - p
    for i in range(1, 4):
        x[2 + i] = lib == i
    x[6] = lib >= 4
    x[7] = (st == 0) & (la == 0)
    for i in range(1, 6):
        x[7 + i] = la == i
    x[13] = la >= 6
    for i in range(1, 7):
        x[13 + i] = kill == i
    x[20] = kill >= 7
    for i in range(1, 6):
        x[20 + i] = age == i
    x[26] = lad >= 1
    if 1 <= rank <= 9:
        x[27 + rank] = 1.0
    if ko:
        x[37] = (st == 0) & (planes[1] == KO_MARK)
    return x


def expand_batch(planes: np.ndarray, player: np.ndarray, rank: np.ndarray,
                 ko: bool = False) -> np.ndarray:
    B = planes.shape[0]
    out = np.zeros((B, NUM_PLANES_KO if ko else NUM_PLANES, BOARD, BOARD), np.float32)
    for b in range(B):
        expand(planes[b], int(player[b]), int(rank[b]), out[b], ko)
    return out


def label_of(x: int, y: int) -> int:
    """1-based SGF coords -> 0-based class 19*(x-1) + (y-1)."""
    return BOARD * (x - 1) + (y - 1)
