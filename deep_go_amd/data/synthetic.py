"""Synthetic 19x19 positions (BASELINE.json: "synthetic 19x19 boards / random-init weights").

Two generators:

* ``random_planes`` — fast numpy boards with plausible stored-plane statistics (stones,
  liberties, liberties-after, kills, age, ladders); labels are empty points.  Used by the
  throughput benchmark, where only the tensor shapes/sparsity matter.
* ``engine_positions`` — positions from random self-play games through the C++ Go
  engine (csrc/engine), so every feature plane is rule-consistent.  Used by the
  loader tests and the real-data style pipeline.
"""
from __future__ import annotations

import numpy as np

BOARD = 19


def random_planes(n: int, seed: int = 0, fill: float = 0.45):
    rng = np.random.default_rng(seed)
    planes = np.zeros((n, 9, BOARD, BOARD), np.uint8)
    st = rng.choice(3, size=(n, BOARD, BOARD), p=[1 - fill, fill / 2, fill / 2]).astype(np.uint8)
    planes[:, 0] = st
    occ = st > 0
    planes[:, 1] = np.where(occ, rng.integers(1, 9, (n, BOARD, BOARD)), 0)
    for c in (2, 3):
        planes[:, c] = np.where(occ, 0, rng.integers(0, 9, (n, BOARD, BOARD)))
    for c in (4, 5):
        k = rng.random((n, BOARD, BOARD)) < 0.02
        planes[:, c] = np.where(~occ & k, rng.integers(1, 9, (n, BOARD, BOARD)), 0)
    age = rng.integers(0, 256, (n, BOARD, BOARD))
    planes[:, 6] = np.where(occ | (rng.random((n, BOARD, BOARD)) < 0.1), age, 0)
    for c in (7, 8):
        k = rng.random((n, BOARD, BOARD)) < 0.005
        planes[:, c] = np.where(~occ & k, rng.integers(1, 6, (n, BOARD, BOARD)), 0)
    player = rng.integers(1, 3, n).astype(np.uint8)
    rank = rng.integers(1, 10, n).astype(np.uint8)
    labels = np.zeros(n, np.int32)
    flat = st.reshape(n, -1)
    for i in range(n):
        empty = np.flatnonzero(flat[i] == 0)
        labels[i] = rng.choice(empty) if len(empty) else 0
    return planes, player, rank, labels


def engine_positions(n: int, seed: int = 0, max_moves: int = 250):
    """Rule-consistent positions from random games played by the C++ engine."""
    from ..ops.native import cpu
    eng = cpu()
    planes, player, rank, labels = eng.random_positions(n, seed, max_moves)
    return (np.asarray(planes), np.asarray(player), np.asarray(rank), np.asarray(labels))
