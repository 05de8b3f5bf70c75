"""Offline data preparation (the reference's makedata.lua, run from a Torch REPL there).

* ``scatter(src, dst, {"train": n, ...}, seed)``  — shuffle raw SGF files and copy them into
  ``dst/<split>/<subdir>/`` (``scatter_to_categories``, makedata.lua:580-598); the shuffle is
  seeded (the reference used Lua's unseeded math.random).
* ``transcribe(src_split_dir, dst_split_dir, threads)`` — parallel SGF -> per-position t7
  files ``<dst>/<subdir>/<game>.sgf/<k>`` (``transcribe_in_parallel``, :506-533) on the C++
  thread pool; games whose ranks are not both dan are dropped; finished games are skipped on
  re-runs (done marker, the reference's "file 100 exists").  ``mark_ko`` (an addition, off by
  default) marks each position's simple-ko point in the stored liberty plane for models built
  with ``ko_plane=1`` (data/features.py).
* ``count(root, split)`` — the ``count_game_moves.sh`` index.
* ``pack(root, split)`` — packed ``<root>/<split>.dgpack.npz`` for fast training.
"""
from __future__ import annotations

import os
import random
import shutil
from pathlib import Path
from typing import Dict

from ..ops.native import cpu
from .dataset import PackedDataset, load_index, write_counts


def all_files(d: str):
    return sorted(str(p) for p in Path(d).rglob("*") if p.is_file())


def scatter(src: str, dst: str, categories: Dict[str, int], seed: int = 0) -> Dict[str, int]:
    files = all_files(src)
    random.Random(seed).shuffle(files)
    out = {}
    i = 0
    for cat, size in categories.items():
        n = 0
        for _ in range(size):
            if i >= len(files):
                break
            f = files[i]
            i += 1
            rel = os.path.relpath(f, src)
            target = os.path.join(dst, cat, rel)
            os.makedirs(os.path.dirname(target), exist_ok=True)
            shutil.copyfile(f, target)
            n += 1
        out[cat] = n
    return out


def transcribe(src: str, dst: str, threads: int = 32, skip_done: bool = True,
               mark_ko: bool = False) -> Dict[str, int]:
    jobs = []
    for f in all_files(src):
        rel = os.path.relpath(f, src)
        jobs.append((f, os.path.join(dst, rel)))
    res = cpu().transcribe_files(jobs, threads, skip_done, mark_ko)
    stats = {"games": len(jobs), "written": sum(1 for r in res if r > 0),
             "positions": sum(r for r in res if r > 0), "dropped_no_dan": res.count(0),
             "illegal": res.count(-1), "skipped_done": res.count(-2), "io_errors": res.count(-3)}
    return stats


def count(root: str, split: str) -> str:
    return str(write_counts(root, split))


def pack(root: str, split: str, threads: int = 8) -> str:
    idx = load_index(root, split)
    out = os.path.join(root, f"{split}.dgpack.npz")
    PackedDataset.from_index(idx, threads).save(out)
    return out
