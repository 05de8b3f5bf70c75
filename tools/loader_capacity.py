"""8-rank input-pipeline capacity (CPU only): P concurrent processes, each with its own
BatchLoader (as one rank per GPU would run), on the packed fixture (tests/fixtures) tiled up
to N positions; reports per-rank and aggregate boards/s and CPU use.

At 8 ranks x ~280k boards/s the host must deliver ~2.3M boards/s.  Each rank's stream is
deterministic (seed, batch number) whatever the thread count (tests/test_data.py).

usage: python tools/loader_capacity.py [--ranks 8] [--threads 2] [--batches 400] [--batch 256]
Reference: the 32-thread Lua loader pool (data.lua:11-27).
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _rank(r, args, q):
    import numpy as np
    import torch
    torch.set_num_threads(1)
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    pk = PackedDataset.load(os.path.join(ROOT, "tests", "fixtures", "train.dgpack.npz"))
    if args.tile > 1:   # a bigger working set than the 4k-position fixture (cache behaviour)
        n = len(pk)
        pk = PackedDataset(np.tile(pk.planes, (args.tile, 1, 1, 1)), np.tile(pk.player, args.tile),
                           np.tile(pk.rank, args.tile), np.tile(pk.label, args.tile),
                           np.concatenate([pk.game_start + k * n for k in range(args.tile)]),
                           np.tile(pk.game_count, args.tile))
    ld = BatchLoader(pk, args.batch, threads=args.threads, prefetch=args.prefetch,
                     seed=1000 + r, pin=False)
    dst = torch.empty(ld.packed.shape[1], dtype=torch.uint8)
    for _ in range(20):
        ld.next_packed_to(dst)
    q.put(("ready", r))
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(args.batches):
        ld.next_packed_to(dst)
    dt = time.perf_counter() - t0
    cpu = time.process_time() - c0
    ld.close()
    q.put(("done", r, args.batches * args.batch / dt, cpu / dt))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--threads", type=int, default=2)
    ap.add_argument("--prefetch", type=int, default=6)
    ap.add_argument("--batches", type=int, default=400)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--tile", type=int, default=16)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, args, q)) for r in range(args.ranks)]
    t0 = time.perf_counter()
    for p in ps:
        p.start()
    res = []
    while len(res) < args.ranks:
        m = q.get()
        if m[0] == "done":
            res.append(m)
    for p in ps:
        p.join()
    rates = [m[2] for m in res]
    out = {"ranks": args.ranks, "threads_per_rank": args.threads, "batch": args.batch,
           "positions": 4139 * args.tile, "host_cpus": os.cpu_count(),
           "per_rank_boards_s_min": round(min(rates)), "per_rank_boards_s_max": round(max(rates)),
           "aggregate_boards_s": round(sum(rates)),
           "cpu_cores_busy_per_rank": round(sum(m[3] for m in res) / len(res), 2),
           "wall_s": round(time.perf_counter() - t0, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
