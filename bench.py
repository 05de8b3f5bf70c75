#!/usr/bin/env python3
"""Headline benchmark: board-positions/sec for the 12-layer d=128 GoCNN training step.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is
launched by torch.distributed.run with one rank per GPU (RCCL over xGMI).  W untimed
warmup steps, then EXACTLY K timed steps bracketed by barrier + device sync on both sides;
the max over ranks is used and rank 0 prints ONE JSON line.

What one step is (nothing skipped inside the timed region):
  next batch (uint8 planes/labels) copied into the static input buffers ->
  GPU feature expansion -> 11 conv layers fwd -> fused head (loss, argmax, head bwd) ->
  bias-grad + wgrad + dgrad for every layer -> [N>1: bucketed RCCL all-reduce overlapped
  with backward] -> SGD with per-step LR decay -> bf16 weight refresh.
Weak scaling: 256 boards per GPU per step (BASELINE.json config "12-layer d=128 CNN bf16
on one MI355X, batch=256"; global batch = 256*N).  Synthetic 19x19 positions, random-init
weights (BASELINE.json: no datasets/checkpoints available).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

METRIC = "board-positions/sec (whole node) 12-layer d=128 CNN; top-1 move accuracy"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--pool", type=int, default=16, help="distinct synthetic batches")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--bucket-mb", type=float, default=3.0,
                    help="DP gradient bucket size (3 MB: head + one 5-layer wgrad group)")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--profile", type=int, default=0, metavar="N",
                    help="after the timed run, N extra steps with roctx ranges (load / segments"
                         " / allreduce / optimizer) and a host phase breakdown; run under "
                         "rocprofv3 --marker-trace --kernel-trace to see them on the timeline")
    ap.add_argument("--force-dp", action="store_true",
                    help="use the DP path (RCCL process group, bucketed all-reduces between "
                         "graph segments) even on 1 GPU: measures its overhead")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: hidden-layer forwards on e4m3 MX-MFMA (BASELINE config 5)")
    args = ap.parse_args()

    import torch
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from deep_go_amd.config import get_preset
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp

    info = dp.init_distributed()
    world = info.world
    if args.force_dp and world == 1 and not torch.distributed.is_initialized():
        import socket
        sk = socket.socket()
        sk.bind(("127.0.0.1", 0))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(sk.getsockname()[1]))
        sk.close()
        torch.distributed.init_process_group("nccl", rank=0, world_size=1,
                                             device_id=torch.device("cuda", 0))
    if world > 1:
        torch.cuda.set_device(info.local_rank)
    dev = torch.device("cuda", info.local_rank if world > 1 else 0)
    torch.cuda.set_device(dev)

    cfg = get_preset("12x128-bf16", numLayers=args.layers, channelSize=args.channels,
                     batchSize=args.batch * world, seed=1234, dtype=args.dtype)
    B = args.batch
    net = HipGoNet(cfg, B, device=dev, global_batch=B * world)
    if world > 1:
        dp.broadcast_(net.params, 0)
        net.refresh_weights()

    # synthetic data pool on device (different per rank)
    planes, player, rank, labels = random_planes(B * args.pool, seed=1000 + info.rank)
    # packed [planes | player | rank | labels] batches: one device copy per step
    from deep_go_amd.models.hip_model import pack_batch
    pool = torch.stack([pack_batch(planes[j * B:(j + 1) * B], player[j * B:(j + 1) * B],
                                   rank[j * B:(j + 1) * B], labels[j * B:(j + 1) * B])
                        for j in range(args.pool)]).to(dev)

    def load(i):
        net.set_batch_packed(pool[i % args.pool])

    bucketer = None
    if world > 1 or args.force_dp:
        lay = net.layout
        ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
        buckets = dp.make_buckets(ranges, int(args.bucket_mb * 2 ** 20), groups=net.wgroups)
        bucketer = dp.GradBucketer(net.grads, buckets, grad_dtype=args.grad_dtype)
    load(0)
    step = SegmentedStep(net, bucketer, use_graphs=not args.no_graph)

    for i in range(args.warmup):
        load(i)
        step()
    dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        load(i)
        step()
    dp.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = t.item()
    phases = None
    if args.profile > 0:
        from deep_go_amd.utils import trace
        trace.enable(True, host_timing=True)
        torch.cuda.synchronize()
        for i in range(args.profile):
            with trace.range("step"):
                with trace.range("load"):
                    load(i)
                step()
        torch.cuda.synchronize()
        phases = {k: round(1e3 * v / args.profile, 4) for k, v in trace.totals(True).items()}
        trace.enable(False)
    # accuracy/loss of the last step (sanity: finite)
    loss = net.mean_loss().item()
    acc = net.correct().item() / B
    total_boards = B * world * args.steps
    value = total_boards / elapsed
    ms = 1000.0 * elapsed / args.steps
    flops = cfg.train_flops_per_board() * B * world * args.steps / elapsed
    if info.rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "boards/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (random 19x19 uint8 feature planes, GPU-expanded to 37 planes; random-init weights)",
            "config": {"model": f"{args.layers}-layer d={args.channels} CNN (5x5 first, 3x3 hidden, 3x3 head, untied biases)",
                       "global_batch": B * world, "seq_len": 361,
                       "parallelism": f"dp{world}"},
            "achieved_tflops": round(flops / 1e12, 2),
            "last_loss": round(loss, 4),
            "last_batch_top1": round(acc, 4),
            "graphs": not args.no_graph,
            **({"profile_host_ms_per_step": phases} if phases else {}),
        }), flush=True)
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
