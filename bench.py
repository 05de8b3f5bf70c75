#!/usr/bin/env python3
"""Headline benchmark: board-positions/sec for the 12-layer d=128 GoCNN training step.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``.
  * N = 1: one process on cuda:0.
  * N > 1 and no WORLD_SIZE in the environment: this process is only a LAUNCHER.  Before
    anything touches the GPU (torch is not even imported) it starts
    ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py ...``
    as a CHILD process (one rank per GPU, RCCL over xGMI), relays rank 0's single JSON line
    and exits with the child's return code (non-zero if any rank failed).  The reference's
    ``makeDataParallel`` asserts the requested GPU count the same way
    (``/root/reference/experiments.lua:155-168``, assert at ``:157``).
  * N > 1 under torch.distributed.run (WORLD_SIZE set): one rank; WORLD_SIZE must equal N and
    N must not exceed the visible device count.
W untimed warmup steps, then EXACTLY K timed steps bracketed by barrier + device sync on both
sides; the MAX elapsed over ranks is used (per-rank min/max ms are reported too) and rank 0
prints ONE JSON line.

What one step is (nothing skipped inside the timed region):
  next batch (uint8 planes/labels) copied into the static input buffers (double-buffered:
  the copy runs on a load stream beside the previous step) ->
  GPU feature expansion -> 11 conv layers fwd -> fused head (loss, argmax, head bwd) ->
  bias-grad + wgrad + dgrad for every layer -> [N>1: bucketed RCCL all-reduce overlapped
  with backward] -> SGD with per-step LR decay -> bf16 weight refresh.
Weak scaling: 256 boards per GPU per step (BASELINE.json config "12-layer d=128 CNN bf16
on one MI355X, batch=256"; global batch = 256*N).  Synthetic 19x19 positions, random-init
weights (BASELINE.json: no datasets/checkpoints available).  Top-1 accuracy on synthetic
random labels is meaningless and is not reported here; held-out top-1 on the real fixture
comes from ``tools/fixture_accuracy.py`` (profiles/).

``--cpu-dry-run``: the same launcher / rank / timing / JSON path on the CPU over gloo with
the fp32 oracle at BASELINE config 1 size (tests/test_bench_launcher.py drives it at N=2, 4).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

METRIC = "board-positions/sec (whole node) 12-layer d=128 CNN; top-1 move accuracy"
HERE = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--pool", type=int, default=16, help="distinct synthetic batches")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--host-pool", action="store_true",
                    help="synthetic batches in pinned host memory (each step's copy is an H2D "
                         "copy, as from the trainer's loader) instead of device memory")
    ap.add_argument("--bucket-mb", type=float, default=6.0,
                    help="DP gradient bucket size (6 MB: head + the grouped hidden layers in "
                         "one bucket, fired beside the first layer's gradient chain; the first "
                         "layer in a second one)")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--comm", default="auto", choices=["auto", "native", "torch", "proxy"],
                    help="DP collectives: native = in-graph RCCL communicator (csrc/comm), "
                         "torch = torch.distributed between graph segments, proxy = world-1 "
                         "stand-in kernel on the comm stream (overlap measurement)")
    ap.add_argument("--profile", type=int, default=0, metavar="N",
                    help="after the timed run, N extra steps with roctx ranges (load / segments"
                         " / allreduce / optimizer) and a host phase breakdown; run under "
                         "rocprofv3 --marker-trace --kernel-trace to see them on the timeline")
    ap.add_argument("--force-dp", action="store_true",
                    help="use the DP path even on 1 GPU (world-1 communicator): measures its "
                         "overhead")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: hidden-layer forwards on e4m3 MX-MFMA (BASELINE config 5)")
    ap.add_argument("--spinup-steps", type=int, default=300,
                    help="untimed steps BEFORE the W warmup steps (a fixed count: every rank "
                         "must run the same number of collectives): "
                         "the GPU leaves its idle clock state over the first ~25 ms of load, so "
                         "without it a 20-step (20 ms) timed window measures the DVFS ramp "
                         "(20/5 steps: 0.97 ms/step, 200/50: 0.90 on the same box)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="launcher/timing/JSON path on CPU over gloo (BASELINE config 1 "
                         "model); no GPU")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(args, argv) -> int:
    """Parent of an N-rank run: torch.distributed.run as a child process (never exec: the
    parent must not replace itself, and it touches no GPU), relay rank 0's JSON line."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env,
                         cwd=HERE)
    lines = []
    for line in p.stdout:
        s = line.strip()
        if s.startswith("{") and '"metric"' in s:
            lines.append(s)
        else:
            sys.stderr.write(line)
    rc = p.wait()
    if rc != 0:
        sys.stderr.write(f"bench: {args.gpus}-rank run failed (rc={rc})\n")
        return rc if rc > 0 else 1
    if len(lines) != 1:
        sys.stderr.write(f"bench: expected one JSON line from rank 0, got {len(lines)}\n")
        return 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != args.gpus:
        sys.stderr.write(f"bench: ranks report n_gpus={rec.get('n_gpus')} != {args.gpus}\n")
        return 1
    print(lines[0], flush=True)
    return 0


def _gather_times(elapsed: float, dev) -> list:
    import torch
    import torch.distributed as dist
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [elapsed]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def _record(args, world, elapsed_all, flops_per_board, extra) -> dict:
    elapsed = max(elapsed_all)
    B = args.batch
    value = B * world * args.steps / elapsed
    ms = 1000.0 * elapsed / args.steps
    model = f"{args.layers}-layer d={args.channels} CNN (5x5 first, 3x3 hidden, 3x3 head, untied biases)"
    rec = {
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
        "data": "synthetic (random 19x19 uint8 feature planes, GPU-expanded to 37 planes; "
                "random-init weights)",
        "config": {"model": model, "global_batch": B * world, "seq_len": 361,
                   "parallelism": f"dp{world}"},
        "achieved_tflops": round(flops_per_board * B * world * args.steps / elapsed / 1e12, 2),
        "rank_ms_per_step_min": round(1000.0 * min(elapsed_all) / args.steps, 4),
        "rank_ms_per_step_max": round(1000.0 * elapsed / args.steps, 4),
    }
    rec.update(extra)
    return rec


def run_cpu_dry(args) -> int:
    """Every rank: fp32 oracle (CPUBackend) step with gloo gradient all-reduce."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from deep_go_amd.config import get_preset
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.parallel import dp
    from deep_go_amd.train.backends import CPUBackend
    info = dp.init_distributed(backend="gloo")
    world = info.world
    if os.environ.get("DG_BENCH_FAIL_RANK") == str(info.rank):   # launcher test hook
        raise SystemExit(f"rank {info.rank}: injected failure")
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} != --gpus {args.gpus}")
    torch.set_num_threads(1)
    cfg = get_preset("cpu-1layer-k16", batchSize=args.batch * world, seed=1234)
    be = CPUBackend(cfg, args.batch, world=world)
    if world > 1:
        dp.broadcast_(be.params.data, 0)
    pool = [random_planes(args.batch, seed=1000 + 97 * info.rank + j) for j in range(4)]
    for i in range(args.warmup):
        be.set_batch(*pool[i % 4])
        be.train_step()
    dp.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        be.set_batch(*pool[i % 4])
        be.train_step()
    dp.barrier()
    elapsed_all = _gather_times(time.perf_counter() - t0, "cpu")
    if info.rank == 0:
        args.layers, args.channels = cfg.numLayers, cfg.channelSize
        rec = _record(args, world, elapsed_all, cfg.train_flops_per_board(),
                      {"dry_run": "cpu-gloo", "dtype": "fp32"})
        rec["config"]["model"] = "cpu-1layer-k16 (BASELINE config 1; dry run, not a GPU number)"
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


def run_gpu(args) -> int:
    import torch
    sys.path.insert(0, HERE)
    from deep_go_amd.config import get_preset
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep, pack_batch
    from deep_go_amd.parallel import dp

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    ndev = torch.cuda.device_count()
    if world_env > ndev:
        raise SystemExit(f"WORLD_SIZE={world_env} > {ndev} visible GPUs")
    info = dp.init_distributed()
    world = info.world
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} != --gpus {args.gpus}")
    dev = torch.device("cuda", info.local_rank if world > 1 else 0)
    torch.cuda.set_device(dev)
    use_dp = world > 1 or args.force_dp
    comm = None
    if use_dp and world == 1 and args.comm == "torch" and not torch.distributed.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if use_dp:
        comm = dp.make_communicator(args.comm, dev)
        if comm.world != world:
            raise SystemExit(f"communicator world {comm.world} != {world}")

    cfg = get_preset("12x128-bf16", numLayers=args.layers, channelSize=args.channels,
                     batchSize=args.batch * world, seed=1234, dtype=args.dtype)
    B = args.batch
    net = HipGoNet(cfg, B, device=dev, global_batch=B * world)
    # input prefetch (the next batch's copy on a load stream beside the previous step): on for
    # the pinned host pool (SDMA copies, +1.1%), off for the device pool (its blit-kernel copy
    # beside the step measured -1%; profiles/r2_input_prefetch_ab.txt); DG_PREFETCH=0/1 forces
    pf = os.environ.get("DG_PREFETCH", "auto")
    prefetch = (pf == "1" or (pf != "0" and args.host_pool)) and net.enable_prefetch()
    if world > 1:
        comm.broadcast_(net.params, 0)
        net.refresh_weights()

    # synthetic data pool on device (different per rank)
    planes, player, rank, labels = random_planes(B * args.pool, seed=1000 + info.rank)
    # packed [planes | player | rank | labels] batches: one device copy per step
    pool = torch.stack([pack_batch(planes[j * B:(j + 1) * B], player[j * B:(j + 1) * B],
                                   rank[j * B:(j + 1) * B], labels[j * B:(j + 1) * B])
                        for j in range(args.pool)])
    pool = pool.pin_memory() if args.host_pool else pool.to(dev)

    def load(i):
        net.set_batch_packed(pool[i % args.pool])

    bucketer = None
    if use_dp:
        lay = net.layout
        ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
        buckets = dp.make_buckets(ranges, int(args.bucket_mb * 2 ** 20), groups=net.wgroups)
        bucketer = dp.GradBucketer(net.grads, buckets, grad_dtype=args.grad_dtype, comm=comm)
    load(0)
    step = SegmentedStep(net, bucketer, use_graphs=not args.no_graph)

    for i in range(args.spinup_steps):    # untimed: clock ramp (see --help)
        load(i)
        step()
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
    elapsed_all = _gather_times(time.perf_counter() - t0, dev)
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
    loss = net.mean_loss().item()  # sanity: finite
    consistent = None
    if world > 1:
        # every rank must hold bit-identical parameters after the run (same init, same
        # all-reduced gradients): a silent collective bug fails the bench here
        sig = torch.stack([net.params.double().sum(), (net.params.double() ** 2).sum()])
        sigs = [torch.zeros_like(sig) for _ in range(world)]
        torch.distributed.all_gather(sigs, sig)
        consistent = all(torch.equal(x, sigs[0]) for x in sigs)
        if not consistent:
            raise SystemExit(f"rank {info.rank}: parameters diverged across ranks: "
                             f"{[x.tolist() for x in sigs]}")
    if info.rank == 0:
        extra = {"last_loss": round(loss, 4), "graphs": not args.no_graph,
                 "step_mode": step.mode, "spinup_steps": args.spinup_steps,
                 "input_prefetch": bool(prefetch)}
        if use_dp:
            extra["comm"] = comm.kind
            extra["ranks_params_identical"] = consistent
            extra["grad_dtype"] = args.grad_dtype
        if phases:
            extra["profile_host_ms_per_step"] = phases
        print(json.dumps(_record(args, world, elapsed_all, cfg.train_flops_per_board(), extra)),
              flush=True)
    if comm is not None:
        comm.close()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()
    return 0


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse(argv)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch(args, argv)
    if args.cpu_dry_run:
        return run_cpu_dry(args)
    return run_gpu(args)


if __name__ == "__main__":
    sys.exit(main())
