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
  next batch (uint8 planes/labels) copied into the static input buffers ->
  GPU feature expansion -> 11 conv layers fwd -> fused head (loss, argmax, head bwd) ->
  bias-grad + wgrad + dgrad for every layer -> [N>1: bucketed RCCL all-reduce overlapped
  with backward] -> SGD with per-step LR decay -> bf16 weight refresh.
Weak scaling: 256 boards per GPU per step (BASELINE.json config "12-layer d=128 CNN bf16
on one MI355X, batch=256"; global batch = 256*N).  Synthetic 19x19 positions, random-init
weights (BASELINE.json: no datasets/checkpoints available).  Top-1 accuracy on synthetic
random labels is meaningless; the metric's accuracy half is measured separately (below).

After the headline timing (never inside it) the same process measures:
  * ``secondary``: the headline network in fp8 (12x128 fp8) and the d=256 configs (BASELINE
    configs 3-5 per GPU: 12x256 bf16 and fp8) with the same K/W and the same communicator
    (under N > 1 that is config 3/5's DP=N step);
  * ``dp`` (N > 1 or --force-dp): communicator kind and RCCL version, per-rank devices, bytes
    all-reduced per step, the step's bucket collectives timed alone (us/step, bus GB/s), the
    same network's step without collectives, and from those the exposed communication time
    and the fraction of it hidden behind compute;
  * ``accuracy`` (rank 0, --accuracy-steps): the headline network trained on the reference's
    bundled games, top-1 / NLL on every position of the held-out validation and test games
    (``fixture_top1`` = validation top-1; one game per split: paper-level parity unpinned;
    ``deep_go_amd/train/accuracy.py``).

Multi-rank safety: every rank arms a phase guard (``utils/faults.PhaseGuard``) before the
process-group rendezvous.  Each phase has its own deadline: ``init`` / ``comm`` / ``capture``
(--comm-timeout, 90 s), ``warmup`` / ``timed`` / ``report`` and each secondary config's
capture / warmup / timed (--phase-timeout, 60 s); on expiry the rank writes
``hang:<phase>:<communicator kind>`` to its status file and exits 42.  Under the driver's
own ``torch.distributed.run`` that bounds a hung rank to ~90 s.  Through this file's launcher
(``--gpus N`` without WORLD_SIZE) the whole job is bounded by --launch-budget (540 s): when a
guard fired on a rank that was on the native in-graph communicator in a phase that issues
its collectives, the launcher re-runs ONCE with ``--comm torch`` inside the remaining budget
and says so in the JSON (``comm_fallback``); any other failure is reported as it is.

``--cpu-dry-run``: the same launcher / rank / timing / JSON path on the CPU over gloo with
the fp32 oracle at BASELINE config 1 size (tests/test_bench_launcher.py drives it at N=2, 4).
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
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
    ap.add_argument("--device-pool", action="store_true",
                    help="synthetic batches in device memory (each step's copy a D2D blit) "
                         "instead of the default pinned host pool (each step's batch an H2D "
                         "copy prefetched beside the previous step, as the trainer's loader "
                         "does; the reference copies host->device every step, train.lua:99-100)")
    ap.add_argument("--host-pool", action="store_true", help="(the default; kept for scripts)")
    ap.add_argument("--bucket-mb", type=float, default=3.0,
                    help="DP gradient bucket size; with --wgrad-group splitting the hidden "
                         "layers, 3 MB gives one bucket per weight-gradient group (head + top "
                         "group | bottom group | first layer)")
    ap.add_argument("--wgrad-group", type=int, default=0,
                    help="DP: hidden layers per grouped weight-gradient launch.  0 = auto: at "
                         "d >= 256 and world > 1 half of them (the top group's all-reduce runs beside the "
                         "bottom group's launch: 3.138 vs 3.178 ms/step with the RCCL-shaped "
                         "proxy), at d = 128 one launch (the split doubles the split-K slab "
                         "traffic: +6%% compute for ~5 us less exposed comm); "
                         "profiles/r3_dp_overlap_proxy.txt")
    ap.add_argument("--grad-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="DP gradient wire format (the bucket all-reduces).  fp32 (default) is "
                         "the reference's precision (DataParallelTable, experiments.lua:155-168). "
                         "bf16 halves the bytes on xGMI (every gradient pass 2 writes the bf16 "
                         "twin itself, the fused update reads it); bounded against fp32 at "
                         "world 8 by tests/test_wire_cpu.py and tests/test_train_gpu.py.  Under "
                         "N > 1 the bf16 wire is also measured, labelled, as secondary "
                         "'dp-bf16-wire' (--no-bf16-wire-secondary: skip)")
    ap.add_argument("--no-bf16-wire-secondary", action="store_true")
    ap.add_argument("--comm", default="auto", choices=["auto", "native", "torch", "proxy"],
                    help="DP collectives: native = in-graph RCCL communicator (csrc/comm), "
                         "torch = torch.distributed between graph segments, proxy = world-1 "
                         "RCCL-shaped stand-in kernel on the comm stream (overlap measurement)")
    ap.add_argument("--proxy-world", type=int, default=8)
    ap.add_argument("--proxy-gbps", type=float, default=300.0,
                    help="proxy: ring bus rate it is paced to (GB/s)")
    ap.add_argument("--proxy-blocks", type=int, default=32)
    ap.add_argument("--profile", type=int, default=0, metavar="N",
                    help="after the timed run, N extra steps with roctx ranges (load / segments"
                         " / allreduce / optimizer) and a host phase breakdown; run under "
                         "rocprofv3 --marker-trace --kernel-trace to see them on the timeline")
    ap.add_argument("--force-dp", action="store_true",
                    help="use the DP path even on 1 GPU (world-1 communicator): measures its "
                         "overhead")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: hidden-layer forwards on e4m3 MX-MFMA (BASELINE config 5)")
    ap.add_argument("--secondary", default="128:fp8,256:bf16,256:fp8,256:bf16:fixture",
                    help="after the headline: other configs as CHANNELS:DTYPE[:fixture],... "
                         "('' = none; fixture = the reference's bundled games through the C++ "
                         "loader, BASELINE config 4)")
    ap.add_argument("--no-report", action="store_true",
                    help="skip the post-timing DP report (isolated collectives, no-comm step)")
    ap.add_argument("--spinup-steps", type=int, default=300,
                    help="untimed steps BEFORE the W warmup steps (a fixed count: every rank "
                         "must run the same number of collectives): "
                         "the GPU leaves its idle clock state over the first ~25 ms of load, so "
                         "without it a 20-step (20 ms) timed window measures the DVFS ramp "
                         "(20/5 steps: 0.97 ms/step, 200/50: 0.90 on the same box)")
    ap.add_argument("--comm-timeout", type=float, default=90.0,
                    help="N > 1: per-rank limit (s) of the process-group init, the communicator "
                         "set-up and the headline's capture phase (each)")
    ap.add_argument("--phase-timeout", type=float, default=60.0,
                    help="N > 1: per-rank limit (s) of every other phase: the headline's warmup, "
                         "timed and report phases, and each secondary config's capture, warmup "
                         "and timed phases (each has its own deadline)")
    ap.add_argument("--launch-budget", type=float, default=540.0,
                    help="N > 1 launcher (no WORLD_SIZE in the environment): wall-clock bound "
                         "of the whole job including one --comm torch fallback run.  The first "
                         "run may use the budget minus a 150-s reserve; if a rank's guard "
                         "reports a hang while it was on the native communicator, the "
                         "fallback run gets what is left.  Worst case: %(default)s s")
    ap.add_argument("--accuracy-steps", type=int, default=3000,
                    help="after the timed phases (untimed): train the bench's network this many "
                         "SGD steps (batch 64) on the reference's bundled training games and "
                         "report top-1 / NLL on the held-out validation and test games "
                         "(\"accuracy\" in the JSON; rank 0 only; 0 = skip)")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="launcher/timing/JSON path on CPU over gloo (BASELINE config 1 "
                         "model); no GPU")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ranks(args, argv, status_dir, limit_s):
    """One torch.distributed.run child (its own process group, so a wedged run can be ended
    as a whole); returns (rc, json lines)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    env["DG_BENCH_STATUS_DIR"] = status_dir
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=None, text=True, env=env,
                         cwd=HERE, start_new_session=True)
    t_end = time.monotonic() + limit_s

    def on_alarm(*_):
        sys.stderr.write(f"bench: the {args.gpus}-rank run exceeded {limit_s:.0f} s: "
                         "ending its process group\n")
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
    old = signal.signal(signal.SIGALRM, on_alarm)
    signal.alarm(max(1, int(t_end - time.monotonic())))
    lines = []
    try:
        for line in p.stdout:
            s = line.strip()
            if s.startswith("{") and '"metric"' in s:
                lines.append(s)
            else:
                sys.stderr.write(line)
        rc = p.wait()
    finally:
        signal.alarm(0)
        signal.signal(signal.SIGALRM, old)
    return rc, lines


def _hangs(status_dir):
    """{rank file: (phase, comm kind)} of every rank whose phase guard fired."""
    out = {}
    for f in sorted(os.listdir(status_dir)):
        try:
            txt = open(os.path.join(status_dir, f)).read().strip()
        except OSError:
            continue
        if txt.startswith("hang:"):
            parts = txt.split(":")
            out[f] = (parts[1], parts[2] if len(parts) > 2 else "")
    return out


# phases in which a rank issues collectives through the chosen communicator (the process-group
# init comes before any choice)
_COMM_PHASES = ("comm", "capture", "warmup", "timed", "report")


def _native_hang(hangs) -> bool:
    """A guard fired while its rank was on (or setting up) the native communicator, in a phase
    that issues its collectives: the case a --comm torch re-run can cure."""
    return any(kind == "native" and (ph in _COMM_PHASES or ph.startswith("sec-"))
               for ph, kind in hangs.values())


def launch(args, argv) -> int:
    """Parent of an N-rank run: torch.distributed.run as a child process (never exec: the
    parent must not replace itself, and it touches no GPU), relay rank 0's JSON line.
    If a rank's phase guard reports a hang while that rank was on the native communicator
    (--comm auto), re-run once with torch.distributed collectives.  The whole job is bounded
    by --launch-budget: the first run by the budget minus a 150-s reserve, the fallback by
    what is left."""
    t_start = time.monotonic()
    budget = max(60.0, args.launch_budget)
    reserve = min(150.0, budget / 3)
    status_dir = tempfile.mkdtemp(prefix="dg_bench_")
    fallback = None
    hangs = {}
    try:
        rc, lines = _run_ranks(args, argv, status_dir, budget - reserve)
        hangs = _hangs(status_dir)
        left = budget - (time.monotonic() - t_start)
        if (rc != 0 and args.comm == "auto" and _native_hang(hangs) and left > 30):
            fallback = f"native communicator run hung ({hangs}); re-run with --comm torch"
            sys.stderr.write(f"bench: {fallback}\n")
            for f in os.listdir(status_dir):
                os.remove(os.path.join(status_dir, f))
            rc, lines = _run_ranks(args, argv + ["--comm", "torch"], status_dir, left)
            hangs = _hangs(status_dir)
    finally:
        shutil.rmtree(status_dir, ignore_errors=True)
    if rc != 0:
        sys.stderr.write(f"bench: {args.gpus}-rank run failed (rc={rc})"
                         + (f"; hung phases {hangs}" if hangs else "") + "\n")
        return rc if rc > 0 else 1
    if len(lines) != 1:
        sys.stderr.write(f"bench: expected one JSON line from rank 0, got {len(lines)}\n")
        return 1
    rec = json.loads(lines[0])
    if rec.get("n_gpus") != args.gpus:
        sys.stderr.write(f"bench: ranks report n_gpus={rec.get('n_gpus')} != {args.gpus}\n")
        return 1
    if fallback:
        rec["comm_fallback"] = fallback
        print(json.dumps(rec), flush=True)
    else:
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


def _model_name(layers, channels):
    return (f"{layers}-layer d={channels} CNN (5x5 first, 3x3 hidden, 3x3 head, "
            "untied biases)")


def _record(args, world, elapsed_all, flops_per_board, extra) -> dict:
    elapsed = max(elapsed_all)
    B = args.batch
    value = B * world * args.steps / elapsed
    ms = 1000.0 * elapsed / args.steps
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
        "config": {"model": _model_name(args.layers, args.channels), "global_batch": B * world,
                   "seq_len": 361, "parallelism": f"dp{world}"},
        "achieved_tflops": round(flops_per_board * B * world * args.steps / elapsed / 1e12, 2),
        "rank_ms_per_step_min": round(1000.0 * min(elapsed_all) / args.steps, 4),
        "rank_ms_per_step_max": round(1000.0 * elapsed / args.steps, 4),
    }
    rec.update(extra)
    return rec


class _NoGuard:
    def phase(self, *_):
        pass

    def set_comm(self, *_):
        pass

    def stop(self):
        pass


def _guard(args):
    """The rank's phase guard, armed BEFORE torch.distributed's rendezvous (rank / world from
    the environment torch.distributed.run sets)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return _NoGuard()
    from deep_go_amd.utils.faults import PhaseGuard
    return PhaseGuard(int(os.environ.get("RANK", "0")), os.environ.get("DG_BENCH_STATUS_DIR"))


def _test_hang(rank, phase, comm=""):
    """Test hook (tests/test_bench_launcher.py): DG_BENCH_HANG=RANK:PHASE[:COMM] sleeps there
    (with COMM: only while this rank is on that communicator kind)."""
    spec = os.environ.get("DG_BENCH_HANG", "")
    if not spec:
        return
    parts = spec.split(":")
    if parts[:2] == [str(rank), phase] and (len(parts) < 3 or parts[2] == comm):
        time.sleep(3600)


def run_cpu_dry(args) -> int:
    """Every rank: fp32 oracle (CPUBackend) step with gloo gradient all-reduce."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, HERE)
    from deep_go_amd.config import get_preset
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.parallel import dp
    from deep_go_amd.train.backends import CPUBackend
    guard = _guard(args)
    guard.phase("init", args.comm_timeout)
    info = dp.init_distributed(backend="gloo")
    world = info.world
    if os.environ.get("DG_BENCH_FAIL_RANK") == str(info.rank):   # launcher test hook
        raise SystemExit(f"rank {info.rank}: injected failure")
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} != --gpus {args.gpus}")
    # communicator set-up.  There is no RCCL on the CPU: --comm auto / native rehearses the
    # native communicator's set-up phase (the guard reports the rank as on "native" while a
    # gloo barrier stands in for ncclCommInitRank), so the launcher's hang -> --comm torch
    # fallback path runs here; the collectives themselves are gloo's either way
    kind = "native" if args.comm in ("auto", "native") else "torch"
    guard.phase("comm", args.comm_timeout)
    guard.set_comm(kind)
    _test_hang(info.rank, "comm", kind)
    dp.barrier()
    torch.set_num_threads(1)
    cfg = get_preset("cpu-1layer-k16", batchSize=args.batch * world, seed=1234)
    be = CPUBackend(cfg, args.batch, world=world)
    if world > 1:
        dp.broadcast_(be.params.data, 0)
    pool = [random_planes(args.batch, seed=1000 + 97 * info.rank + j) for j in range(4)]
    guard.phase("warmup", args.phase_timeout)
    _test_hang(info.rank, "warmup")
    for i in range(args.warmup):
        be.set_batch(*pool[i % 4])
        be.train_step()
    dp.barrier()
    guard.phase("timed", args.phase_timeout)
    _test_hang(info.rank, "timed")
    t0 = time.perf_counter()
    for i in range(args.steps):
        be.set_batch(*pool[i % 4])
        be.train_step()
    dp.barrier()
    elapsed_all = _gather_times(time.perf_counter() - t0, "cpu")
    guard.stop()
    if info.rank == 0:
        args.layers, args.channels = cfg.numLayers, cfg.channelSize
        rec = _record(args, world, elapsed_all, cfg.train_flops_per_board(),
                      {"dry_run": "cpu-gloo", "dtype": "fp32", "grad_dtype": "fp32",
                       "comm": f"gloo ({kind} set-up rehearsed)"})
        rec["config"]["model"] = "cpu-1layer-k16 (BASELINE config 1; dry run, not a GPU number)"
        print(json.dumps(rec), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


FIXTURE_TRAIN = os.path.join(HERE, "tests", "fixtures", "train.dgpack.npz")


class _Case:
    """One configuration's network, input source, optional DP bucketer and step graph.

    Input sources: the synthetic pool (``data="synthetic"``: --pool packed batches in pinned
    host memory, each step's batch an H2D copy prefetched beside the previous step — the
    reference's per-step host->device copy, train.lua:99-100 — or, with --device-pool, in
    device memory) or ``data="fixture"``: the reference's bundled training games
    (tests/fixtures/train.dgpack.npz, 4139 real positions) sampled game-uniformly by the C++
    loader threads into pinned ring slots, one prefetched H2D copy per step, the 37 planes
    expanded on the GPU (BASELINE config 4: data.lua:82-96, dataloader.lua:113-125)."""

    def __init__(self, args, channels, dtype, world, info, dev, comm, use_dp,
                 grad_dtype=None, data="synthetic"):
        import torch
        from deep_go_amd.config import get_preset
        from deep_go_amd.data.synthetic import random_planes
        from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep, pack_batch
        from deep_go_amd.parallel import dp
        self.args, self.channels, self.dtype = args, channels, dtype
        self.grad_dtype = grad_dtype or args.grad_dtype
        self.data = data
        self.loader = None
        B = args.batch
        self.cfg = get_preset("12x128-bf16", numLayers=args.layers, channelSize=channels,
                              batchSize=B * world, seed=1234, dtype=dtype)
        n_hidden = args.layers - 2
        wg = None
        if use_dp:
            # auto: split the hidden layers' weight-gradient launch in two at d >= 256 only
            # when there is communication to hide (world > 1): the top group's all-reduce
            # then runs beside the second launch.  At world 1 (--force-dp) the split is pure
            # cost: -2.5% (12x256 bf16) / -4.5% (fp8) vs one launch, which matches the plain
            # step (profiles/r5_dp_fusion.txt)
            wg = args.wgrad_group or (max(1, (n_hidden + 1) // 2)
                                      if channels >= 256 and world > 1 else 16)
        # (--grad-dtype bf16: the gradient reduces write the bf16 wire twin themselves)
        self.net = net = HipGoNet(self.cfg, B, device=dev, global_batch=B * world,
                                  wgrad_group=wg,
                                  grad_wire=self.grad_dtype if use_dp else "fp32")
        host = data == "fixture" or not args.device_pool
        # input prefetch (the next batch's H2D copy on a load stream beside the previous step,
        # SDMA): on for host sources; off for the device pool (its blit-kernel copy beside the
        # step measured -1%, profiles/r2_input_prefetch_ab.txt).  The host pool + prefetch
        # costs 1.2-1.5% against the device pool (the step graph waits on the copy's event:
        # ~8 us more at the step boundary than the in-stream blit,
        # profiles/r6_host_pool_prefetch.txt).  DG_PREFETCH=0 / 1 forces
        pf = os.environ.get("DG_PREFETCH", "auto")
        self.prefetch = (pf == "1" or (pf != "0" and host)) and net.enable_prefetch()
        if world > 1:
            comm.broadcast_(net.params, 0)
            net.refresh_weights()
        self.pool = None
        if data == "fixture":
            from deep_go_amd.data.dataset import PackedDataset
            from deep_go_amd.data.loader import BatchLoader
            self.loader = BatchLoader(PackedDataset.load(FIXTURE_TRAIN), B, threads=4,
                                      prefetch=6, seed=7 + 1009 * info.rank)
        else:
            # synthetic data pool (different per rank), packed [planes | player | rank |
            # labels] batches: one copy per step
            planes, player, rank, labels = random_planes(B * args.pool, seed=1000 + info.rank)
            pool = torch.stack([pack_batch(planes[j * B:(j + 1) * B], player[j * B:(j + 1) * B],
                                           rank[j * B:(j + 1) * B], labels[j * B:(j + 1) * B])
                                for j in range(args.pool)])
            self.pool = pool.pin_memory() if host else pool.to(dev)
        self.bucketer = None
        if use_dp:
            lay = net.layout
            ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
            buckets = dp.make_buckets(ranges, int(args.bucket_mb * 2 ** 20), groups=net.wgroups)
            self.bucketer = dp.GradBucketer(net.grads, buckets, grad_dtype=self.grad_dtype,
                                            comm=comm, shadow=net.grads16)
        self.load(0)
        self.step = SegmentedStep(net, self.bucketer, use_graphs=not args.no_graph)
        self.input = ("host pinned, H2D prefetched on a load stream" if host and self.prefetch
                      else "host pinned, H2D in the step" if host else "device-resident pool")

    def load(self, i):
        if self.loader is not None:
            self.net.set_batch_packed_from(self.loader)
        else:
            self.net.set_batch_packed(self.pool[i % self.args.pool])

    def close(self):
        if self.loader is not None:
            self.loader.close()
            self.loader = None

    def run(self, n):
        for i in range(n):
            self.load(i)
            self.step()

    def timed(self, n, dev):
        import torch
        from deep_go_amd.parallel import dp
        dp.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        self.run(n)
        dp.barrier()
        torch.cuda.synchronize()
        return _gather_times(time.perf_counter() - t0, dev)

    def params_identical(self, world) -> bool:
        """Every rank must hold bit-identical parameters after the run (same init, same
        all-reduced gradients): a silent collective bug fails the bench."""
        import torch
        if world == 1:
            return True
        p = self.net.params.double()
        sig = torch.stack([p.sum(), (p ** 2).sum()])
        sigs = [torch.zeros_like(sig) for _ in range(world)]
        torch.distributed.all_gather(sigs, sig)
        return all(torch.equal(x, sigs[0]) for x in sigs)


def _dp_report(case, comm, world, dev, args, step_ms) -> dict:
    """Post-timing DP evidence: the step's bucket collectives alone, and the same network's
    step without collectives (so exposed comm = step - step without comm)."""
    import torch
    from deep_go_amd.models.hip_model import SegmentedStep
    from deep_go_amd.parallel import dp
    bk = case.bucketer
    esize = 2 if args.grad_dtype == "bf16" else 4
    nbytes = sum(e - s for s, e, _ in bk.buckets) * esize
    rep = {"comm": comm.kind, "buckets": len(bk.buckets),
           "bucket_mb": [round((e - s) * esize / 2 ** 20, 3) for s, e, _ in bk.buckets],
           "wgrad_groups": [len(g) for g in case.net.wgroups],
           "allreduce_bytes_per_step": nbytes, "grad_dtype": args.grad_dtype}
    if comm.kind == "native":
        rep["rccl_version"] = comm.version()
    else:
        try:
            rep["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
        except Exception:  # noqa: BLE001
            pass
    if comm.kind == "proxy":
        rep["proxy"] = {"world": comm.proxy_world, "gbps": comm.gbps, "blocks": comm.blocks}
    devs = {"rank": dp.env_info().rank, "device": dev.index,
            "pci_bus_id": getattr(torch.cuda.get_device_properties(dev), "pci_bus_id", None)}
    # what the communicator itself reports (RCCL's rank count / rank / device for native)
    devs.update({f"comm_{k}": v for k, v in comm.seen().items()})
    if world > 1:
        allv = [None] * world
        torch.distributed.all_gather_object(allv, devs)
        rep["devices"] = allv
        rep["ranks_seen"] = sorted({d.get("comm_ranks_seen") for d in allv}, key=str)
    else:
        rep["devices"] = [devs]
        rep["ranks_seen"] = [devs.get("comm_ranks_seen")]
    # (a) the bucket collectives alone, back to back on the comm stream (same count on every
    # rank): us per step and the ring bus bandwidth 2(n-1)/n * bytes / time
    reps = 20
    n = max(world, comm.proxy_world if comm.kind == "proxy" else world)
    for _ in range(3):
        for b in range(len(bk.buckets)):
            bk.fire(b)
        bk.wait()
    dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for b in range(len(bk.buckets)):
            bk.fire(b)
        bk.wait()
    torch.cuda.synchronize()
    t_iso = _gather_times(time.perf_counter() - t0, dev)
    us = 1e6 * max(t_iso) / reps
    rep["comm_isolated_us_per_step"] = round(us, 2)
    if n > 1:
        rep["bus_gbps"] = round(2.0 * (n - 1) / n * nbytes / (us * 1e-6) / 1e9, 1)
    # (b) the same network's step without collectives (one graph), timed like the headline
    plain = SegmentedStep(case.net, None, use_graphs=not args.no_graph)
    for i in range(max(20, args.warmup)):
        case.load(i)
        plain()
    dp.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        case.load(i)
        plain()
    torch.cuda.synchronize()
    t_plain = _gather_times(time.perf_counter() - t0, dev)
    ms_plain = 1000.0 * max(t_plain) / args.steps
    exposed = max(0.0, (step_ms - ms_plain) * 1000.0)
    rep["step_nocomm_ms"] = round(ms_plain, 4)
    rep["comm_exposed_us_per_step"] = round(exposed, 2)
    rep["overlap_frac"] = round(max(0.0, min(1.0, 1.0 - exposed / us)), 3) if us > 0 else None
    return rep


def run_gpu(args) -> int:
    import torch
    sys.path.insert(0, HERE)
    from deep_go_amd.parallel import dp

    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    ndev = torch.cuda.device_count()
    if world_env > ndev:
        raise SystemExit(f"WORLD_SIZE={world_env} > {ndev} visible GPUs")
    guard = _guard(args)
    guard.phase("init", args.comm_timeout)
    info = dp.init_distributed()
    world = info.world
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} != --gpus {args.gpus}")
    dev = torch.device("cuda", info.local_rank if world > 1 else 0)
    torch.cuda.set_device(dev)
    use_dp = world > 1 or args.force_dp
    comm = None
    extra_comm = {}
    guard.phase("comm", args.comm_timeout)
    guard.set_comm("native" if args.comm in ("auto", "native") else args.comm)
    _test_hang(info.rank, "comm", "native" if args.comm in ("auto", "native") else args.comm)
    if use_dp and world == 1 and args.comm == "torch" and not torch.distributed.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    if use_dp:
        comm = dp.make_communicator(args.comm, dev, world=args.proxy_world,
                                    gbps=args.proxy_gbps, blocks=args.proxy_blocks)
        guard.set_comm(comm.kind)
        extra_comm = {"comm_seen": comm.seen()}
        if comm.world != world:
            raise SystemExit(f"communicator world {comm.world} != {world}")
        seen = comm.seen()
        if world > 1 and seen.get("ranks_seen", world) != world:
            raise SystemExit(f"rank {info.rank}: the communicator reports "
                             f"{seen.get('ranks_seen')} ranks, WORLD_SIZE is {world}")

    guard.phase("capture", args.comm_timeout)
    case = _Case(args, args.channels, args.dtype, world, info, dev, comm, use_dp)
    guard.phase("warmup", args.phase_timeout)
    case.run(args.spinup_steps)     # untimed: clock ramp (see --help)
    case.run(args.warmup)
    guard.phase("timed", args.phase_timeout)
    _test_hang(info.rank, "timed", comm.kind if comm is not None else "")
    elapsed_all = case.timed(args.steps, dev)
    guard.phase("report", args.phase_timeout)
    phases = None
    if args.profile > 0:
        from deep_go_amd.utils import trace
        trace.enable(True, host_timing=True)
        torch.cuda.synchronize()
        for i in range(args.profile):
            with trace.range("step"):
                with trace.range("load"):
                    case.load(i)
                case.step()
        torch.cuda.synchronize()
        phases = {k: round(1e3 * v / args.profile, 4) for k, v in trace.totals(True).items()}
        trace.enable(False)
    loss = case.net.mean_loss().item()  # sanity: finite
    consistent = case.params_identical(world)
    if not consistent:
        raise SystemExit(f"rank {info.rank}: parameters diverged across ranks")
    extra = {"last_loss": round(loss, 4), "graphs": not args.no_graph,
             "step_mode": case.step.mode, "spinup_steps": args.spinup_steps,
             "input_prefetch": bool(case.prefetch), "input": case.input}
    step_ms = 1000.0 * max(elapsed_all) / args.steps
    # gradient precision of the step: single-GPU gradients are reduced in fp32 (split-K slabs
    # + fused update); under DP the bucket all-reduces run in --grad-dtype
    extra["grad_dtype"] = args.grad_dtype if use_dp else "fp32"
    if use_dp:
        extra["comm"] = comm.kind
        extra["ranks_params_identical"] = consistent
        extra.update(extra_comm)
        if not args.no_report:
            extra["dp"] = _dp_report(case, comm, world, dev, args, step_ms)
    if phases:
        extra["profile_host_ms_per_step"] = phases
    headline = _record(args, world, elapsed_all, case.cfg.train_flops_per_board(), extra)
    case.close()
    del case
    torch.cuda.synchronize()
    torch.cuda.empty_cache()

    # secondary configurations (never inside the headline's timed region): CH:DTYPE[:fixture]
    # (fixture = the reference's games through the C++ loader, BASELINE config 4), and under
    # DP the headline network on the bf16 gradient wire (labelled: the headline is fp32)
    items = [x.split(":") for x in args.secondary.split(",") if x]
    if (use_dp and world > 1 and args.grad_dtype == "fp32"
            and not args.no_bf16_wire_secondary):
        items.append([str(args.channels), args.dtype, "wire16"])
    sec = {}
    for it in items:
        ch, dt = it[0], it[1]
        var = it[2] if len(it) > 2 else ""
        if var not in ("", "fixture", "wire16"):
            raise SystemExit(f"--secondary {':'.join(it)}: unknown variant {var!r}")
        if int(ch) == args.channels and dt == args.dtype and not var:
            continue
        tag = "-".join(it)     # (the status file is colon-separated)
        guard.phase(f"sec-{tag}-capture", args.phase_timeout)
        c2 = _Case(args, int(ch), dt, world, info, dev, comm, use_dp,
                   grad_dtype="bf16" if var == "wire16" else None,
                   data="fixture" if var == "fixture" else "synthetic")
        guard.phase(f"sec-{tag}-warmup", args.phase_timeout)
        c2.run(100)
        c2.run(args.warmup)
        guard.phase(f"sec-{tag}-timed", args.phase_timeout)
        if c2.loader is not None:
            c2.loader.wait_s = 0.0
        t = c2.timed(args.steps, dev)
        ok = c2.params_identical(world)
        if not ok:
            raise SystemExit(f"rank {info.rank}: parameters diverged across ranks ({tag})")
        el = max(t)
        name = (f"12x{ch}-{dt}" if args.layers == 12 else f"{args.layers}x{ch}-{dt}")
        name = {"fixture": name + "-fixture", "wire16": "dp-bf16-wire"}.get(var, name)
        rec = {
            "value": round(args.batch * world * args.steps / el, 1), "unit": "boards/s",
            "ms_per_step": round(1000.0 * el / args.steps, 4), "steps": args.steps,
            "warmup": args.warmup, "spinup_steps": 100, "dtype": dt,
            "model": _model_name(args.layers, int(ch)), "global_batch": args.batch * world,
            "parallelism": f"dp{world}", "step_mode": c2.step.mode, "input": c2.input,
            "achieved_tflops": round(c2.cfg.train_flops_per_board() * args.batch * world
                                     * args.steps / el / 1e12, 2)}
        if use_dp:
            rec["grad_dtype"] = c2.grad_dtype
        if var == "wire16":
            rec["label"] = ("the headline network with the bf16 gradient wire (NOT the "
                            "reference's fp32 gradient reduce)")
        if c2.loader is not None:
            rec["data"] = ("fixture (C++ loader): the reference's 20 bundled training games, "
                           "4139 real positions, game-uniform sampling, 4 loader threads")
            rec["loader_wait_us_per_step"] = round(1e6 * c2.loader.wait_s / args.steps, 1)
            rec["loader_errors"] = c2.loader.errors()
        sec[name] = rec
        c2.close()
        del c2
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    if sec:
        headline["secondary"] = sec
    if args.accuracy_steps > 0:
        # the metric's accuracy half (train.lua:14-45,122), untimed; rank 0 trains its own
        # single-GPU copy while the other ranks wait at the barrier
        guard.phase("accuracy", args.phase_timeout)
        acc = None
        if info.rank == 0:
            from deep_go_amd.train.accuracy import fixture_accuracy
            acc = fixture_accuracy(dev, layers=args.layers, channels=args.channels,
                                   dtype=args.dtype, steps=args.accuracy_steps)
        dp.barrier()
        if acc is not None:
            headline["fixture_top1"] = acc["validation_top1"]
            headline["accuracy"] = acc
    guard.stop()
    if info.rank == 0:
        print(json.dumps(headline), flush=True)
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
