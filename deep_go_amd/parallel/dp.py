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


class TorchComm:
    """Collectives through torch.distributed (ProcessGroupNCCL = RCCL on ROCm, or gloo).
    Issued from the host between graph segments (they cannot sit inside our step graph)."""
    kind = "torch"
    in_graph = False

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0

    def all_reduce_async(self, t: torch.Tensor):
        return dist.all_reduce(t, group=self.group, async_op=True)

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        if self.world > 1:
            dist.broadcast(t, root, group=self.group)
        return t

    def seen(self) -> dict:
        return {"ranks_seen": self.world, "user_rank": self.rank}

    def async_error(self) -> str:
        return ""

    def close(self):
        pass


class IpcOneShot:
    """One-shot IPC all-reduce of SMALL buckets on one node (csrc/comm/oneshot.hip; SURVEY
    §5.8's optional small-bucket path): each rank stages its bucket in an uncached,
    IPC-exported buffer, signals every peer, and one kernel sums all `world` buffers over
    xGMI in rank order — one kernel instead of a ring's 2(n-1) latency-bound steps.
    Stream-ordered and graph-capturable like the RCCL calls.  Handles travel through a c10d
    store (the default process group's, or ``store``).  A peer that never arrives does not
    hang the kernel: it gives up after ``timeout_s`` and ``error()`` turns non-zero.

    A timed-out call writes NaN (not a sum of possibly stale peer buffers) over the shares it
    could not complete, so the optimizer's finite gate skips that step, and ``error()``
    reports it (the watchdog aborts on it).  The kernel's sequence counters assume its calls
    are serialized: NativeComm issues every IPC call on ``self.stream`` (ordered after the
    caller's stream and joined back).  Its ``blocks`` workgroups must all get scheduled for a
    call to complete (csrc/comm/oneshot.hip: co-residency), so keep ``blocks`` small.

    Validated with two processes sharing one GPU (tests/test_ipc_gpu.py); the cross-GPU
    path over xGMI has not been measured by the builder (no multi-GPU box), so NativeComm
    routes small buckets here only when asked (``ipc_small_bytes`` / DG_IPC_SMALL)."""
    kind = "ipc"
    in_graph = True
    _seq = 0

    def __init__(self, device, capacity_bytes: int, world: Optional[int] = None,
                 rank: Optional[int] = None, store=None, mod=None, timeout_s: float = 10.0,
                 blocks: int = 16):
        if mod is None:
            from ..ops.native import comm as _comm_mod
            mod = _comm_mod()
        self.device = torch.device(device)
        if world is None:
            world = dist.get_world_size() if dist.is_initialized() else 1
            rank = dist.get_rank() if dist.is_initialized() else 0
        self.world, self.rank, self.blocks = world, rank, blocks
        self.c = mod.IpcOneShot(world, rank, self.device.index or 0, int(capacity_bytes),
                                float(timeout_s))
        self.capacity = int(self.c.capacity())
        key = f"dg_ipc_{IpcOneShot._seq}"
        IpcOneShot._seq += 1
        if world > 1:
            if store is None:
                store = dist.distributed_c10d._get_default_store()
            hb, hf = bytes(self.c.handle_buf()), bytes(self.c.handle_flags())
            store.set(f"{key}_{rank}", (hb + hf).hex())
            pairs = []
            for j in range(world):
                v = bytes.fromhex(store.get(f"{key}_{j}").decode())
                pairs.append((v[:len(hb)], v[len(hb):]))
        else:
            pairs = [(b"", b"")]
        self.c.open_peers(pairs)
        self.stream = torch.cuda.Stream(device=self.device)

    def fits(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return (t.dtype in (torch.float32, torch.bfloat16) and t.is_contiguous()
                and nb <= self.capacity and nb % 16 == 0)

    def all_reduce_(self, t: torch.Tensor, stream=None, op: str = "sum"):
        if op != "sum" or not self.fits(t):
            raise ValueError("ipc one-shot: contiguous fp32/bf16 sum, a multiple of 16 B "
                             "within capacity")
        s = stream if stream is not None else self.stream
        self.c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(),
                          "fp32" if t.dtype == torch.float32 else "bf16", self.blocks,
                          int(s.cuda_stream))
        return t

    def error(self) -> int:
        return int(self.c.error())

    def close(self):
        torch.cuda.synchronize(self.device)
        self.c.close()


class NativeComm:
    """The native RCCL communicator (csrc/comm/comm.cpp, ``_dgcomm``) on its own HIP stream.

    Its collectives are plain stream-ordered ncclAllReduce calls, so the training step can
    capture them INSIDE its hipGraph: forked from the compute stream by an event once a
    bucket's gradients are final, joined back before the optimizer (``SegmentedStep`` mode
    "dp-graph").  Rendezvous: rank 0's unique id travels through torch.distributed's store;
    world 1 (``bench.py --force-dp``) needs no process group."""
    kind = "native"
    in_graph = True
    _seq = 0

    def __init__(self, device, mod=None, stream=None, ipc_small_bytes: Optional[int] = None):
        if mod is None:
            from ..ops.native import comm as _comm_mod
            mod = _comm_mod()
        self.mod = mod
        device = torch.device(device)
        self.device = device
        if dist.is_initialized():
            self.world, self.rank = dist.get_world_size(), dist.get_rank()
        else:
            self.world, self.rank = 1, 0
        # every rank constructs its communicators in the same order, so the n-th one of
        # each rank meets under the same store key
        self.key = f"dg_rccl_uid_{NativeComm._seq}"
        NativeComm._seq += 1
        if self.world > 1:
            store = dist.distributed_c10d._get_default_store()
            if self.rank == 0:
                store.set(self.key, mod.unique_id().hex())
            uid = bytes.fromhex(store.get(self.key).decode())
        else:
            uid = mod.unique_id()
        self.uid = uid
        self.c = mod.Comm(uid, self.world, self.rank, device.index or 0)
        self.stream = stream if stream is not None else torch.cuda.Stream(device=device)
        # buckets up to ipc_small_bytes take the one-shot IPC all-reduce (one node only;
        # off unless asked: DG_IPC_SMALL=<bytes>)
        if ipc_small_bytes is None:
            ipc_small_bytes = int(os.environ.get("DG_IPC_SMALL", "0"))
        one_node = int(os.environ.get("LOCAL_WORLD_SIZE", self.world)) == self.world
        self.ipc = (IpcOneShot(device, ipc_small_bytes, self.world, self.rank, mod=mod)
                    if ipc_small_bytes > 0 and self.world > 1 and one_node else None)

    def version(self) -> int:
        return int(self.mod.version())

    @staticmethod
    def _dt(t: torch.Tensor) -> str:
        return {torch.float32: "fp32", torch.bfloat16: "bf16", torch.float64: "fp64",
                torch.int32: "i32", torch.int64: "i64", torch.float16: "fp16"}[t.dtype]

    def all_reduce_(self, t: torch.Tensor, stream=None, op: str = "sum", use_ipc: bool = True):
        """In-place all-reduce of a contiguous tensor on ``stream`` (default: comm stream).
        Buckets the IPC one-shot takes run on ITS stream (every IPC call serialized there:
        the kernel's sequence counters assume one call at a time), ordered after ``stream``
        and joined back into it; ``use_ipc=False`` forces RCCL."""
        s = stream if stream is not None else self.stream
        if use_ipc and self.ipc is not None and op == "sum" and self.ipc.fits(t):
            ist = self.ipc.stream
            if s != ist:
                ist.wait_stream(s)
            self.ipc.all_reduce_(t, stream=ist)
            if s != ist:
                s.wait_stream(ist)
            return t
        self.c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), op,
                          int(s.cuda_stream))
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        """Blocking (w.r.t. the current stream) broadcast, e.g. the initial parameters."""
        if self.world > 1:
            cur = torch.cuda.current_stream(self.device)
            self.stream.wait_stream(cur)
            self.c.broadcast(t.data_ptr(), t.numel(), self._dt(t), root,
                             int(self.stream.cuda_stream))
            cur.wait_stream(self.stream)
        return t

    def seen(self) -> dict:
        """What the RCCL communicator itself reports (ncclCommCount / UserRank / CuDevice),
        independent of the environment this rank was started with."""
        try:
            return {"ranks_seen": int(self.c.count()), "user_rank": int(self.c.user_rank()),
                    "device": int(self.c.device())}
        except (AttributeError, RuntimeError) as e:   # an older _dgcomm build / aborted comm
            return {"error": str(e)}

    def async_error(self) -> str:
        if self.ipc is not None and self.ipc.error():
            return "ipc one-shot all-reduce: a peer never arrived (timed out)"
        return self.c.async_error()

    def abort(self):
        self.c.abort()

    def close(self):
        torch.cuda.synchronize(self.device)
        if self.ipc is not None:
            self.ipc.close()
        self.c.destroy()


class ProxyComm:
    """World-1 stand-in for an in-graph collective (``bench.py --force-dp --comm proxy``):
    ``all_reduce_`` launches an RCCL-shaped kernel on the comm stream, where the ring
    all-reduce would run: ``blocks`` channel workgroups stream 2(n-1)/n x the bucket's bytes
    (values unchanged), paced to the wire time at ``gbps`` (csrc/kernels/elementwise.hip
    comm_proxy_kernel).  The step time with it vs without prices the comm kernels'
    co-scheduling beside the compute launches; its kernel trace shows the overlap
    (tools/overlap_report.py).  Not a collective: world must be 1."""
    kind = "proxy"
    in_graph = True

    def __init__(self, device, world: int = 8, gbps: float = 300.0, blocks: int = 32):
        from ..ops.native import hip
        self.h = hip()
        self.device = torch.device(device)
        self.world, self.rank = 1, 0
        self.proxy_world, self.gbps, self.blocks = world, gbps, blocks
        self.stream = torch.cuda.Stream(device=self.device)

    def all_reduce_(self, t: torch.Tensor, stream=None, op: str = "sum"):
        s = stream if stream is not None else self.stream
        nbytes = t.numel() * t.element_size() // 16 * 16
        self.h.comm_proxy(t.data_ptr(), nbytes, self.proxy_world, self.gbps, self.blocks,
                          int(s.cuda_stream))
        return t

    def broadcast_(self, t: torch.Tensor, root: int = 0):
        return t

    def seen(self) -> dict:
        return {"ranks_seen": 1, "user_rank": 0, "proxy_world": self.proxy_world}

    def async_error(self) -> str:
        return ""

    def close(self):
        pass


def agree(ok: bool, device=None) -> bool:
    """True iff ``ok`` holds on EVERY rank (MIN all-reduce over the default process group;
    world 1 / no process group: ``ok`` itself).  Used so that a per-rank decision (native
    communicator or fallback) is taken by all ranks together: a rank that silently chose
    differently would issue collectives its peers never pair with."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(ok)
    dev = device if (dist.get_backend() == "nccl" and device is not None) else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def make_communicator(kind: str, device, selftest: Optional[Callable] = None,
                      load_module: Optional[Callable] = None,
                      native_factory: Optional[Callable] = None, **proxy_kw):
    """``native`` | ``torch`` | ``auto`` (| ``proxy``, world 1 only).

    ``auto`` takes the native in-graph communicator when EVERY rank can: the choice is made
    collectively in three phases, each closed by an ``agree`` (MIN all-reduce of an ok flag)
    so no rank ever waits in a collective its peers skipped:
      1. local prerequisites (the ``_dgcomm`` module loads) — agreed BEFORE any rank enters
         the collective ``ncclCommInitRank``;
      2. ``ncclCommInitRank`` (unique id through the c10d store) and ``selftest`` (an eager
         and a graph-captured all-reduce, the same collective sequence on every rank, the
         sums checked only after all of them ran);
      3. if any rank failed 1 or 2, the ranks whose native communicator came up abort it and
         ALL ranks return a ``TorchComm`` (reported by ``comm.kind``; bench JSON "comm").
    ``native``: the same, but a failure on any rank raises on every rank.
    A rank that hangs inside RCCL is not recoverable here: bench.py's per-rank hang guard
    and the trainer's StepWatchdog bound that case.

    ``selftest`` / ``load_module`` / ``native_factory(module)`` are injectable so the
    protocol runs under a CPU gloo world with a stub module (tests/test_dist_cpu.py)."""
    if kind == "torch":
        return TorchComm()
    if kind == "proxy":
        if dist.is_initialized() and dist.get_world_size() > 1:
            raise ValueError("the proxy communicator is world-1 only")
        return ProxyComm(device, **proxy_kw)
    if kind not in ("auto", "native"):
        raise ValueError(f"unknown communicator kind {kind!r}")
    import sys
    selftest = selftest_in_graph if selftest is None else selftest
    if load_module is None:
        from ..ops.native import comm as load_module
    factory = native_factory or (lambda mod: NativeComm(device, mod=mod))
    err = None
    mod = None
    try:
        mod = load_module()
    except Exception as e:  # noqa: BLE001
        err = e
    if agree(err is None, device):
        c = None
        try:
            c = factory(mod)
            if kind == "auto":
                selftest(c)
        except Exception as e:  # noqa: BLE001
            err = e
        if agree(err is None, device):
            return c
        if c is not None:
            try:
                c.abort()
            except Exception:  # noqa: BLE001
                pass
    why = err if err is not None else "another rank failed its native communicator set-up"
    if kind == "native":
        raise RuntimeError(f"native communicator unavailable on some rank: {why}")
    print(f"[dp] native communicator unavailable ({why}); every rank uses torch.distributed",
          file=sys.stderr, flush=True)
    return TorchComm()


def selftest_in_graph(c: NativeComm, n: int = 4096):
    """Capture ONE all-reduce on the comm stream into a hipGraph forked from / joined to the
    capturing stream (the step graph's structure), replay it twice, check the sums.  Every
    collective runs before any check raises, so all ranks issue the same sequence."""
    dev = c.device
    # RCCL itself (use_ipc=False: a small test buffer would otherwise take the one-shot IPC
    # path when DG_IPC_SMALL covers it, and the RCCL connection would go untested)
    rccl = {"use_ipc": False} if getattr(c, "ipc", None) is not None else {}
    x = torch.empty(n, dtype=torch.float32, device=dev)
    x.fill_(float(c.rank + 1))
    c.all_reduce_(x, stream=torch.cuda.current_stream(dev), **rccl)   # eager: connects it
    torch.cuda.synchronize(dev)
    want = float(c.world * (c.world + 1) // 2)
    eager_ok = bool((x == want).all())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        cur = torch.cuda.current_stream(dev)
        x.fill_(float(c.rank + 1))
        c.stream.wait_stream(cur)
        c.all_reduce_(x, **rccl)
        cur.wait_stream(c.stream)
        x.mul_(2.0)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize(dev)
    graph_ok = bool((x == 2 * want).all())
    del g
    if not eager_ok:
        raise RuntimeError("native all-reduce self-test: wrong eager sum")
    if not graph_ok:
        raise RuntimeError("native all-reduce self-test: wrong in-graph sum")


class GradBucketer:
    """All-reduces flat-gradient buckets.

    torch communicator: ``fire(b)`` issues an async all-reduce from the host (between graph
    segments); ``wait()`` joins them all.
    native communicator: ``enqueue(b)`` forks the comm stream from the current (compute)
    stream and queues the bucket's all-reduce there — graph-capturable; ``join()`` makes the
    current stream wait for every queued bucket.

    ``grad_dtype="bf16"``: the wire format is bf16 (half the bytes).  With ``shadow`` (the
    model's bf16 gradient twin, HipGoNet(grad_wire="bf16").grads16, written by the gradient
    reduce kernels themselves) the buckets are all-reduced in place on it and the optimizer
    reads it: no conversion kernels.  Without, the bucket is rounded into a private bf16
    shadow on the comm stream and the sum written back to the fp32 gradients."""

    def __init__(self, grads: torch.Tensor, buckets: List[Tuple[int, int, int]],
                 group=None, grad_dtype: str = "fp32", comm=None,
                 shadow: Optional[torch.Tensor] = None):
        self.grads = grads
        self.buckets = buckets
        self.comm = comm if comm is not None else TorchComm(group)
        self.group = group
        self.grad_dtype = grad_dtype
        self.works = []
        self._shadow = None
        self.direct = False          # all-reduce the model's own bf16 twin (no copies)
        # DG_CHECK_STREAMS=1: the fork / join hand-offs with the comm stream are checked too
        # (the model's checker when the step attaches it: SegmentedStep)
        self.sc = None
        if grad_dtype == "bf16":
            if shadow is not None:
                if shadow.dtype != torch.bfloat16 or shadow.numel() != grads.numel():
                    raise ValueError("shadow must be a bf16 twin of the flat gradient")
                self._shadow = shadow
                self.direct = True
            else:
                self._shadow = torch.empty(grads.numel(), dtype=torch.bfloat16,
                                           device=grads.device)

    @property
    def in_graph(self) -> bool:
        return self.comm.in_graph

    # -- torch.distributed path (host-issued between segments)
    def fire(self, b: int):
        if self.in_graph:
            return self.enqueue(b)
        s, e, _ = self.buckets[b]
        if self._shadow is not None:
            sh = self._shadow[s:e]
            if not self.direct:
                sh.copy_(self.grads[s:e])
            self.works.append((self.comm.all_reduce_async(sh), b))
        else:
            self.works.append((self.comm.all_reduce_async(self.grads[s:e]), b))

    def wait(self):
        if self.in_graph:
            return self.join()
        for w, b in self.works:
            w.wait()
            if self._shadow is not None and not self.direct:
                s, e, _ = self.buckets[b]
                self.grads[s:e].copy_(self._shadow[s:e])
        self.works = []

    # -- native path (stream-ordered; capturable)
    def enqueue(self, b: int):
        s, e, _ = self.buckets[b]
        cs = self.comm.stream
        cur = torch.cuda.current_stream()
        if self.sc:
            self.sc.produce(f"bucket{b}->comm", cur)
        cs.wait_stream(cur)                              # bucket's gradients final
        if self.sc:
            self.sc.consume(f"bucket{b}->comm", cs)
        with torch.cuda.stream(cs):
            if self._shadow is not None:
                sh = self._shadow[s:e]
                if self.direct:
                    self.comm.all_reduce_(sh)
                else:
                    sh.copy_(self.grads[s:e])
                    self.comm.all_reduce_(sh)
                    self.grads[s:e].copy_(sh)
            else:
                self.comm.all_reduce_(self.grads[s:e])

    def join(self):
        cur = torch.cuda.current_stream()
        if self.sc:
            self.sc.produce("comm->join", self.comm.stream)
        cur.wait_stream(self.comm.stream)
        if self.sc:
            self.sc.consume("comm->join", cur)


BF16_UNIT_ROUNDOFF = 2.0 ** -8    # bf16: 8 significand bits, round to nearest even


def ring_allreduce_emulate(parts: Sequence[torch.Tensor],
                           buckets: Optional[Sequence[Tuple[int, int, int]]] = None,
                           wire: torch.dtype = torch.bfloat16) -> torch.Tensor:
    """What a ring all-reduce of ``len(parts)`` ranks' flat gradients (each already in the
    wire dtype: the bf16 twin every gradient pass 2 writes) hands back, rounding like RCCL's
    reduction kernels: every hop of the reduce-scatter loads the incoming partial sum and the
    local value, adds them in fp32 and stores the result in the wire dtype.  Each bucket is
    cut into ``n`` contiguous chunks; chunk c is accumulated in rank order c+1, c+2, ...,
    c+n (mod n), so its n-1 additions are rounded n-1 times (the all-gather half copies).
    That is the most roundings any of RCCL's algorithms applies to one element (a tree's
    reduce rounds at most depth <= n-1 times), so bounds shown for this emulation hold for
    the real collective.  Returns the reduced gradient in the wire dtype.
    Reference: the DataParallelTable reduces fp32 gradients (experiments.lua:155-168)."""
    n = len(parts)
    if n == 0:
        raise ValueError("no ranks")
    numel = parts[0].numel()
    if any(p.numel() != numel for p in parts):
        raise ValueError("every rank's gradient must have the same size")
    stack = torch.stack([p.reshape(-1).to(wire) for p in parts])     # [n, numel]
    out = torch.empty(numel, dtype=wire, device=stack.device)
    for s, e, _ in (buckets or [(0, numel, 0)]):
        bounds = [s + (e - s) * c // n for c in range(n + 1)]
        for c in range(n):
            lo, hi = bounds[c], bounds[c + 1]
            if hi <= lo:
                continue
            order = [(c + 1 + j) % n for j in range(n)]
            acc = stack[order[0], lo:hi]
            for r in order[1:]:
                acc = (acc.float() + stack[r, lo:hi].float()).to(wire)
            out[lo:hi] = acc
    return out


def recursive_sum_bound(parts: Sequence[torch.Tensor], u: float = BF16_UNIT_ROUNDOFF) -> torch.Tensor:
    """Elementwise a-priori bound on |fl(ring sum) - exact sum| for n terms summed with n-1
    roundings of unit roundoff u (Higham, recursive summation): gamma_{n-1} * sum |x_i|,
    gamma_k = k u / (1 - k u).  The terms are the wire-dtype values themselves."""
    n = len(parts)
    k = n - 1
    gamma = k * u / (1.0 - k * u)
    return gamma * torch.stack([p.reshape(-1).double().abs() for p in parts]).sum(0)


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
