"""Experiment = config + state + checkpoint, and the training / validation loop.

Reference map:
* ``Experiment:new`` / ``basicGoExperiment`` / ``init`` / ``run`` / ``save`` / ``load``
  (``experiments.lua:8-131``) -> ``Experiment(cfg)``, ``init()``, ``run(iters)``, ``save()``,
  ``Experiment.load(path, reset_optimizer=...)`` (``reset_optimizer`` = ``repeated.lua:17``).
* ``train(experiment, {iters})`` (``train.lua:47-142``): a fixed validation set drawn once per
  ``run`` call; per iteration fwd+bwd, EMA(0.95/0.05) of the training cost,
  ``iterations += 1``, logging / validation + checkpoint, THEN the optimizer step (same order
  as ``train.lua:113-131``).  The reference ran fwd/bwd twice per iteration
  (``train.lua:106-111``, pcall + eval); that doubling is not replicated.
* ``eval_validation`` (``train.lua:14-45``): exact by default (every sample, partial last
  chunk included); ``reference_validation_quirks=True`` reproduces floor(N/bs) chunks and the
  (bs-1) cost weight with denominator N.
* The validation check runs every iteration (the reference only looked when
  ``iterations % 10 == 0``, so intervals not divisible by 10 never validated).
"""
from __future__ import annotations

import collections
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import ExperimentConfig
from ..data.dataset import GameIndex, PackedDataset, load_index
from ..data.loader import BatchLoader
from ..parallel import dp
from ..utils import trace
from ..utils import checkpoint as ckpt
from ..utils.faults import (NonFiniteLoss, SkipGuard, StepWatchdog, check_finite, dump_batch,
                            maybe_inject, parse_fault)
from ..utils.metrics import MetricsSink

# step timeout (seconds) armed under the native RCCL communicator when DG_STEP_TIMEOUT is
# unset: a hung in-graph collective of a live-but-stuck peer raises no async error
DEFAULT_NATIVE_STEP_TIMEOUT = 600.0


def synthetic_dataset(n: int, seed: int) -> PackedDataset:
    from ..data.synthetic import engine_positions
    planes, player, rank, label = engine_positions(n, seed, max_moves=250)
    return PackedDataset.from_arrays(planes, player, rank, label, game_size=200)


class Experiment:
    def __init__(self, cfg: ExperimentConfig, id: Optional[str] = None):
        self.cfg = cfg
        self.id = id or cfg.id or f"{np.random.default_rng().random():.14f}"
        self.iterations = 0
        self.validation_costs: List[float] = []
        self.validation_accuracies: List[float] = []
        self.train_costs: List[float] = []
        self.initialized = False
        self.loader_seq = 0           # batches consumed from the training stream
        self._restore_params = None
        self._restore_opt = None
        self.backend = None
        self.info = dp.env_info()

    # ------------------------------------------------------------------ setup
    def _device_kind(self) -> str:
        return "hip" if (self.cfg.useCuda and torch.cuda.is_available()) else "cpu"

    def _source(self, split: str):
        cfg = self.cfg
        if cfg.synthetic:
            n = {"train": 4096, "validation": 1024, "test": 1024}[split]
            seed = cfg.seed * 7 + {"train": 1, "validation": 2, "test": 3}[split]
            return synthetic_dataset(n, seed)
        pack = os.path.join(cfg.data_root, f"{cfg.directory(split)}.dgpack.npz")
        if os.path.exists(pack):
            return PackedDataset.load(pack)
        return load_index(cfg.data_root, cfg.directory(split))

    def init(self):
        cfg = self.cfg
        torch.manual_seed(cfg.seed)
        info = dp.init_distributed() if self.info.world > 1 else self.info
        self.info = info
        world = info.world
        if cfg.batchSize % world:
            raise ValueError(f"batchSize {cfg.batchSize} not divisible by world {world}")
        self.local_batch = cfg.batchSize // world
        if self._device_kind() == "hip":
            from .backends import HIPBackend
            self.backend = HIPBackend(cfg, self.local_batch, flat=self._restore_params,
                                      world=world, bucket_mb=cfg.bucket_mb,
                                      grad_dtype=cfg.grad_dtype, comm=cfg.comm)
        else:
            from .backends import CPUBackend
            self.backend = CPUBackend(cfg, self.local_batch, flat=self._restore_params,
                                      world=world, bucket_mb=cfg.bucket_mb)
            if world > 1 and self._restore_params is None:
                dp.broadcast_(self.backend.params.data, 0)
        if self._restore_opt is not None:
            self.backend.load_state_dict({"optimizer": self._restore_opt})
        self.sources = {s: self._source(s) for s in ("train", "validation")}
        self.metrics = MetricsSink(cfg.metrics_path, rank=info.rank)
        self.initialized = True
        self.metrics.line("initializing model...")

    def _train_loader(self) -> BatchLoader:
        c = self.cfg
        return BatchLoader(self.sources["train"], self.local_batch, threads=c.loader_threads,
                           prefetch=c.prefetch, seed=c.seed * 1000003 + self.info.rank,
                           sampling=c.sampling, start_seq=self.loader_seq)

    def _regenerate_batch(self, seq):
        """The training batch the loader produced at sequence number ``seq`` (the loader is
        deterministic per (seed, rank, sequence): a fresh one started at ``seq`` yields the
        same batch), or None."""
        if seq is None:
            return None
        try:
            c = self.cfg
            ld = BatchLoader(self.sources["train"], self.local_batch, threads=1, prefetch=2,
                             seed=c.seed * 1000003 + self.info.rank, sampling=c.sampling,
                             start_seq=seq, pin=False)
            try:
                return ld.next_numpy()
            finally:
                ld.close()
        except Exception:  # noqa: BLE001  (the dump is best effort; the raise is what matters)
            return None

    # ------------------------------------------------------------------ validation
    def draw_validation(self, n: int, split: str = "validation", seed_offset: int = 0):
        src = self.sources.get(split) or self._source(split)
        ld = BatchLoader(src, n, threads=self.cfg.loader_threads, prefetch=2,
                         seed=self.cfg.seed * 7919 + 17 + seed_offset + self.iterations,
                         sampling=self.cfg.sampling, pin=False)
        batch = ld.next_numpy()
        ld.close()
        return batch

    def eval_batch_set(self, data, quirks: Optional[bool] = None):
        """(cost, accuracy) of a fixed sample set, chunked by the local batch size and sharded
        across DP ranks (sums all-reduced)."""
        quirks = self.cfg.reference_validation_quirks if quirks is None else quirks
        planes, player, rank, labels = data
        N = len(labels)
        bs = self.local_batch
        world, r = self.info.world, self.info.rank
        nchunks = N // bs if quirks else (N + bs - 1) // bs
        cost_sum = 0.0
        err = 0.0
        for c in range(r, nchunks, world):
            lo, hi = c * bs, min(N, (c + 1) * bs)
            n = hi - lo
            sl = slice(lo, hi)
            if n < bs:  # pad the partial last chunk; only n boards are scored
                pad = bs - n
                pp = np.concatenate([planes[sl], np.zeros((pad,) + planes.shape[1:], np.uint8)])
                py_ = np.concatenate([player[sl], np.ones(pad, np.uint8)])
                rk = np.concatenate([rank[sl], np.ones(pad, np.uint8)])
                lb = np.concatenate([labels[sl], np.zeros(pad, np.int32)])
                self.backend.set_batch(pp, py_, rk, lb)
            else:
                self.backend.set_batch(planes[sl], player[sl], rank[sl], labels[sl])
            self.backend.evaluate(n)
            ls, corr = self.backend.loss_sum(), self.backend.correct()
            if quirks:
                cost_sum += (ls / n) * (n - 1)  # train.lua:40-41 weight = range[2]-range[1]
            else:
                cost_sum += ls
            err += n - corr
        cost_sum, err = dp.all_reduce_scalars([cost_sum, err])
        return cost_sum / N, 1.0 - err / N

    # ------------------------------------------------------------------ training
    def run(self, iters: int) -> Dict[str, float]:
        assert iters > 0  # experiments.lua:111
        if not self.initialized:
            self.init()
        cfg, be, info = self.cfg, self.backend, self.info
        val = self.draw_validation(cfg.validationSize)
        loader = self._train_loader()
        fault = parse_fault()
        # step timeout (DG_STEP_TIMEOUT seconds) and, with the native RCCL communicator,
        # ncclCommGetAsyncError polling.  RCCL reports no async error for a peer that is
        # alive but stuck, so under the native communicator a step timeout is always armed
        # (default DEFAULT_NATIVE_STEP_TIMEOUT s: generous against any step, validation or
        # checkpoint between two beats)
        comm = getattr(be, "comm", None)
        comm = comm if comm is not None and comm.kind == "native" else None
        timeout = os.environ.get("DG_STEP_TIMEOUT")
        if timeout is None and comm is not None:
            timeout = str(DEFAULT_NATIVE_STEP_TIMEOUT)
        watchdog = (StepWatchdog(float(timeout or 0), comm=comm)
                    if timeout or comm is not None else None)
        ema = self.train_costs[-1] if self.train_costs else None
        skipguard = (SkipGuard(cfg.nan_max_skips, be.bad_steps())
                     if cfg.nan_policy == "guard" else None)
        # guard: the loader sequence number of each recent step's batch, so the batch dumped
        # when SkipGuard raises is the FIRST of the skipped run (regenerated from the
        # deterministic loader), not the batch of the step whose check noticed it
        seq_ring = collections.deque(maxlen=cfg.nan_max_skips + 2 * cfg.log_interval + 2)
        t_start = time.perf_counter()
        t_log = t_start
        n_log = 0
        last_val = None
        save_now = False
        try:
            for _ in range(iters):
                seq0 = loader.consumed
                with trace.range("load_batch"):
                    batch = be.load_next(loader)
                self.loader_seq = loader.consumed
                step = self.iterations + 1
                seq_ring.append((step, seq0))
                # nothing reads the pre-update state this iteration (no validation, no host NaN
                # check before the update): forward/backward + update as one fused step
                fused = (step % cfg.validation_interval != 0 and cfg.nan_policy != "raise"
                         and not fault)
                # the rate this iteration's update uses, read before the step so fused and unfused
                # iterations log the same thing (only on logging iterations: it syncs the device)
                lr_now = (be.rate if step % cfg.log_interval == 0
                          or step % cfg.validation_interval == 0 else None)
                with trace.range("fwd_bwd"):
                    if fused:
                        be.train_step()
                    else:
                        be.forward_backward()
                inj = maybe_inject(info.rank, step, fault) if fault else None
                need_cost = (step % cfg.log_interval == 0) or (step % cfg.validation_interval == 0) \
                    or ema is None or cfg.nan_policy == "raise"
                if need_cost:
                    loss = be.loss_sum() / self.local_batch
                    if inj == "nan":
                        loss = float("nan")
                    if cfg.nan_policy == "raise" and be.gradient_tagged():
                        # a gradient producer's range check fired (finite loss, |dZ| or a
                        # gradient out of range): raise like a non-finite loss, with the dump,
                        # instead of letting the update skip the step silently
                        loss = float("nan")
                    if batch is None and not np.isfinite(loss):
                        batch = be.current_batch()  # only for the bad-batch dump
                    if not check_finite(loss, step, cfg.nan_policy, batch, cfg.checkpoint_dir):
                        loss = ema if ema is not None else 0.0
                    ema = loss if ema is None else 0.95 * ema + 0.05 * loss
                self.iterations = step
                n_log += 1
                if step % cfg.validation_interval == 0:
                    with trace.range("validation"):
                        vc, va = self.eval_batch_set(val)
                    last_val = vc
                    self.validation_costs.append(vc)
                    self.validation_accuracies.append(va)
                    self.metrics.line(f"validation at iteration {step}: cost={vc}, accuracy={va}")
                    self.metrics.record(kind="validation", step=step, val_cost=vc, val_acc=va,
                                        lr=lr_now)
                    # the reference saves here, BEFORE this iteration's update (train.lua:124):
                    # that checkpoint pairs iteration N with N-1 updates.  We save after the
                    # update below so a resumed run continues bit-exactly (auto-resume).
                    save_now = info.is_main
                if step % cfg.log_interval == 0:
                    now = time.perf_counter()
                    bps = n_log * cfg.batchSize / max(now - t_log, 1e-9)
                    self.train_costs.append(ema)
                    if step % cfg.validation_interval != 0:
                        self.metrics.line(f"training {ema} (samples per second {bps:.1f})")
                    self.metrics.record(kind="train", step=step, loss_ema=ema, boards_per_sec=bps,
                                        lr=lr_now)
                    t_log, n_log = now, 0
                if not fused:
                    with trace.range("optimizer"):
                        be.optimizer_step()
                # (after the update: the device's skip counter then includes this step)
                if skipguard is not None:
                    skipguard.step()
                    if need_cost:
                        try:
                            skipguard.check(be.bad_steps(), step)
                        except NonFiniteLoss:
                            first = step - skipguard.run + 1
                            b = self._regenerate_batch(dict(seq_ring).get(first))
                            if b is None:
                                first = step
                                b = batch if batch is not None else be.current_batch()
                            dump_batch(b, first, cfg.checkpoint_dir)
                            raise
                if save_now:
                    with trace.range("checkpoint"):
                        self.save()
                    save_now = False
                if watchdog:
                    watchdog.beat()
            if torch.cuda.is_available() and self._device_kind() == "hip":
                torch.cuda.synchronize()
            total = time.perf_counter() - t_start
        finally:
            # also when the loop raises (NonFiniteLoss, a loader error): a live watchdog would
            # later os._exit() a process that may still be saving or running other work
            loader.close()
            if watchdog:
                watchdog.stop()
        tps = cfg.batchSize * iters / total
        self.metrics.line(f"total samples per second {tps:.1f}")
        row = {"name": f"{cfg.name}:{self.id}", "numLayers": cfg.numLayers,
               "channelSize": cfg.channelSize, "batchSize": cfg.batchSize, "rate": cfg.rate,
               "rateDecay": cfg.rateDecay, "train_cost": ema, "runningTime": total,
               "val_cost": last_val, "iterations": self.iterations}
        self.metrics.run_summary(row)
        return {"train_cost": ema, "val_cost": last_val, "samples_per_sec": tps,
                "iterations": self.iterations}

    def evaluate_split(self, split: str = "test", n: Optional[int] = None):
        """Top-1 accuracy / NLL on a split (the reference never evaluated its test split)."""
        if not self.initialized:
            self.init()
        data = self.draw_validation(n or self.cfg.validationSize, split=split, seed_offset=99)
        return self.eval_batch_set(data)

    def close(self):
        """Release the backend's communicator (ncclCommDestroy after a device sync) while
        every peer is still alive, instead of in a destructor at interpreter teardown."""
        be = self.backend
        if be is not None and hasattr(be, "close"):
            be.close()

    # ------------------------------------------------------------------ checkpoint
    def state(self):
        return {"id": self.id, "iterations": self.iterations,
                "validation_costs": self.validation_costs,
                "validation_accuracies": self.validation_accuracies,
                "train_costs": self.train_costs, "loader_seq": self.loader_seq,
                "world": self.info.world}

    def checkpoint_path(self) -> str:
        return os.path.join(self.cfg.checkpoint_dir, f"{self.id}.model")

    def save(self, path: Optional[str] = None) -> str:
        path = path or self.checkpoint_path()
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        opt = self.backend.state_dict()["optimizer"]
        return ckpt.save_checkpoint(path, self.cfg, self.backend.flat_params(), self.state(), opt)

    def export_t7(self, path: str) -> str:
        return ckpt.export_t7(path, self.cfg, self.backend.flat_params(), self.state(),
                              self.backend.rate)

    @classmethod
    def load(cls, path: str, reset_optimizer: bool = False, **overrides) -> "Experiment":
        cfg, flat, state, opt = ckpt.load_checkpoint(path)
        if overrides:
            cfg = cfg.replace(**overrides)
        e = cls(cfg, id=state.get("id"))
        e.iterations = int(state.get("iterations", 0))
        e.validation_costs = list(state.get("validation_costs", []))
        e.validation_accuracies = list(state.get("validation_accuracies", []))
        e.train_costs = list(state.get("train_costs", []))
        e.loader_seq = int(state.get("loader_seq", 0))
        e._restore_params = flat
        if not reset_optimizer:  # repeated.lua:17 resets to the original rate
            e._restore_opt = opt
        return e
