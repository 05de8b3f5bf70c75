"""Compute backends behind the Experiment (one per device type).

Both expose the same small surface used by the training loop:
  set_batch(planes uint8 [B,9,19,19], player, rank, labels)   (host numpy or tensors)
  forward_backward()         loss/argmax of the batch + gradients (global-batch mean)
  optimizer_step()           SGD/RMSProp + per-step LR decay
  evaluate(n)                forward only on the first n boards of the current batch
  loss_sum() / correct()     of the last forward (host floats; synchronising)
  params / rate / state_dict / load_state_dict

* ``CPUBackend`` — fp32 PyTorch on the CPU (the reference's useCuda=false path,
  experiments.lua:97; also the numerical oracle).  DP over gloo.
* ``HIPBackend`` — the MI355X executor (models/hip_model.py) with hipGraph replay and, for
  world > 1, RCCL gradient buckets overlapped with backward.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

import torch
import torch.nn.functional as F

from ..config import ExperimentConfig
from ..models.gocnn import ParamLayout, init_params, reference_forward
from ..ops.native import cpu
from ..parallel import dp
from .optim import SGD, RMSProp


def _np(x, dtype):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().astype(dtype, copy=False)
    return np.asarray(x, dtype=dtype)


class CPUBackend:
    def __init__(self, cfg: ExperimentConfig, batch: int, flat: Optional[torch.Tensor] = None,
                 world: int = 1, bucket_mb: float = 4.0):
        self.cfg = cfg
        self.layout = ParamLayout(cfg)
        self.B = batch
        self.world = world
        self.params = (flat.clone().float() if flat is not None
                       else init_params(self.layout, cfg.seed)).contiguous()
        self.params.requires_grad_(True)
        if cfg.optimizer == "rmsprop":
            self.opt = RMSProp(cfg.rate, cfg.rmsprop_decay, self.layout.numel)
        else:
            self.opt = SGD(cfg.rate, cfg.rateDecay)
        self._x = None
        self._y = None
        self._loss_sum = 0.0
        self._correct = 0
        self.bucketer = None
        if world > 1:
            ranges = [self.layout.layer_range(i) for i in range(len(self.layout.layers))]
            self.buckets = dp.make_buckets(ranges, int(bucket_mb * 2 ** 20))
        self.nan_skipped = 0
        self._last = "train"
        self._eval = (0.0, 0)

    @property
    def rate(self) -> float:
        return self.opt.rate

    def load_next(self, loader):
        batch = loader.next_numpy()
        self.set_batch(*batch)
        return batch

    def set_batch(self, planes, player, rank, labels):
        pl = _np(planes, np.uint8).reshape(-1, 9, 19, 19)
        self._x = torch.from_numpy(cpu().expand(pl, _np(player, np.uint8), _np(rank, np.uint8),
                                                 self.cfg.ko_plane))
        self._y = torch.from_numpy(_np(labels, np.int64))

    def _forward(self, x):
        return reference_forward(self.layout, self.params, x, head_relu=self.cfg.head_relu)

    def forward_backward(self):
        if self.params.grad is not None:
            self.params.grad.zero_()
        logp = self._forward(self._x)
        # mean over the GLOBAL batch: local mean / world, then SUM all-reduce
        loss = F.nll_loss(logp, self._y, reduction="sum") / (self.B * self.world)
        loss.backward()
        with torch.no_grad():
            self._loss_sum = float(F.nll_loss(logp, self._y, reduction="sum"))
            self._correct = int((logp.argmax(1) == self._y).sum())
        self._last = "train"
        if self.world > 1:
            g = self.params.grad
            works = [torch.distributed.all_reduce(g[s:e], async_op=True)
                     for s, e, _ in self.buckets]
            for w in works:
                w.wait()

    def train_step(self):
        """forward_backward + optimizer_step with nothing in between."""
        self.forward_backward()
        self.optimizer_step()

    def optimizer_step(self):
        # skip on non-finite (all-reduced) gradients: every rank sees the same reduced
        # gradient, so all ranks skip together (a rank-local loss check would not)
        if self.cfg.nan_policy != "raise" and not (
                np.isfinite(self._loss_sum) if self.world == 1
                else bool(torch.isfinite(self.params.grad).all())):
            self.nan_skipped += 1
            self.opt.rate = self.opt.rate * (1.0 - getattr(self.opt, "rate_decay", 0.0))
            return
        with torch.no_grad():
            self.opt.step(self.params, self.params.grad)

    @torch.no_grad()
    def evaluate(self, n: Optional[int] = None):
        x, y = self._x, self._y
        if n is not None:
            x, y = x[:n], y[:n]
        logp = self._forward(x)
        self._eval = (float(F.nll_loss(logp, y, reduction="sum")),
                      int((logp.argmax(1) == y).sum()))
        self._last = "eval"
        return logp

    def loss_sum(self) -> float:
        return self._eval[0] if self._last == "eval" else self._loss_sum

    def correct(self) -> int:
        return self._eval[1] if self._last == "eval" else self._correct

    def bad_steps(self) -> int:
        """Updates skipped for a non-finite loss / gradient so far."""
        return self.nan_skipped

    def gradient_tagged(self) -> bool:
        """(HIP only: the gradient producers' range-check tag; the fp32 oracle has none)"""
        return False

    def flat_params(self) -> torch.Tensor:
        return self.params.detach()

    def load_params(self, flat: torch.Tensor):
        with torch.no_grad():
            self.params.copy_(flat.float())

    def state_dict(self):
        return {"optimizer": self.opt.state_dict()}

    def load_state_dict(self, d):
        self.opt.load_state_dict(d["optimizer"])


class HIPBackend:
    def __init__(self, cfg: ExperimentConfig, batch: int, flat: Optional[torch.Tensor] = None,
                 world: int = 1, device=None, use_graphs: bool = True, bucket_mb: float = 4.0,
                 grad_dtype: str = "fp32", comm: str = "auto"):
        from ..models.hip_model import HipGoNet, SegmentedStep
        self.cfg = cfg
        self.B = batch
        self.world = world
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.net = HipGoNet(cfg, batch, device=self.device, flat_params=flat,
                            global_batch=batch * world,
                            grad_wire=grad_dtype if world > 1 else "fp32")
        self.layout = self.net.layout
        if world > 1 and flat is None:
            dp.broadcast_(self.net.params, 0)
            self.net.refresh_weights()
        self.bucketer = None
        self.comm = None
        if world > 1:
            # RCCL needs one GPU per rank: a gloo process group (e.g. several ranks sharing
            # one GPU in tests) keeps torch.distributed collectives
            kind = comm if torch.distributed.get_backend() == "nccl" else "torch"
            self.comm = dp.make_communicator(kind, self.device)
            ranges = [self.layout.layer_range(i) for i in range(len(self.layout.layers))]
            self.bucketer = dp.GradBucketer(self.net.grads,
                                            dp.make_buckets(ranges, int(bucket_mb * 2 ** 20),
                                                            groups=self.net.wgroups),
                                            grad_dtype=grad_dtype, comm=self.comm,
                                            shadow=self.net.grads16)
        # the loader's pinned slots are copied on a load stream beside the previous step
        # (HipGoNet.enable_prefetch; +1.1% with host batches, DG_PREFETCH=0: off)
        if os.environ.get("DG_PREFETCH", "auto") != "0":
            self.net.enable_prefetch()
        self._step = SegmentedStep(self.net, self.bucketer, use_graphs=use_graphs)
        self._eval_n = batch
        self._last = "train"

    @property
    def rate(self) -> float:
        return float(self.net.lr.item())

    @property
    def params(self):
        return self.net.params

    def load_next(self, loader):
        """Next training batch straight from the loader's pinned packed slot into the
        network's input buffer: one async H2D copy, ordered before the step on the same
        stream.  Returns None (the host copy is gone; ``current_batch`` reads it back)."""
        self.net.set_batch_packed_from(loader)
        return None

    def current_batch(self):
        from ..data.batch import unpack_views
        pl, py_, rk, lb = unpack_views(self.net.inbuf.cpu(), self.B)
        return (pl.numpy().reshape(self.B, 9, 19, 19), py_.numpy(), rk.numpy(), lb.numpy())

    def set_batch(self, planes, player, rank, labels):
        dev = self.device
        t = lambda a, dt: (a if isinstance(a, torch.Tensor) else torch.from_numpy(np.asarray(a)))
        self.net.set_batch(t(planes, None).to(dev), t(player, None).to(dev),
                           t(rank, None).to(dev), t(labels, None).to(dev, torch.int32))

    def forward_backward(self):
        self._step.forward_backward()
        self._last = "train"

    def train_step(self):
        """forward_backward + optimizer_step with nothing in between: without DP buckets
        SegmentedStep replays both as ONE hipGraph (no graph boundary before the update)."""
        self._step()
        self._last = "train"

    def optimizer_step(self):
        self._step.optimizer()

    def evaluate(self, n: Optional[int] = None):
        self._eval_n = n or self.B
        self.net.evaluate()
        self._last = "eval"

    def loss_sum(self) -> float:
        if self._last == "eval":
            return float(self.net.eval_loss[:self._eval_n].sum().item())
        return float(self.net.loss.sum().item())

    def correct(self) -> int:
        if self._last == "eval":
            n = self._eval_n
            return int((self.net.eval_pred[:n] == self.net.labels[:n]).sum().item())
        return int((self.net.pred == self.net.labels).sum().item())

    def bad_steps(self) -> int:
        """Updates the device gate / fused update skipped so far (syncs)."""
        return int(self.net.bad_steps.item())

    def gradient_tagged(self) -> bool:
        """Whether a gradient producer tagged the step in flight (before its update: a value
        out of range — dg_common.h grad_out_of_range; the update would skip it).  Syncs.
        Single-GPU only: under DP the tag is rank-local and the all-reduced gradient's finite
        gate decides, the same on every rank."""
        if self.world > 1:
            return False
        step, tag = self.net._stepflag.tolist()
        return tag == step + 1

    def flat_params(self) -> torch.Tensor:
        return self.net.params.detach().cpu()

    def load_params(self, flat: torch.Tensor):
        self.net.load_params(flat)

    def state_dict(self):
        d = {"optimizer": {"kind": self.cfg.optimizer, "rate": self.rate,
                           "rate_decay": self.cfg.rateDecay}}
        if self.net.ms is not None:
            d["optimizer"]["ms"] = self.net.ms.detach().cpu()
        return d

    def close(self):
        if self.comm is not None:
            torch.cuda.synchronize(self.device)
            self.comm.close()
            self.comm = None

    def load_state_dict(self, d):
        o = d["optimizer"]
        self.net.lr.fill_(float(o["rate"]))
        if "ms" in o and self.net.ms is not None:
            self.net.ms.copy_(o["ms"].to(self.net.ms.device))
