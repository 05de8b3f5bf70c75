"""Optimizers over the flat parameter vector (CPU path; the GPU path runs the same math in
``sgd_kernel`` / ``rmsprop_kernel``, csrc/kernels/elementwise.hip).

* ``SGD`` (optimizer.lua:16-27): theta -= rate * g, then rate *= (1 - decay) — so after t
  steps rate_t = rate_0 * (1 - decay)^t.  The rate is a Python float (double), as in Lua.
* ``RMSProp`` — the reference's misnamed ``AdagradOptimizer`` (optimizer.lua:1-14):
  ms = decay*ms + (1-decay)*g^2, theta -= rate * g / sqrt(ms), ms initialised to 1.  The
  reference version crashes (undefined global ``grads``); this one works and is opt-in.
"""
from __future__ import annotations

import torch


class SGD:
    def __init__(self, rate: float, rate_decay: float):
        self.rate = float(rate)
        self.rate_decay = float(rate_decay)

    @torch.no_grad()
    def step(self, params: torch.Tensor, grads: torch.Tensor):
        params.add_(grads, alpha=-self.rate)
        self.rate = self.rate * (1.0 - self.rate_decay)

    def state_dict(self):
        return {"kind": "sgd", "rate": self.rate, "rate_decay": self.rate_decay}

    def load_state_dict(self, d):
        self.rate = float(d["rate"])
        self.rate_decay = float(d["rate_decay"])


class RMSProp:
    def __init__(self, rate: float, decay: float, numel: int):
        self.rate = float(rate)
        self.decay = float(decay)
        self.ms = torch.ones(numel, dtype=torch.float32)

    @torch.no_grad()
    def step(self, params: torch.Tensor, grads: torch.Tensor):
        self.ms.mul_(self.decay).addcmul_(grads, grads, value=1.0 - self.decay)
        params.addcdiv_(grads, self.ms.sqrt(), value=-self.rate)

    def state_dict(self):
        return {"kind": "rmsprop", "rate": self.rate, "decay": self.decay, "ms": self.ms}

    def load_state_dict(self, d):
        self.rate = float(d["rate"])
        self.decay = float(d["decay"])
        self.ms = d["ms"].float().clone()
