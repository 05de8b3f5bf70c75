"""GoCNN parameter layout, initialisation and the fp32 PyTorch oracle model.

Architecture parity with ``getBasicModel`` (``experiments.lua:133-153``): for each layer
``ZeroPad((k-1)/2) -> Conv(k x k, per-channel bias) -> untied per-position bias
(nn.Add(c*361)) -> ReLU``; the head (c_out = 1) also ends in ReLU before
``Reshape(361) -> LogSoftMax`` (VERIFIED in ``Run Experiment.ipynb:61-67``).

MI355X-first storage (not the reference's layout):

* All parameters live in ONE flat fp32 master buffer (the analogue of
  ``model:getParameters()`` at ``experiments.lua:107``); gradients in a second flat
  buffer with the same layout, so DP buckets are plain views.
* Conv weights are stored OHWI ``[c_out][kh][kw][c_in]`` (channels innermost, the
  layout the implicit-GEMM MFMA kernels consume); per-position bias is stored
  ``[361][c_out]`` so the conv epilogue reads it contiguously per pixel.
  ``to_reference_layout`` converts to the reference ``SpatialConvolutionMM`` layout
  ``weight[c_out][c_in*kh*kw]`` and ``nn.Add`` layout ``bias[c*361]`` (c, h, w order).
* Every tensor starts on a 64-element (256 B) boundary so vectorised device loads never
  straddle tensors.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

from ..config import BOARD, NUM_POINTS, ExperimentConfig

ALIGN = 64


def _align(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


@dataclass(frozen=True)
class LayerSpec:
    index: int          # 0-based layer index
    cin: int
    cout: int
    k: int
    w_off: int          # offsets (elements) into the flat buffer
    b_off: int
    pos_off: int

    @property
    def pad(self) -> int:
        return (self.k - 1) // 2

    @property
    def w_numel(self) -> int:
        return self.cout * self.k * self.k * self.cin

    @property
    def is_head(self) -> bool:
        return self.cout == 1


class ParamLayout:
    """Offsets of every parameter tensor inside the flat master buffer."""

    def __init__(self, cfg: ExperimentConfig):
        self.cfg = cfg
        self.layers: List[LayerSpec] = []
        off = 0
        for i, (cin, cout, k) in enumerate(cfg.layer_specs()):
            w_off = off
            off = _align(off + cout * k * k * cin)
            b_off = off
            off = _align(off + cout)
            pos_off = off
            off = _align(off + NUM_POINTS * cout)
            self.layers.append(LayerSpec(i, cin, cout, k, w_off, b_off, pos_off))
        self.numel = off
        self.num_params = cfg.num_params()

    # views into a flat buffer -------------------------------------------------
    def weight(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        L = self.layers[i]
        return flat[L.w_off:L.w_off + L.w_numel].view(L.cout, L.k, L.k, L.cin)

    def bias(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        L = self.layers[i]
        return flat[L.b_off:L.b_off + L.cout]

    def pos_bias(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        L = self.layers[i]
        return flat[L.pos_off:L.pos_off + NUM_POINTS * L.cout].view(NUM_POINTS, L.cout)

    def named_views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for L in self.layers:
            n = L.index + 1
            out[f"conv{n}.weight"] = self.weight(flat, L.index)
            out[f"conv{n}.bias"] = self.bias(flat, L.index)
            out[f"pos_bias{n}"] = self.pos_bias(flat, L.index)
        return out

    def tensor_ranges(self) -> List[Tuple[str, int, int]]:
        """(name, offset, numel) in flat order; used for DP bucketing."""
        out = []
        for L in self.layers:
            n = L.index + 1
            out.append((f"conv{n}.weight", L.w_off, L.w_numel))
            out.append((f"conv{n}.bias", L.b_off, L.cout))
            out.append((f"pos_bias{n}", L.pos_off, NUM_POINTS * L.cout))
        return out

    def layer_range(self, i: int) -> Tuple[int, int]:
        """[start, end) of layer i's parameters in the flat buffer (aligned)."""
        start = self.layers[i].w_off
        end = self.layers[i + 1].w_off if i + 1 < len(self.layers) else self.numel
        return start, end


def init_params(layout: ParamLayout, seed: int = 0, device="cpu") -> torch.Tensor:
    """Torch7 ``nn`` default init (EXTERNAL behaviour):
    conv W,b ~ U(+-1/sqrt(k*k*c_in)); nn.Add bias ~ U(+-1/sqrt(c*361))."""
    g = torch.Generator().manual_seed(seed)
    flat = torch.zeros(layout.numel, dtype=torch.float32)
    for L in layout.layers:
        s = 1.0 / math.sqrt(L.k * L.k * L.cin)
        w = layout.weight(flat, L.index)
        w.copy_((torch.rand(w.shape, generator=g) * 2 - 1) * s)
        b = layout.bias(flat, L.index)
        b.copy_((torch.rand(b.shape, generator=g) * 2 - 1) * s)
        sp = 1.0 / math.sqrt(L.cout * NUM_POINTS)
        p = layout.pos_bias(flat, L.index)
        p.copy_((torch.rand(p.shape, generator=g) * 2 - 1) * sp)
    return flat.to(device)


def reference_forward(layout: ParamLayout, flat: torch.Tensor, x: torch.Tensor,
                      head_relu: bool = True) -> torch.Tensor:
    """fp32 oracle: x [B,37,19,19] (NCHW) -> log-probs [B,361].

    Uses plain torch conv2d on the CPU as an *oracle only* (SURVEY.md §4.3)."""
    h = x
    n = len(layout.layers)
    for L in layout.layers:
        w = layout.weight(flat, L.index).permute(0, 3, 1, 2)  # OHWI -> OIHW
        h = F.conv2d(h, w, layout.bias(flat, L.index), padding=L.pad)
        pb = layout.pos_bias(flat, L.index).t().reshape(1, L.cout, BOARD, BOARD)
        h = h + pb
        if L.index < n - 1 or head_relu:
            h = F.relu(h)
    logits = h.reshape(h.shape[0], NUM_POINTS)
    return F.log_softmax(logits, dim=1)


def to_reference_layout(layout: ParamLayout, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Export to the Torch7 module layouts: SpatialConvolutionMM weight
    ``[c_out, c_in*k*k]`` row-major over (c_in, kh, kw); nn.Add bias ``[c*361]`` (c,h,w)."""
    out = {}
    flat = flat.detach().float().cpu()
    for L in layout.layers:
        n = L.index + 1
        w = layout.weight(flat, L.index).permute(0, 3, 1, 2).reshape(L.cout, L.cin * L.k * L.k)
        out[f"conv{n}.weight"] = w.contiguous()
        out[f"conv{n}.bias"] = layout.bias(flat, L.index).clone()
        out[f"add{n}.bias"] = layout.pos_bias(flat, L.index).t().reshape(-1).contiguous()
    return out


def from_reference_layout(layout: ParamLayout, tensors: Dict[str, torch.Tensor]) -> torch.Tensor:
    flat = torch.zeros(layout.numel, dtype=torch.float32)
    for L in layout.layers:
        n = L.index + 1
        w = tensors[f"conv{n}.weight"].float().reshape(L.cout, L.cin, L.k, L.k)
        layout.weight(flat, L.index).copy_(w.permute(0, 2, 3, 1))
        layout.bias(flat, L.index).copy_(tensors[f"conv{n}.bias"].float().reshape(-1))
        layout.pos_bias(flat, L.index).copy_(
            tensors[f"add{n}.bias"].float().reshape(L.cout, NUM_POINTS).t())
    return flat
