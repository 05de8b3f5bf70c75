"""Experiment checkpoints.

Reference (``experiments.lua:55-72,124-131``): ``save()`` pickles the whole experiment table
to ``<id>.model`` with ``torch.save`` at every validation; ``Experiment:load`` unpickles it and
re-reads the dataset index; ``experiments/repeated.lua`` loads one and resets the optimizer.

Here, one file per experiment id holds the same state (hyper-parameters, ``iterations``,
``validation_costs``, train-cost history, optimizer state incl. the decayed ``rate``, model
weights named per layer) plus what the reference forgot (RNG/sampler cursor so a resumed run
replays the exact data stream).  Format: safetensors (weights + optimizer tensors, nothing
executable) with the JSON metadata in the safetensors header; written atomically
(tmp + rename); only rank 0 writes under DP.

``export_t7`` writes the reference-compatible Torch7 experiment table (nn.Sequential of
SpatialZeroPadding / SpatialConvolutionMM / Reshape / Add / ReLU / LogSoftMax modules with
the reference layouts) so a Torch7 user can ``torch.load`` it; ``import_t7`` reads one back.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch
from safetensors.torch import load_file, save_file

from ..config import ExperimentConfig
from ..models.gocnn import ParamLayout, from_reference_layout, to_reference_layout

FORMAT = "deep_go_amd.checkpoint.v1"


def save_checkpoint(path: str, cfg: ExperimentConfig, flat: torch.Tensor,
                    state: Dict[str, Any], optimizer: Dict[str, Any]) -> str:
    layout = ParamLayout(cfg)
    flat = flat.detach().float().cpu().contiguous()
    tensors = {k: v.clone().contiguous() for k, v in layout.named_views(flat).items()}
    meta_opt = {}
    for k, v in optimizer.items():
        if isinstance(v, torch.Tensor):
            tensors[f"optimizer.{k}"] = v.detach().float().cpu().contiguous()
        else:
            meta_opt[k] = v
    meta = {"format": FORMAT, "config": cfg.to_dict(), "state": state, "optimizer": meta_opt}
    tmp = path + ".tmp"
    save_file(tensors, tmp, metadata={"deep_go_amd": json.dumps(meta)})
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str) -> Tuple[ExperimentConfig, torch.Tensor, Dict, Dict]:
    from safetensors import safe_open
    with safe_open(path, framework="pt") as f:
        meta = json.loads(f.metadata()["deep_go_amd"])
    if meta.get("format") != FORMAT:
        raise ValueError(f"{path}: not a {FORMAT} checkpoint")
    tensors = load_file(path)
    cfg = ExperimentConfig.from_dict(meta["config"])
    layout = ParamLayout(cfg)
    flat = torch.zeros(layout.numel, dtype=torch.float32)
    views = layout.named_views(flat)
    for k, v in views.items():
        v.copy_(tensors[k].reshape(v.shape))
    opt = dict(meta["optimizer"])
    for k, v in tensors.items():
        if k.startswith("optimizer."):
            opt[k[len("optimizer."):]] = v
    return cfg, flat, meta["state"], opt


# ----------------------------------------------------------------------------- Torch7
def _module(cls: str, **fields) -> Dict[str, Any]:
    d = {"__torch_class__": cls, "train": True}
    d.update(fields)
    return d


def export_t7(path: str, cfg: ExperimentConfig, flat: torch.Tensor, state: Dict[str, Any],
              rate: float) -> str:
    """Reference-compatible experiment table (experiments.lua:124-127 / getBasicModel
    :133-153).  Grad buffers are written as zero tensors of the right shape."""
    from ..ops.native import cpu
    layout = ParamLayout(cfg)
    ref = to_reference_layout(layout, flat)
    modules = []
    channels = cfg.channels
    for L in layout.layers:
        n = L.index + 1
        p = L.pad
        modules.append(_module("nn.SpatialZeroPadding", pad_l=float(p), pad_r=float(p),
                               pad_t=float(p), pad_b=float(p)))
        w = ref[f"conv{n}.weight"].numpy()
        b = ref[f"conv{n}.bias"].numpy()
        modules.append(_module("nn.SpatialConvolutionMM", nInputPlane=float(L.cin),
                               nOutputPlane=float(L.cout), kW=float(L.k), kH=float(L.k),
                               dW=1.0, dH=1.0, padW=0.0, padH=0.0, weight=w, bias=b,
                               gradWeight=np.zeros_like(w), gradBias=np.zeros_like(b)))
        d = L.cout * 361
        modules.append(_module("nn.Reshape", size=np.array([d], np.int64), nelement=float(d)))
        ab = ref[f"add{n}.bias"].numpy()
        modules.append(_module("nn.Add", bias=ab, gradBias=np.zeros_like(ab), scalar=False))
        modules.append(_module("nn.Reshape", size=np.array([L.cout, 19, 19], np.int64),
                               nelement=float(d)))
        modules.append(_module("nn.ReLU", threshold=0.0, val=0.0, inplace=False))
    modules.append(_module("nn.Reshape", size=np.array([361], np.int64), nelement=361.0))
    modules.append(_module("nn.LogSoftMax"))
    model = _module("nn.Sequential", modules=modules)
    exp = {
        "name": cfg.name, "numLayers": float(cfg.numLayers), "channelSize": float(cfg.channelSize),
        "kernels": [float(k) for k in cfg.kernels], "strides": [1.0] * cfg.numLayers,
        "channels": [float(c) for c in channels], "batchSize": float(cfg.batchSize),
        "rate": float(cfg.rate), "rateDecay": float(cfg.rateDecay),
        "validationSize": float(cfg.validationSize),
        "validation_interval": float(cfg.validation_interval), "useCuda": bool(cfg.useCuda),
        "numGPUs": float(cfg.numGPUs), "data_root": cfg.data_root,
        "directories": {k: v for k, v in cfg.directories},
        "id": str(state.get("id")), "iterations": float(state.get("iterations", 0)),
        "validation_costs": [float(c) for c in state.get("validation_costs", [])],
        "initialized": True,
        "optimizer": {"rate": float(rate), "rate_decay": float(cfg.rateDecay)},
        "criterion": _module("nn.ClassNLLCriterion", sizeAverage=True),
        "model": model,
    }
    cpu().t7_save(path, exp)
    return path


def import_t7(path: str, cfg: Optional[ExperimentConfig] = None):
    """Read a reference-style experiment table (weights + state) written by export_t7 (or a
    Torch7 checkpoint with the same module structure).  Loader executes nothing."""
    from ..ops.native import cpu
    exp = cpu().t7_load(path)
    if cfg is None:
        cfg = ExperimentConfig(name=str(exp.get("name", "imported")),
                               numLayers=int(exp["numLayers"]),
                               channelSize=int(exp["channelSize"]),
                               batchSize=int(exp["batchSize"]), rate=float(exp["rate"]),
                               rateDecay=float(exp["rateDecay"]))
    mods = exp["model"]["modules"]
    convs = [m for _, m in sorted(mods.items()) if m["__torch_class__"] == "nn.SpatialConvolutionMM"]
    adds = [m for _, m in sorted(mods.items()) if m["__torch_class__"] == "nn.Add"]
    tensors = {}
    for i, (c, a) in enumerate(zip(convs, adds)):
        tensors[f"conv{i + 1}.weight"] = torch.from_numpy(np.asarray(c["weight"]))
        tensors[f"conv{i + 1}.bias"] = torch.from_numpy(np.asarray(c["bias"]))
        tensors[f"add{i + 1}.bias"] = torch.from_numpy(np.asarray(a["bias"]))
    flat = from_reference_layout(ParamLayout(cfg), tensors)
    vc = exp.get("validation_costs", {})
    state = {"id": exp.get("id"), "iterations": int(exp.get("iterations", 0)),
             "validation_costs": [vc[k] for k in sorted(vc)] if isinstance(vc, dict) else vc}
    return cfg, flat, state, float(exp["optimizer"]["rate"])
