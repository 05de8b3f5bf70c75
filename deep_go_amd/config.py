"""Experiment configuration: a frozen dataclass plus named presets.

Parity notes (reference = Torch7 ``vipmath/deep-go``):

* Field names mirror the reference's prototype tables so configs read the same:
  ``numLayers, channelSize, kernels, channels, batchSize, rate, rateDecay,
  validationSize, validation_interval, numGPUs, data_root, directories``
  (``experiments.lua:8-17``, ``experiments.lua:33-46``).
* The reference builds ``kernels``/``channels`` by *appending* to tables shared with
  the prototype (``experiments.lua:88-94``), which silently corrupts later
  experiments.  Here the layer schedule is derived, never mutated.
* Unknown override keys are rejected (the reference silently ignored the typo
  ``validation_size`` in ``localtest.lua:8``).
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, Tuple

BOARD = 19
NUM_POINTS = BOARD * BOARD  # 361
# Network input planes (dataloader.lua:6-14): STONE=1, LIBERTIES=4, LIBERTIES_AFTER=8,
# KILL=15, AGE=22, LADDER=27, RANK=28, TOTAL=37 (plane 28 is always zero).
NUM_INPUT_PLANES = 37
# + the optional simple-ko plane (ExperimentConfig.ko_plane; data/features.py)
NUM_INPUT_PLANES_KO = 38
# Stored uint8 planes per position (dataloader.lua:20-27).
NUM_STORED_PLANES = 9


@dataclass(frozen=True)
class ExperimentConfig:
    # -- reference fields (experiments.lua:8-46) --
    name: str = "basicGoExperiment"
    numLayers: int = 3
    channelSize: int = 64
    first_kernel: int = 5          # kernels = {5, 3, 3, ...}
    hidden_kernel: int = 3
    head_kernel: int = 3           # reference: 3x3 head (experiments.lua:88-94)
    batchSize: int = 32
    rate: float = 0.01
    rateDecay: float = 1e-7
    validationSize: int = 2000
    validation_interval: int = 2000
    useCuda: bool = False
    numGPUs: int = 1
    data_root: str = "data"
    directories: Tuple[Tuple[str, str], ...] = (
        ("train", "train"), ("validation", "validation"), ("test", "test"))
    # -- additions --
    dtype: str = "bf16"            # GPU compute dtype: bf16 | fp8 ; CPU path is fp32
    seed: int = 1234
    synthetic: bool = False        # synthetic boards instead of the on-disk dataset
    head_relu: bool = True         # reference applies ReLU to the head (parity)
    optimizer: str = "sgd"         # sgd | rmsprop (the reference's misnamed AdagradOptimizer)
    rmsprop_decay: float = 0.9
    bucket_mb: float = 6.0         # DP gradient bucket size (12x128: head + hidden layers | layer 0)
    # DP all-reduce dtype: fp32 (the reference's DataParallelTable reduces fp32 gradients,
    # experiments.lua:155-168) | bf16 (opt-in: the wire twin every gradient pass 2 writes; half
    # the xGMI bytes; tests/test_wire_cpu.py and tests/test_train_gpu.py bound it against fp32)
    grad_dtype: str = "fp32"
    # DP gradient collectives in the trainer: auto (the native in-graph RCCL communicator when
    # every rank's set-up and in-graph self-test pass, else torch — a collective decision,
    # parallel/dp.py make_communicator; what bench.py measures) | native | torch
    # (torch.distributed's process group between graph segments)
    comm: str = "auto"
    reference_validation_quirks: bool = False  # train.lua:23-44 floor/off-by-one
    sampling: str = "game"         # game (reference, data.lua:29-37) | position
    loader_threads: int = 8
    prefetch: int = 4
    checkpoint_dir: str = "."
    metrics_path: Optional[str] = None
    # non-finite loss / gradient: guard (default: the device gate skips the update, the host
    # checks at log intervals and raises — dumping the batch — after nan_max_skips
    # consecutive skipped steps; the training step stays one fused graph) | skip (never
    # raises) | raise (host check every step, unfused; the reference's pcall dump)
    nan_policy: str = "guard"
    nan_max_skips: int = 10
    log_interval: int = 10         # train.lua:119
    # optional 38th input plane: the simple-ko point (needs data made with makedata --ko;
    # off = the reference's 37-plane layout)
    ko_plane: bool = False
    id: Optional[str] = None

    # ---- derived layer schedule ----
    @property
    def kernels(self) -> List[int]:
        return [self.first_kernel] + [self.hidden_kernel] * (self.numLayers - 2) + (
            [self.head_kernel] if self.numLayers >= 2 else [])

    @property
    def input_planes(self) -> int:
        return NUM_INPUT_PLANES_KO if self.ko_plane else NUM_INPUT_PLANES

    @property
    def channels(self) -> List[int]:
        return [self.input_planes] + [self.channelSize] * (self.numLayers - 1) + [1]

    def layer_specs(self) -> List[Tuple[int, int, int]]:
        """(c_in, c_out, kernel) per layer; layer 1 sees the 37 (38) input planes."""
        if self.numLayers == 1:
            return [(self.input_planes, 1, self.first_kernel)]
        ch, ks = self.channels, self.kernels
        return [(ch[i], ch[i + 1], ks[i]) for i in range(self.numLayers)]

    def num_params(self) -> int:
        n = 0
        for cin, cout, k in self.layer_specs():
            n += cout * cin * k * k + cout + cout * NUM_POINTS
        return n

    def train_flops_per_board(self) -> float:
        """Useful training FLOPs per board: 2*MACs over 361 output points per layer for the
        forward, the weight gradient and the input gradient — except the FIRST layer's input
        gradient, which nothing needs and the step never computes (BASELINE.md's "train ~=
        3x forward" counted it: +2.5% at 12x128, +1.3% at 12x256).  Real channel counts (37
        input planes, not the 40 the kernels pad to)."""
        f = 0.0
        for i, (cin, cout, k) in enumerate(self.layer_specs()):
            fwd = 2.0 * cout * cin * k * k * NUM_POINTS
            f += fwd * (2.0 if i == 0 else 3.0)
        return f

    def replace(self, **kw) -> "ExperimentConfig":
        return override(self, kw)

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["directories"] = [list(x) for x in self.directories]
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "ExperimentConfig":
        d = dict(d)
        if "directories" in d:
            d["directories"] = tuple(tuple(x) for x in d["directories"])
        return override(ExperimentConfig(), d)

    def directory(self, split: str) -> str:
        return dict(self.directories)[split]


_FIELD_TYPES = {f.name: f.type for f in fields(ExperimentConfig)}


def _coerce(name: str, value: Any, current: Any) -> Any:
    if isinstance(value, str) and not isinstance(current, str):
        if isinstance(current, bool):
            lv = value.lower()
            if lv in ("1", "true", "yes", "on"):
                return True
            if lv in ("0", "false", "no", "off"):
                return False
            raise ValueError(f"bad bool for {name}: {value}")
        if isinstance(current, int):
            return int(value)
        if isinstance(current, float):
            return float(value)
        if current is None:
            try:
                return json.loads(value)
            except json.JSONDecodeError:
                return value
        if isinstance(current, tuple):
            return tuple(tuple(x) for x in json.loads(value))
    if isinstance(current, float) and isinstance(value, int) and not isinstance(value, bool):
        return float(value)
    return value


_CHOICES = {"nan_policy": ("guard", "skip", "raise"), "comm": ("auto", "native", "torch"),
            "optimizer": ("sgd", "rmsprop"), "grad_dtype": ("fp32", "bf16"),
            "sampling": ("game", "position")}


def override(cfg: ExperimentConfig, kw: Dict[str, Any]) -> ExperimentConfig:
    """Return a copy with overrides; unknown keys raise (fixes localtest.lua:8 typo class)."""
    unknown = [k for k in kw if k not in _FIELD_TYPES]
    if unknown:
        raise KeyError(f"unknown config key(s): {unknown}; valid: {sorted(_FIELD_TYPES)}")
    vals = {k: _coerce(k, v, getattr(cfg, k)) for k, v in kw.items()}
    for k, v in vals.items():
        if k in _CHOICES and v not in _CHOICES[k]:
            raise ValueError(f"{k}={v!r}: expected one of {_CHOICES[k]}")
    return dataclasses.replace(cfg, **vals)


def parse_overrides(items: List[str]) -> Dict[str, Any]:
    out = {}
    for it in items:
        if "=" not in it:
            raise ValueError(f"override must be key=value, got {it!r}")
        k, v = it.split("=", 1)
        out[k.strip()] = v.strip()
    return out


# ---------------------------------------------------------------- presets
PRESETS: Dict[str, ExperimentConfig] = {}


def _preset(name: str, **kw) -> None:
    PRESETS[name] = override(ExperimentConfig(), dict(name=name, **kw))


# experiments.lua:33-46
_preset("basicGoExperiment", numLayers=3, channelSize=64, rate=0.01, rateDecay=1e-7, batchSize=32)
# localtest.lua:4-10 (validation_size typo has no effect -> validationSize stays 2000)
_preset("localtest", numLayers=3, channelSize=64, batchSize=2, validation_interval=20,
        data_root="data", useCuda=False)
# default-experiment.lua:8-29
_preset("default-experiment", numLayers=6, channelSize=64, batchSize=64, rate=0.512,
        rateDecay=1e-7, validationSize=1000, validation_interval=20, useCuda=True)
# notebook cell 1 (Run Experiment.ipynb:10-33)
_preset("notebook", numLayers=3, channelSize=64, batchSize=64, validationSize=200, useCuda=True)
# BASELINE.json configs
# "1-layer 19x19 conv k=16, batch=16 on CPU": ONE 5x5 conv layer of 16 filters (37 -> 16,
# + bias + ReLU) under the 3x3 output head (16 -> 1, log-softmax) — numLayers counts the head
# (experiments.lua:133-153), so a single conv of 16 filters is numLayers=2 (numLayers=1 would
# be the bare 37 -> 1 head, where channelSize has no effect)
_preset("cpu-1layer-k16", numLayers=2, first_kernel=5, channelSize=16, batchSize=16,
        useCuda=False, synthetic=True)
_preset("12x128-bf16", numLayers=12, channelSize=128, batchSize=256, useCuda=True,
        synthetic=True, dtype="bf16")
# (batchSize is the global batch: 2048 over 8 ranks = 256 boards per GPU)
_preset("12x256-dp8", numLayers=12, channelSize=256, batchSize=2048, useCuda=True,
        numGPUs=8, synthetic=True, dtype="bf16")
_preset("full36-d256-dp8", numLayers=12, channelSize=256, batchSize=2048, useCuda=True,
        numGPUs=8, synthetic=False, dtype="bf16")
_preset("fp8-d256-dp8", numLayers=12, channelSize=256, batchSize=2048, useCuda=True,
        numGPUs=8, synthetic=True, dtype="fp8")


def get_preset(name: str, **kw) -> ExperimentConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; have {sorted(PRESETS)}")
    return override(PRESETS[name], kw)
