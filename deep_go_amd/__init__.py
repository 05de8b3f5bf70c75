"""deep_go_amd: an MI355X-native (gfx950 / CDNA4) Go move-prediction CNN trainer.

Same capabilities as the Torch7 project vipmath/deep-go (Clark & Storkey, arXiv
1412.6564 replication), re-designed for AMD Instinct MI355X: PyTorch-ROCm for tensors and
process groups, hand-written HIP/MFMA kernels for every hot op, RCCL over xGMI for data
parallelism, and a C++ runtime for the Go engine, data codec and loader.
"""
import torch  # noqa: F401  (loads the HIP runtime before any native extension)

__version__ = "0.1.0"
