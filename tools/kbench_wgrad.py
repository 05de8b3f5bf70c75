"""Micro-benchmark + ablations of the weight-gradient kernels for one hidden 128->128 3x3
layer at B=256: 128x128 im2col tiles vs three-slice 128x384 tiles (t3), plus the slab
reduce.  Ablation bits (conv_wgrad_set_ablate): 1 no MFMA, 2 no LDS fragment reads,
4 no LDS-DMA, 8 no slab store.  Prints one JSON object (us per launch)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops import layouts as LY  # noqa: E402
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    h = hip()
    B, C = 256, 128
    dev = "cuda"
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    dz = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(dz, 1).copy_(torch.randn(B, 19, 19, C, device=dev))
    _, KPw, _ = LY.conv_dims(3, C, C, 128)
    s = stream_handle()
    flops = 2.0 * C * C * 9 * 361 * B
    res = {}
    cfg = {}
    for t3 in (1,):     # (the three-slice kernel is the only one for K = 9 x 128)
        kt = h.conv_wgrad_ktile(KPw)
        splits = LY.pick_wgrad_splits(B * 361, KPw, 128, wgs_per_cu=h.conv_wgrad_wgs_per_cu_for(KPw),
                                      ktile=kt)
        cfg[f"t3={t3}"] = {"ktile": kt, "splits": splits}
        slab = torch.empty(splits * 128 * KPw, device=dev)
        gw = torch.empty(C * 9 * C, device=dev)

        def wg():
            h.conv_wgrad(3, dz.data_ptr(), 1, C, 128, x.data_ptr(), 1, C, B, KPw, splits,
                         slab.data_ptr(), s)

        def red():
            h.wgrad_reduce(slab.data_ptr(), gw.data_ptr(), splits, C, 128, KPw, 9, C, C, 0, 0,
                           0, 0, 0, s)
        for rnd in range(2):
            for mode in (0, 1, 2, 4, 8, 3, 6, 12, 14, 15):
                h.conv_wgrad_set_ablate(mode)
                res.setdefault(f"t3={t3}_abl{mode}", []).append(round(timeit(wg), 2))
            h.conv_wgrad_set_ablate(0)
            res.setdefault(f"t3={t3}_reduce", []).append(round(timeit(red), 2))
    out = {k: {"us": v, "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)} for k, v in res.items()}
    out["config"] = cfg
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
