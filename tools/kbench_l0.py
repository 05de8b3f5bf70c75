"""Micro-benchmark + ablations of the first layer's 5x5 weight gradient (conv_wgrad_kernel<5>:
128 co x 128 k tiles, K = 25 taps x 40 staged channels -> 1024, split-K over pixels) alone on
the GPU, at the plan's split count and a few others.  Ablation bits (conv_wgrad_set_ablate):
1 no MFMA, 2 no LDS fragment reads, 4 no LDS-DMA, 8 no slab store, 16 no K-step barrier.
Usage: python tools/kbench_l0.py [C=128] [B=256].  Prints one JSON object (us per launch)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops import layouts as LY  # noqa: E402
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
    h = hip()
    dev = "cuda"
    CIN = 40                                   # 37 planes staged as 40 channels, pad 2
    x = LY.alloc_frame(B, CIN, 2, dev)
    LY.frame_interior(x, 2).copy_(torch.rand(B, 19, 19, CIN, device=dev).round())
    dz = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(dz, 1).copy_(torch.randn(B, 19, 19, C, device=dev))
    _, KPw, Mpad = LY.conv_dims(5, CIN, C, 128)
    s = stream_handle()
    flops = 2.0 * C * 25 * CIN * 361 * B
    plan = LY.pick_wgrad_splits(B * 361, KPw, Mpad, wgs_per_cu=h.conv_wgrad_wgs_per_cu_for(KPw),
                                ktile=h.conv_wgrad_ktile(KPw))
    res = {}
    for splits in sorted({plan, plan // 2, plan * 2}):
        slab = torch.empty(splits * Mpad * KPw, device=dev)

        def wg():
            h.conv_wgrad(5, dz.data_ptr(), 1, C, Mpad, x.data_ptr(), 2, CIN, B, KPw, splits,
                         slab.data_ptr(), s)
        modes = (0, 1, 2, 4, 8, 16, 3, 7, 15) if splits == plan else (0,)
        for rnd in range(2):
            for mode in modes:
                h.conv_wgrad_set_ablate(mode)
                res.setdefault(f"s{splits}_abl{mode}", []).append(round(timeit(wg), 2))
        h.conv_wgrad_set_ablate(0)
    # conv_wgrad_pipe_kernel (32-pixel K-steps, NS LDS-DMA stages) vs conv_wgrad_kernel (ns 0)
    for splits in sorted({plan // 2, plan, plan * 2}):
        slab = torch.empty(splits * Mpad * KPw, device=dev)

        def wgp():
            h.conv_wgrad(5, dz.data_ptr(), 1, C, Mpad, x.data_ptr(), 2, CIN, B, KPw, splits,
                         slab.data_ptr(), s)
        for rnd in range(3):
            for ns in (0, 4):
                h.conv_wgrad5_set_ns(ns)
                res.setdefault(f"pipe_ns{ns}_s{splits}", []).append(round(timeit(wgp), 2))
    h.conv_wgrad5_set_ns(int(os.environ.get("DG_WGRAD5_NS", "4")))
    # the three-slice kernel (128 co x 384 k, dZ staged once per 3 k-tiles) at K padded to
    # 1152 (12.5% more MFMA work, a third less LDS-DMA per k-tile)
    KP3 = 1152
    s3 = LY.pick_wgrad_splits(B * 361, KP3, Mpad, wgs_per_cu=h.conv_wgrad_wgs_per_cu_for(KP3),
                              ktile=h.conv_wgrad_ktile(KP3))
    for splits in sorted({s3, s3 // 2}):
        slab = torch.empty(splits * Mpad * KP3, device=dev)

        def wg3():
            h.conv_wgrad(5, dz.data_ptr(), 1, C, Mpad, x.data_ptr(), 2, CIN, B, KP3, splits,
                         slab.data_ptr(), s)
        for rnd in range(2):
            res.setdefault(f"t3_s{splits}", []).append(round(timeit(wg3), 2))
    out = {k: {"us": v, "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)} for k, v in res.items()}
    out["config"] = {"C": C, "B": B, "KPw": KPw, "plan_splits": plan,
                     "ktile": h.conv_wgrad_ktile(KPw)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
