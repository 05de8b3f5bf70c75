"""Micro-benchmark + ablations of the sliding-window weight gradient (conv_wgrad_win.hip)
against the grouped three-slice kernel (conv_wgrad_multi) for NL hidden 3x3 layers at
B=256.  Ablation bits (conv_wgrad_win_set_ablate): 1 no MFMA, 2 no LDS fragment reads,
4 no LDS-DMA (ablations at prefetch distance 2); full kernel at distance 1..4.  Prints one JSON object (us per launch).  Usage: kbench_win.py [C] [NL]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops import layouts as LY  # noqa: E402
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    h = hip()
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    NL = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    B = 256
    dev = "cuda"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    xs, dzs = [], []
    for _ in range(NL):
        x = LY.alloc_frame(B, C, 1, dev)
        LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
        dz = LY.alloc_frame(B, C, 1, dev)
        LY.frame_interior(dz, 1).copy_(torch.randn(B, 19, 19, C, device=dev))
        xs.append(x)
        dzs.append(dz)
    _, KPw, _ = LY.conv_dims(3, C, C, 128)
    s = stream_handle()
    flops = 2.0 * C * C * 9 * 361 * B * NL
    res, cfg = {}, {}
    Sw = h.conv_wgrad_win_splits(NL, C, C, B, ncu)
    slab_w = torch.empty(NL * 2 * Sw * C * KPw, device=dev)
    per = Sw * C * KPw
    tw = np.array([[dzs[i].data_ptr(), xs[i].data_ptr(), slab_w.data_ptr() + 4 * i * per]
                   for i in range(NL)], dtype=np.int64)
    tiles = (KPw // 384) * (C // 128) * NL
    St = max(1, min((ncu * h.conv_wgrad_wgs_per_cu_for(KPw)) // tiles, B * 361 // 256))
    slab_t = torch.empty(NL * St * C * KPw, device=dev)
    per_t = St * C * KPw
    tt = np.array([[dzs[i].data_ptr(), xs[i].data_ptr(), slab_t.data_ptr() + 4 * i * per_t]
                   for i in range(NL)], dtype=np.int64)
    cfg = {"C": C, "NL": NL, "win_splits": Sw, "t3_splits": St}

    def win():
        h.conv_wgrad_win(tw.ctypes.data, NL, C, C, C, B, KPw, Sw, 0, s)

    def t3():
        h.conv_wgrad_multi(3, tt.ctypes.data, NL, 1, C, C, 1, C, B, KPw, St, s)
    for rnd in range(2):
        for mode in (1, 2, 4, 3, 5, 6, 7):
            h.conv_wgrad_win_set_ablate(mode)
            res.setdefault(f"win_nw4_abl{mode}", []).append(round(timeit(win), 2))
        h.conv_wgrad_win_set_ablate(0)
        res.setdefault(f"win_S{Sw}", []).append(round(timeit(win), 2))
        res.setdefault("t3_multi", []).append(round(timeit(t3), 2))
    out = {k: {"us": v, "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)} for k, v in res.items()}
    out["config"] = cfg
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
