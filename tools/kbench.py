"""Kernel micro-benchmarks + ablations (run on the GPU box).

Times each hot kernel in isolation with HIP events, interleaving variants in ONE process
(cdna guide rule 24), on random data (rule 25)."""
import argparse
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops import layouts as LY  # noqa: E402
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402


def timeit(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=256)
    ap.add_argument("--C", type=int, default=128)
    a = ap.parse_args()
    h = hip()
    B, C, k = a.B, a.C, 3
    dev = "cuda"
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    y = LY.alloc_frame(B, C, 1, dev)
    w = torch.randn(C, 3, 3, C, device=dev) / (3 * C ** 0.5)
    KP, KPw, Mpad = LY.conv_dims(3, C, C, 128)
    A = LY.fwd_weight(w, C, KP, Mpad)
    bias = torch.zeros(C, device=dev)
    posb = torch.zeros(361, C, device=dev)
    s = stream_handle()
    flops = 2.0 * C * C * 9 * 361 * B
    res = {}

    def board(bm=128, epi=None):
        e = h.EPI_FWD if epi is None else epi
        h.conv_board(e, 3, bm, A.data_ptr(), KP, C, Mpad, x.data_ptr(), 1, C, B,
                     y.data_ptr(), 1, bias.data_ptr(), posb.data_ptr(),
                     x.data_ptr() if e == h.EPI_DGRAD else 0, 1, s)

    def nt(bm, bn):
        def f():
            h.conv_nt(h.EPI_FWD, 3, bm, bn, A.data_ptr(), KP, C, Mpad, x.data_ptr(), 1, C,
                      B * 361, y.data_ptr(), 1, bias.data_ptr(), posb.data_ptr(), 0, 0, s)
        return f

    for rnd in range(2):
        for mode in (0, 8, 14):
            h.conv_board_set_ablate(mode)
            t = timeit(board)
            res.setdefault(f"board_ablate{mode}", []).append(round(t, 2))
        h.conv_board_set_ablate(0)
        for bm in (64, 128):
            for en, e in (("fwd", h.EPI_FWD), ("dgrad", h.EPI_DGRAD)):
                res.setdefault(f"board{bm}_{en}", []).append(
                    round(timeit(lambda: board(bm, e)), 2))
        for mode in (1, 2, 4, 8, 14, 16, 6, 12):
            h.conv_board_set_ablate(mode)
            res.setdefault(f"board64_fwd_ablate{mode}", []).append(round(timeit(lambda: board(64)), 2))
        h.conv_board_set_ablate(0)
        for bm, bn in ((128, 128), (128, 192)):
            res.setdefault(f"nt_{bm}x{bn}", []).append(round(timeit(nt(bm, bn)), 2))
        dz = LY.alloc_frame(B, C, 1, dev)
        LY.frame_interior(dz, 1).copy_(torch.randn(B, 19, 19, C, device=dev))
        splits = LY.pick_wgrad_splits(B * 361, KPw, 128, wgs_per_cu=2)
        slab = torch.empty(splits * 128 * KPw, device=dev)

        def wg():
            h.conv_wgrad(3, dz.data_ptr(), 1, C, 128, x.data_ptr(), 1, C, B, KPw, splits,
                         slab.data_ptr(), s)
        for mode in (0, 4, 6):
            h.conv_wgrad_set_ablate(mode)
            res.setdefault(f"wgrad_ablate{mode}", []).append(round(timeit(wg), 2))
        h.conv_wgrad_set_ablate(0)
        res.setdefault("splits", []).append(splits)
        gw = torch.empty(C * 9 * C, device=dev)

        def red(sp):
            def f():
                h.wgrad_reduce(slab.data_ptr(),
                               gw.data_ptr(), sp, C, 128, KPw, 9, C, C, 0, 0, 0, 0, 0, s)
            return f
        res.setdefault("reduce_im2col_splits", []).append(round(timeit(red(splits)), 2))
    out = {k: {"us": v, "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)} for k, v in res.items()}
    print(json.dumps({"B": B, "C": C, **out}, indent=1))


if __name__ == "__main__":
    main()
