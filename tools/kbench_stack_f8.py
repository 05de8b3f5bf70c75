"""Micro-benchmark + timing ablations of the fp8 board-resident layer stack (conv_stack_f8.hip):
10 hidden C -> C 3x3 layers of 256 boards (C = 128 and 256), forward (e4m3) and backward-data
(e5m2).  Ablation modes (wrong results, timing only) of the production
variants (fp8 copies, no bf16 frames but the last; backward-data with stochastic rounding):
2 = no A loads, 4 = no copy-out,
64 = no epilogue, 128 = no B reads, and their sums.  Also 1- and 2-layer launches (the fixed
prologue / per-layer cost).  Pure-MFMA floor per layer: 1728 (C = 128) | 6912 (C = 256)
16x16x128 MX-MFMAs of 32 cycles per board over 4 SIMDs.  Random data; prints one JSON line.

  python tools/kbench_stack_f8.py [--modes 0,2,4,64,128,68,196,198] [--C 128,256]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops import layouts as LY  # noqa: E402
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def bench_c(h, C, modes, dmodes, B, NL, s):
    dev = "cuda"
    torch.manual_seed(0)
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    ys = [LY.alloc_frame(B, C, 1, dev) for _ in range(NL)]
    ms = [torch.randint(0, 255, (B, 361, C // 8), dtype=torch.uint8, device=dev) for _ in range(NL)]
    pbs = [(0.01 * torch.randn(24 * 2 * 4 * 64 * 4 * (C // 128), device=dev)).to(torch.bfloat16)
           for _ in range(NL)]
    w8 = [LY.stack_frag_f8(torch.randint(0, 0x78, (C, 9, C), dtype=torch.uint8, device=dev))
          for _ in range(NL)]
    sc = torch.full((NL + 1,), 2.0 ** -6, device=dev)
    amax = torch.zeros(NL + 1, dtype=torch.int32, device=dev)
    t8 = np.array([[w8[i].data_ptr(), pbs[i].data_ptr(), ys[i].data_ptr(), ms[i].data_ptr(),
                    sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * (i + 1),
                    amax.data_ptr() + 4 * (i + 1)] for i in range(NL)], dtype=np.int64)
    # the production launches: fp8 copies of every non-last layer's output (the MX-fp8 weight
    # gradients' operands), no bf16 frame but the last layer's; backward-data with SR
    t8[:-1, 2] = 0
    t8d = t8.copy()
    t8d[:, 1] = 0
    x8 = [torch.zeros(B * 448 * C, dtype=torch.uint8, device=dev) for _ in range(NL)]
    sr = torch.full((1,), 5, dtype=torch.int64, device=dev)

    def y8tab(nl):
        return np.array([x8[0].data_ptr()] + [x8[i + 1].data_ptr() if i + 1 < nl else 0
                                              for i in range(nl)], dtype=np.int64)
    y8s = {nl: y8tab(nl) for nl in (1, 2, NL)}

    def run(mode=0, nl=NL, epi=None):
        tt = t8.copy() if epi is None else t8d.copy()
        tt[nl - 1, 2] = ys[nl - 1].data_ptr()
        tt = np.ascontiguousarray(tt[:nl])
        y8 = y8s[nl]

        def f():
            h.conv_stack_f8_set_mode(mode)
            if epi is None:
                h.conv_stack_f8_y8(C, h.EPI_FWD, tt.ctypes.data, nl, x.data_ptr(), sc.data_ptr(),
                                   amax.data_ptr(), B, y8.ctypes.data, s)
            else:
                h.conv_stack_f8_dgrad(C, tt.ctypes.data, nl, x.data_ptr(), sc.data_ptr(),
                                      amax.data_ptr(), B, y8.ctypes.data, sr.data_ptr(), s)
        f.keep = (tt, y8)
        return f
    times = {}
    for _ in range(3):
        for m in modes:
            times.setdefault(f"fwd_mode{m}", []).append(timeit(run(m)))
        for m in dmodes:
            times.setdefault(f"dgrad_mode{m}", []).append(timeit(run(m, epi=h.EPI_DGRAD)))
        times.setdefault("fwd_1layer", []).append(timeit(run(nl=1)))
        times.setdefault("fwd_2layers", []).append(timeit(run(nl=2)))
    h.conv_stack_f8_set_mode(0)
    mfma_per_board = 1728 * (C // 128) ** 2
    out = {}
    for k, v in times.items():
        t = min(v)
        nl = 1 if k.endswith("1layer") else 2 if k.endswith("2layers") else NL
        out[k] = {"us": round(t, 1), "us_per_layer": round(t / nl, 2),
                  # per-SIMD MFMA cycles per layer / wall cycles per layer at the clock implied
                  "mfma_cycles_per_layer": mfma_per_board * 32 // 4}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="0,2,4,64,128,68,196,198")
    ap.add_argument("--dmodes", default="0,2,4,64,68,198")
    ap.add_argument("--C", default="128,256")
    ap.add_argument("--boards", type=int, default=256)
    a = ap.parse_args()
    h = hip()
    s = stream_handle()
    modes = [int(m) for m in a.modes.split(",")]
    res = {"boards": a.boards, "layers": 10}
    for C in [int(c) for c in a.C.split(",")]:
        res[f"C{C}"] = bench_c(h, C, modes, [int(m) for m in a.dmodes.split(",")], a.boards,
                               10, s)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
