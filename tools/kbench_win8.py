"""Micro-benchmark + timing ablations of the MX-fp8 sliding-window weight gradient
(conv_wgrad_win8.hip) for NL hidden 3x3 layers at B = 256, C = 128 and 256 (the 12x128 /
12x256 fp8 step's launch shapes and split counts).  Ablation bits (conv_wgrad_win8_set_ablate,
wrong results, timing only): 1 no MFMA, 2 no LDS fragment reads, 4 no LDS-DMA, 8 no slab
store, 16 no per-super-step barrier, and sums.  Random e4m3 / e5m2 frames.  Prints one JSON
line (us per launch, min over rounds; MFMA floor = 32 cycles x MFMAs per SIMD).

  python tools/kbench_win8.py [--C 128,256] [--modes 0,1,2,4,8,16,3,6,7,20,31]

(The 128-co workgroup tiles measured in round 5 were removed in round 6.)"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deep_go_amd.ops.native import hip, stream_handle  # noqa: E402
from tools.kbench import timeit  # noqa: E402

FP = 448   # fp8 frame pitch (rows per board)


def bench_c(h, C, NL, B, modes, rounds, s):
    dev = "cuda"
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    g = torch.Generator(device=dev).manual_seed(C)
    dz, xs = [], []
    for _ in range(NL):
        # bytes 0x00..0x77: finite e4m3 / e5m2 values of both signs
        dz.append(torch.randint(0, 0x78, (B * FP * C,), dtype=torch.uint8, device=dev,
                                generator=g))
        xs.append(torch.randint(0, 0x78, (B * FP * C,), dtype=torch.uint8, device=dev,
                                generator=g))
    KP = 9 * C
    splits = h.conv_wgrad_win8_splits(NL, C, C, B, ncu)
    per = splits * C * KP
    slab = torch.empty(NL * per, device=dev)
    sc = torch.full((2,), 2.0 ** -8, device=dev)
    tab = np.array([[dz[i].data_ptr(), xs[i].data_ptr(), slab.data_ptr() + 4 * i * per,
                     sc.data_ptr(), sc.data_ptr() + 4] for i in range(NL)], dtype=np.int64)

    def run(mode):
        def f():
            h.conv_wgrad_win8_set_ablate(mode)
            h.conv_wgrad_win8(tab.ctypes.data, NL, C, C, C, B, KP, splits, 0, s)
        return f
    times = {}
    for _ in range(rounds):
        for m in modes:
            times.setdefault(f"mode{m}", []).append(timeit(run(m)))
    h.conv_wgrad_win8_set_ablate(0)
    # MFMAs per SIMD: NL x (C/64)^2 workgroups' worth of 64x64 tiles x 9 taps x K = B*13*32 rows
    # / 128 per MFMA x 16 (16x16 fragments of a 64x64 tile) spread over ncu*4 SIMDs
    n_mfma = NL * (C // 64) ** 2 * 9 * 16 * (B * 13 * 32 // 128)
    floor_cyc = n_mfma * 32 / (ncu * 4)
    return {"splits": splits, "mfma_floor_cycles_per_simd": round(floor_cyc),
            "us": {k: round(min(v), 1) for k, v in times.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", default="128,256")
    ap.add_argument("--layers", type=int, default=10)
    ap.add_argument("--boards", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--modes", default="0,1,2,4,8,16,3,6,7,20,31")
    a = ap.parse_args()
    h = hip()
    s = stream_handle()
    modes = [int(m) for m in a.modes.split(",")]
    out = {"boards": a.boards, "layers": a.layers}
    for C in [int(c) for c in a.C.split(",")]:
        out[f"C{C}"] = bench_c(h, C, a.layers, a.boards, modes, a.rounds, s)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
