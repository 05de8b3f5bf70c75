"""The staggered two-group schedule of the bf16 board-resident stack (conv_stack2.hip STAG) vs
the barrier schedule: 10 hidden 128 -> 128 layers of 256 boards, forward and backward-data.

Checks first that every layer's output frame (and the forward's ReLU bits) is bit-identical
between the schedules, then times (us, HIP events, interleaved rounds): the barrier schedule,
its no-epilogue ablation (MODE 16: the epilogue's cost), and the staggered schedule for each
co-half-0 priority / co-half-1 start delay in --variants.  Prints one JSON line.

  python tools/kbench_stag.py [--variants 1,0,0;1,1,0;1,2,0;1,1,1]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,0,0;1,1,0;1,2,0;1,1,1")
    ap.add_argument("--boards", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    h = hip()
    B, C, NL = a.boards, 128, 10
    dev = "cuda"
    torch.manual_seed(0)
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    KP, _, Mpad = LY.conv_dims(3, C, C, 128)
    ff, fd, ys, ms, pbs = [], [], [], [], []
    for _ in range(NL):
        w = torch.randn(C, 3, 3, C, device=dev) / (3 * C ** 0.5)
        ff.append(LY.stack_frag(LY.fwd_weight(w, C, KP, Mpad)))
        fd.append(LY.stack_frag(LY.dgrad_weight(w, KP, Mpad)))
        ys.append(LY.alloc_frame(B, C, 1, dev))
        ms.append(torch.randint(0, 255, (B, 361, 16), dtype=torch.uint8, device=dev))
        pbs.append((0.01 * torch.randn(24 * 2 * 4 * 64 * 4, device=dev)).to(torch.bfloat16))
    # the backward-data chain gates with its own (fixed) bits, not the forward's
    md = [torch.randint(0, 255, (B, 361, 16), dtype=torch.uint8, device=dev) for _ in range(NL)]
    tf = np.array([[ff[i].data_ptr(), pbs[i].data_ptr(), ys[i].data_ptr(), ms[i].data_ptr()]
                   for i in range(NL)], dtype=np.int64)
    td = np.array([[fd[i].data_ptr(), 0, ys[i].data_ptr(), md[i].data_ptr()]
                   for i in range(NL)], dtype=np.int64)
    s = stream_handle()

    def run(epi, sched, mode=0):
        t = tf if epi == h.EPI_FWD else td

        def f():
            h.conv_stack2_set_mode(mode)
            h.conv_stack2_set_sched(*sched)
            h.conv_stack2(epi, t.ctypes.data, NL, x.data_ptr(), 0, B, s)
        return f

    variants = [tuple(int(v) for v in g.split(",")) for g in a.variants.split(";")]
    out = {"boards": B, "layers": NL}
    # bit-identity of every layer's frame (+ the forward's bits) against the barrier schedule
    ident = {}
    for epi, name in ((h.EPI_FWD, "fwd"), (h.EPI_DGRAD, "dgrad")):
        run(epi, (0, 0, 0))()
        torch.cuda.synchronize()
        ref = [y.clone() for y in ys] + ([m.clone() for m in ms] if name == "fwd" else [])
        for v in variants:
            for y in ys:
                y.zero_()
            run(epi, v)()
            torch.cuda.synchronize()
            got = ys + (ms if name == "fwd" else [])
            ident[f"{name}_{v}"] = all(torch.equal(r, g) for r, g in zip(ref, got))
    out["bit_identical"] = ident
    times = {}
    for _ in range(a.rounds):
        for epi, name in ((h.EPI_FWD, "fwd"), (h.EPI_DGRAD, "dgrad")):
            times.setdefault(f"{name}_barrier", []).append(timeit(run(epi, (0, 0, 0))))
            times.setdefault(f"{name}_barrier_noepi", []).append(timeit(run(epi, (0, 0, 0), 16)))
            for v in variants:
                times.setdefault(f"{name}_stag{v}", []).append(timeit(run(epi, v)))
            times.setdefault(f"{name}_stag_noepi", []).append(timeit(run(epi, (1, 1, 0), 16)))
    h.conv_stack2_set_mode(0)
    h.conv_stack2_set_sched(0, 1, 0)
    out["us"] = {k: round(min(v), 1) for k, v in times.items()}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
