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
    ap.add_argument("--timeline", action="store_true",
                    help="only the fp8 phase stamps (conv_stack_f8_set_debug) per schedule")
    a = ap.parse_args()
    h = hip()
    if a.timeline:
        print(json.dumps(fp8_stag(h, a.boards, 10, stream_handle(), a.rounds, timeline=True)))
        return
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
    h.conv_stack2_set_sched(2, 1, 0)
    out["us"] = {k: round(min(v), 1) for k, v in times.items()}
    out["fp8"] = fp8_stag(h, B, NL, s, a.rounds)
    print(json.dumps(out))


def fp8_stag(h, B, NL, s, rounds, timeline=False):
    """conv_stack_f8 C = 128 (the production variants: fp8 copies of every non-last output, the
    last layer's bf16 frame; backward-data e5m2 with SR): bit-identity of every output, the
    |y| maxima included, between the barrier and staggered schedules, then their times."""
    C, dev = 128, "cuda"
    torch.manual_seed(1)
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    ys = [LY.alloc_frame(B, C, 1, dev) for _ in range(NL)]
    ms = [torch.randint(0, 255, (B, 361, C // 8), dtype=torch.uint8, device=dev)
          for _ in range(NL)]
    md = [m.clone() for m in ms]
    pbs = [(0.01 * torch.randn(24 * 2 * 4 * 64 * 4, device=dev)).to(torch.bfloat16)
           for _ in range(NL)]
    w8 = [LY.stack_frag_f8(torch.randint(0, 0x78, (C, 9, C), dtype=torch.uint8, device=dev))
          for _ in range(NL)]
    sc = torch.full((NL + 1,), 2.0 ** -6, device=dev)
    amax = torch.zeros(NL + 1, dtype=torch.int32, device=dev)
    x8 = [torch.zeros(B * 448 * C, dtype=torch.uint8, device=dev) for _ in range(NL)]
    sr = torch.full((1,), 5, dtype=torch.int64, device=dev)

    def table(fwd):
        t = np.array([[w8[i].data_ptr(), pbs[i].data_ptr() if fwd else 0,
                       ys[i].data_ptr() if i == NL - 1 else 0,
                       (ms if fwd else md)[i].data_ptr(), sc.data_ptr() + 4 * i,
                       sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * (i + 1),
                       amax.data_ptr() + 4 * (i + 1)] for i in range(NL)], dtype=np.int64)
        return np.ascontiguousarray(t)
    tf, td = table(True), table(False)
    y8 = np.array([x8[0].data_ptr()] + [x8[i + 1].data_ptr() if i + 1 < NL else 0
                                        for i in range(NL)], dtype=np.int64)

    def run(fwd, stag, delay=0):
        def f():
            h.conv_stack_f8_set_sched(stag, delay)
            if fwd:
                h.conv_stack_f8_y8(C, h.EPI_FWD, tf.ctypes.data, NL, x.data_ptr(),
                                   sc.data_ptr(), amax.data_ptr(), B, y8.ctypes.data, s)
            else:
                h.conv_stack_f8_dgrad(C, td.ctypes.data, NL, x.data_ptr(), sc.data_ptr(),
                                      amax.data_ptr(), B, y8.ctypes.data, sr.data_ptr(), s)
        return f
    out = {}
    if timeline:
        dbg = torch.zeros(8 * 8 * 24 * 8, dtype=torch.int64, device=dev)
        for fwd, name in ((True, "fwd"), (False, "dgrad")):
            for stag, mode in ((0, 0), (1, 0), (0, 4)):
                h.conv_stack_f8_set_mode(mode)
                run(fwd, stag)()
                dbg.zero_()
                h.conv_stack_f8_set_debug(dbg.data_ptr())
                run(fwd, stag)()
                torch.cuda.synchronize()
                h.conv_stack_f8_set_debug(0)
                h.conv_stack_f8_set_mode(0)
                out[f"{name}_stag{stag}_mode{mode}"] = summarize(
                    dbg.view(8, 8, 24, 8).cpu().numpy(), NL)
        h.conv_stack_f8_set_sched(1, 0)
        return out
    for fwd, name in ((True, "fwd"), (False, "dgrad")):
        outs = []
        for stag in (0, 1):
            for t in x8 + [ys[-1], amax] + (ms if fwd else []):
                t.zero_()
            run(fwd, stag)()
            torch.cuda.synchronize()
            outs.append([t.clone() for t in x8 + [ys[-1], amax] + (ms if fwd else [])])
        out[f"{name}_bit_identical"] = all(torch.equal(p, q) for p, q in zip(*outs))
    times = {}
    for _ in range(rounds):
        for fwd, name in ((True, "fwd"), (False, "dgrad")):
            times.setdefault(f"{name}_barrier", []).append(timeit(run(fwd, 0)))
            times.setdefault(f"{name}_stag", []).append(timeit(run(fwd, 1)))
            times.setdefault(f"{name}_stag_delay1", []).append(timeit(run(fwd, 1, 1)))
    h.conv_stack_f8_set_sched(1, 0)
    out["us"] = {k: round(min(v), 1) for k, v in times.items()}
    return out


def summarize(t, NL):
    """Phase lengths (cycles, mean over boards 0..7 and layers 1..NL-2) per co-half from the
    stamps [board][wave][layer][k]: k 0 layer top, 1 after the input waits, 2 K loop end,
    3 after the epilogue's wait (R or barrier), 4 epilogue end (+ amax), 5 after the barrier
    schedule's closing barrier; and the co-half-1 lag (its layer top minus co-half 0's)."""
    t = t.astype(np.int64)
    ls = slice(1, NL - 1)
    out = {}
    for g in (0, 1):
        w = t[:, 4 * g:4 * g + 4, ls, :]
        nxt = t[:, 4 * g:4 * g + 4, 2:NL, 0]
        out[f"g{g}"] = {
            "in_wait": float(np.mean(w[..., 1] - w[..., 0])),
            "kloop": float(np.mean(w[..., 2] - w[..., 1])),
            "epi_wait": float(np.mean(w[..., 3] - w[..., 2])),
            "epi": float(np.mean(w[..., 4] - w[..., 3])),
            "layer": float(np.mean(nxt - w[..., 0])),
        }
    out["g1_lag"] = float(np.mean(t[:, 4:8, ls, 0] - t[:, 0:4, ls, 0]))
    return {k: ({kk: round(vv) for kk, vv in v.items()} if isinstance(v, dict) else round(v))
            for k, v in out.items()}


if __name__ == "__main__":
    main()
