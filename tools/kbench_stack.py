"""Micro-benchmark of the board-resident layer stack (conv_stack2.hip): 10 hidden 128->128
3x3 layers of 256 boards, forward and dgrad, plus (--ablate) its timing ablations (no A
loads / no copy-out / no B reads).  Random data; prints one JSON object.  (The round-1
LDS-ring kernel it replaced is compared in profiles/r2_kbench_stack2.json.)"""
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
    B = int(os.environ.get("KB_BOARDS", "256"))
    C, NL = 128, 10
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

    def table(ws, fwd):
        return np.array([[ws[i].data_ptr(), pbs[i].data_ptr() if fwd else 0, ys[i].data_ptr(),
                          ms[i].data_ptr()] for i in range(NL)], dtype=np.int64)
    tabs = {"fwd": table(ff, True), "dgrad": table(fd, False)}
    s = stream_handle()
    epis = {"fwd": h.EPI_FWD, "dgrad": h.EPI_DGRAD}

    def run(name, mode=0):
        t = tabs[name]

        def f():
            h.conv_stack2_set_mode(mode)
            h.conv_stack2(epis[name], t.ctypes.data, NL, x.data_ptr(), 0, B, s)
        return f
    abl = [2, 4, 6, 10, 14] if "--ablate" in sys.argv else []
    out = {}
    # the fp8 forward stack (conv_stack_f8) on the same shapes: e4m3 weights / image
    w8 = [LY.stack_frag_f8(torch.randint(0, 0x78, (C, 9, C), dtype=torch.uint8, device=dev))
          for _ in range(NL)]
    sc = torch.full((NL + 1,), 2.0 ** -6, device=dev)
    amax = torch.zeros(NL + 1, dtype=torch.int32, device=dev)
    t8 = np.array([[w8[i].data_ptr(), pbs[i].data_ptr(), ys[i].data_ptr(), ms[i].data_ptr(),
                    sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * (i + 1),
                    amax.data_ptr() + 4 * (i + 1)] for i in range(NL)], dtype=np.int64)

    t8d = t8.copy()
    t8d[:, 1] = 0

    def run8(mode=0, nl=NL, epi=None):
        tt = t8 if epi is None else t8d

        def f():
            h.conv_stack_f8_set_mode(mode)
            h.conv_stack_f8(C, epi or h.EPI_FWD, tt.ctypes.data, nl, x.data_ptr(), sc.data_ptr(),
                            amax.data_ptr(), B, s)
        return f
    flops = 2.0 * C * C * 9 * 361 * B * NL
    times = {}
    for _ in range(3):
        for name in ("fwd", "dgrad"):
            times.setdefault(name, []).append(round(timeit(run(name)), 1))
        for m in abl:
            times.setdefault(f"fwd_mode{m}", []).append(round(timeit(run("fwd", m)), 1))
        times.setdefault("fp8_fwd", []).append(round(timeit(run8()), 1))
        times.setdefault("fp8_dgrad", []).append(round(timeit(run8(epi=h.EPI_DGRAD)), 1))
        times.setdefault("fp8_fwd_1layer", []).append(round(timeit(run8(nl=1)), 1))
        times.setdefault("fp8_fwd_2layers", []).append(round(timeit(run8(nl=2)), 1))
        for m in ([2, 4, 6] if abl else []):
            times.setdefault(f"fp8_fwd_mode{m}", []).append(round(timeit(run8(m)), 1))
    h.conv_stack2_set_mode(0)
    h.conv_stack_f8_set_mode(0)
    for k, v in times.items():
        out[k] = {"us": v, "us_per_layer": round(min(v) / NL, 2),
                  "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)}
    out["boards"] = B
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
