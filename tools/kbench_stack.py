"""Micro-benchmark + ablations of the board-resident layer-stack kernel (conv_stack.hip):
10 hidden 128->128 3x3 layers of 256 boards, forward and dgrad, ring depth 2 vs 3.
Interleaved in one process, random data.  Prints one JSON object (us per launch)."""
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
    ablations = "--ablate" in sys.argv
    h = hip()
    B, C, NL = 256, 128, 10
    dev = "cuda"
    x = LY.alloc_frame(B, C, 1, dev)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=dev).relu())
    KP, _, Mpad = LY.conv_dims(3, C, C, 128)
    ws, ys, ms, pbs = [], [], [], []
    for _ in range(NL):
        w = torch.randn(C, 3, 3, C, device=dev) / (3 * C ** 0.5)
        ws.append(LY.fwd_weight(w, C, KP, Mpad))
        ys.append(LY.alloc_frame(B, C, 1, dev))
        ms.append(torch.randint(0, 255, (B, 361, 16), dtype=torch.uint8, device=dev))
        pbs.append((0.01 * torch.randn(24 * 2 * 4 * 64 * 4, device=dev)).to(torch.bfloat16))  # fragment order
    tf = np.array([[ws[i].data_ptr(), pbs[i].data_ptr(), ys[i].data_ptr(), ms[i].data_ptr()]
                   for i in range(NL)], dtype=np.int64)
    td = np.array([[ws[i].data_ptr(), 0, ys[i].data_ptr(), ms[i].data_ptr()]
                   for i in range(NL)], dtype=np.int64)
    s = stream_handle()
    flops = 2.0 * C * C * 9 * 361 * B * NL
    res = {}

    def run(epi, table):
        return lambda: h.conv_stack(epi, table.ctypes.data, NL, x.data_ptr(), KP, B, s)
    # correctness of the variants against each other (same inputs -> same outputs)
    outs = {}
    for ring in (2, 3, 16):
        if ring == 16:
            h.conv_stack_set_waves(16)
        else:
            h.conv_stack_set_ring(ring)
        run(h.EPI_FWD, tf)()
        torch.cuda.synchronize()
        outs[ring] = [y.clone() for y in ys] + [m.clone() for m in ms]
    h.conv_stack_set_ring(0)
    h.conv_stack_set_waves(8)
    res_ok = all(torch.equal(a, b) for a, b in zip(outs[2], outs[3]))
    res_ok16 = all(torch.equal(a, b) for a, b in zip(outs[2], outs[16]))
    for rnd in range(2):
        for ring in (2, 3):
            h.conv_stack_set_ring(ring)
            for name, epi, t in (("fwd", h.EPI_FWD, tf), ("dgrad", h.EPI_DGRAD, td)):
                res.setdefault(f"ring{ring}_{name}", []).append(round(timeit(run(epi, t)), 1))
            for abl in ((1, 2, 4, 8, 16, 6, 12, 14) if ablations and ring > 1 else ()):
                h.conv_stack_set_ablate(abl)
                res.setdefault(f"ring{ring}_fwd_abl{abl}", []).append(
                    round(timeit(run(h.EPI_FWD, tf)), 1))
                h.conv_stack_set_ablate(0)
        h.conv_stack_set_ring(0)
        h.conv_stack_set_bpf(0)
        for name, epi, t in (("fwd", h.EPI_FWD, tf), ("dgrad", h.EPI_DGRAD, td)):
            res.setdefault(f"ring2_nobpf_{name}", []).append(round(timeit(run(epi, t)), 1))
        h.conv_stack_set_bpf(1)
        h.conv_stack_set_waves(16)
        for name, epi, t in (("fwd", h.EPI_FWD, tf), ("dgrad", h.EPI_DGRAD, td)):
            res.setdefault(f"w16_{name}", []).append(round(timeit(run(epi, t)), 1))
        h.conv_stack_set_waves(8)
        h.conv_stack_set_stagger(1)
        for name, epi, t in (("fwd", h.EPI_FWD, tf), ("dgrad", h.EPI_DGRAD, td)):
            res.setdefault(f"ring2_stagger_{name}", []).append(round(timeit(run(epi, t)), 1))
        h.conv_stack_set_stagger(0)
    out = {k: {"us": v, "us_per_layer": round(min(v) / NL, 2),
               "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)} for k, v in res.items()}
    out["variants_bit_identical"] = res_ok
    out["w16_bit_identical"] = res_ok16
    # phase breakdown (s_memtime per wave; the timestamps pin the schedule, ~+10%)
    names = ["copyout+dma_issue", "kk0(readA+mma)", "kk1(reads+mma)", "dma_wait", "barrier"]
    for mode, tag in ((32, ""), (40, "_nocopyout")):
        prof = torch.zeros(B * 8 * 8, dtype=torch.int64, device=dev)
        h.conv_stack_set_prof(prof.data_ptr())
        h.conv_stack_set_ablate(mode)
        run(h.EPI_FWD, tf)()
        torch.cuda.synchronize()
        h.conv_stack_set_ablate(0)
        h.conv_stack_set_prof(0)
        pr = prof.view(B, 8, 8).double()
        steps = pr[..., 6].mean().item()
        out["phase_cycles_per_step" + tag] = {n: round(pr[..., k].mean().item() / steps, 1)
                                              for k, n in enumerate(names)}
        out["epilogue_cycles_per_layer" + tag] = round(pr[..., 5].mean().item() / NL, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
