"""Micro-benchmark of the board-resident layer-stack kernels: 10 hidden 128->128 3x3 layers
of 256 boards, forward and dgrad, conv_stack (LDS weight ring, barrier per K-step) vs
conv_stack2 (fragment-ordered weights streamed into VGPRs).  Interleaved in one process on
random data; the two kernels' outputs must be bit-identical.  Prints one JSON object."""
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
    wf, wd, ff, fd, ys, ms, pbs = [], [], [], [], [], [], []
    for _ in range(NL):
        w = torch.randn(C, 3, 3, C, device=dev) / (3 * C ** 0.5)
        wf.append(LY.fwd_weight(w, C, KP, Mpad))
        wd.append(LY.dgrad_weight(w, KP, Mpad))
        ff.append(LY.stack_frag(wf[-1]))
        fd.append(LY.stack_frag(wd[-1]))
        ys.append(LY.alloc_frame(B, C, 1, dev))
        ms.append(torch.randint(0, 255, (B, 361, 16), dtype=torch.uint8, device=dev))
        pbs.append((0.01 * torch.randn(24 * 2 * 4 * 64 * 4, device=dev)).to(torch.bfloat16))

    def table(ws, fwd):
        return np.array([[ws[i].data_ptr(), pbs[i].data_ptr() if fwd else 0, ys[i].data_ptr(),
                          ms[i].data_ptr()] for i in range(NL)], dtype=np.int64)
    tabs = {("v1", "fwd"): table(wf, True), ("v1", "dgrad"): table(wd, False),
            ("v2", "fwd"): table(ff, True), ("v2", "dgrad"): table(fd, False)}
    s = stream_handle()
    def v2(bdb):
        def f(*a):
            h.conv_stack2_set_bdb(bdb)
            return h.conv_stack2(*a)
        return f
    fns = {"v1": h.conv_stack, "v2": v2(1), "v2nodb": v2(0)}
    abl = [2, 4, 6, 10, 14] if "--ablate" in sys.argv else []
    for m in abl:
        fns[f"v2m{m}"] = v2(m)
        tabs[(f"v2m{m}", "fwd")] = tabs[("v2", "fwd")]
    tabs[("v2nodb", "fwd")] = tabs[("v2", "fwd")]
    tabs[("v2nodb", "dgrad")] = tabs[("v2", "dgrad")]
    epis = {"fwd": h.EPI_FWD, "dgrad": h.EPI_DGRAD}

    def run(v, name):
        t = tabs[(v, name)]
        return lambda: fns[v](epis[name], t.ctypes.data, NL, x.data_ptr(), KP, B, s)

    out = {}
    mask0 = [m.clone() for m in ms]
    for name in ("fwd", "dgrad"):
        res = []
        for v in ("v1", "v2", "v2nodb"):
            for m, m0 in zip(ms, mask0):
                m.copy_(m0)
            for y in ys:
                y.zero_()
            run(v, name)()
            torch.cuda.synchronize()
            res.append([y.clone() for y in ys] + [m.clone() for m in ms])
        for k in (1, 2):
            bad = [i for i, (a, b) in enumerate(zip(res[0], res[k])) if not torch.equal(a, b)]
            out[f"{name}_v1_vs_{('v2', 'v2nodb')[k - 1]}_mismatch"] = [
                (i, float((res[0][i].float() - res[k][i].float()).abs().max())) for i in bad]
    for m, m0 in zip(ms, mask0):
        m.copy_(m0)
    flops = 2.0 * C * C * 9 * 361 * B * NL
    times = {}
    for _ in range(3):
        for v in ("v1", "v2", "v2nodb"):
            for name in ("fwd", "dgrad"):
                times.setdefault(f"{v}_{name}", []).append(round(timeit(run(v, name)), 1))
        for m in abl:
            times.setdefault(f"v2m{m}_fwd", []).append(round(timeit(run(f"v2m{m}", "fwd")), 1))
    h.conv_stack2_set_bdb(1)
    for k, v in times.items():
        out[k] = {"us": v, "us_per_layer": round(min(v) / NL, 2),
                  "tflops": round(flops / (min(v) * 1e-6) / 1e12, 1)}
    out["boards"] = B
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
