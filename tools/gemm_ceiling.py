"""Practical bf16 / fp8 MFMA ceiling on this box: hipBLASLt GEMMs (torch.matmul / _scaled_mm)
on random data, timed by back-to-back launches after a >2 s clock ramp.

The hand-written conv kernels are priced against this number rather than the 2.5 PF/s
datasheet peak: under load the chip lowers its clock (MI355X_MICROARCH.md, DVFS give-back),
so a dense MFMA body on random operands sustains well under the nominal rate.
"""
import json
import time

import torch


def bench(fn, flops, secs=2.0):
    fn()
    torch.cuda.synchronize()
    t0 = time.time()
    n = 0
    while time.time() - t0 < secs:   # clock ramp
        fn()
        n += 1
        if n % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(8, n // 4)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return flops / (ms * 1e-3) / 1e12, ms


def main():
    torch.manual_seed(0)
    out = {}
    for (m, n, k) in [(8192, 8192, 8192), (16384, 16384, 8192), (128, 92416, 1152),
                      (1152, 128, 92416)]:
        a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
        tf, ms = bench(lambda: torch.matmul(a, b), 2.0 * m * n * k)
        out[f"bf16 {m}x{n}x{k}"] = {"TFLOPs": round(tf, 1), "ms": round(ms, 4)}
        print(f"bf16 {m}x{n}x{k}: {tf:.1f} TF/s ({ms:.3f} ms)", flush=True)
    try:
        m = n = k = 8192
        a = torch.randn(m, k, device="cuda").to(torch.float8_e4m3fn)
        b = torch.randn(n, k, device="cuda").to(torch.float8_e4m3fn).t()
        one = torch.ones((), device="cuda")
        tf, ms = bench(lambda: torch._scaled_mm(a, b, scale_a=one, scale_b=one,
                                                out_dtype=torch.bfloat16), 2.0 * m * n * k)
        out[f"fp8 {m}x{n}x{k}"] = {"TFLOPs": round(tf, 1), "ms": round(ms, 4)}
        print(f"fp8 e4m3 {m}x{n}x{k}: {tf:.1f} TF/s ({ms:.3f} ms)", flush=True)
    except Exception as e:  # noqa: BLE001
        print("fp8 scaled_mm unavailable:", e)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
