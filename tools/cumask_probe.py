"""Does a CU-masked HIP stream keep its mask (a) eagerly, (b) inside a captured hipGraph replayed
on that stream, (c) as the side branch of a graph forked from an unmasked stream (the step
graph's shape: hip_model.py captures its side stream's kernels as a parallel branch)?

VERDICT r5 "next round" 1(a): reserve CUs for the side chain with
hipExtStreamCreateWithCUMask and check that capture keeps the mask.  The probe times one
bf16 GEMM (hipBLASLt) on a stream masked to 1/8 of the CUs: a kept mask shows as ~8x the
unmasked time.

Usage: python tools/cumask_probe.py [--frac 8] [--n 8192]"""
import argparse
import ctypes
import json
import os

import torch


def masked_stream(lib, ncu, keep):
    """A HIP stream limited to the CUs whose mask bit is set (every keep-th CU)."""
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for cu in range(0, ncu, keep):
        mask[cu // 32] |= 1 << (cu % 32)
    h = ctypes.c_void_p()
    err = lib.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
    if err != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask failed: {err}")
    back = (ctypes.c_uint32 * words)()
    err = lib.hipExtStreamGetCUMask(h, ctypes.c_uint32(words), back)
    readback = [int(v) for v in back] if err == 0 else f"error {err}"
    return (torch.cuda.ExternalStream(h.value), sum(bin(m).count("1") for m in mask),
            [int(v) for v in mask], readback)


def timed(fn, stream, reps=10):
    with torch.cuda.stream(stream):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    with torch.cuda.stream(stream):
        for _ in range(reps):
            fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frac", type=int, default=8)
    ap.add_argument("--n", type=int, default=8192)
    a = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    x = torch.randn(a.n, a.n, device="cuda", dtype=torch.bfloat16)
    y = torch.randn(a.n, a.n, device="cuda", dtype=torch.bfloat16)
    out = torch.empty_like(x)
    mm = lambda: torch.matmul(x, y, out=out)  # noqa: E731
    plain = torch.cuda.Stream()
    ms, nbits, asked, readback = masked_stream(lib, ncu, a.frac)
    res = {"cus": ncu, "mask_cus": nbits, "n": a.n, "mask": asked, "readback": readback}
    timed(mm, plain)   # clock ramp
    res["eager_plain_ms"] = timed(mm, plain)
    res["eager_masked_ms"] = timed(mm, ms)

    # (b) graph captured on the masked stream, replayed on it and on an unmasked stream
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(ms):
        mm()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=ms):
        mm()
    res["graph_on_masked_replay_masked_ms"] = timed(g.replay, ms)
    res["graph_on_masked_replay_plain_ms"] = timed(g.replay, plain)

    # (c) fork/join: the GEMM is a side branch captured from the masked stream
    g2 = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream()
    with torch.cuda.graph(g2, stream=cap):
        ev = torch.cuda.Event()
        ev.record(cap)
        ms.wait_event(ev)
        with torch.cuda.stream(ms):
            mm()
        ev2 = torch.cuda.Event()
        ev2.record(ms)
        cap.wait_event(ev2)
    res["graph_side_branch_replay_plain_ms"] = timed(g2.replay, plain)
    res["mask_kept_eager"] = res["eager_masked_ms"] > 2.5 * res["eager_plain_ms"]
    res["mask_kept_graph"] = res["graph_on_masked_replay_masked_ms"] > 2.5 * res["eager_plain_ms"]
    res["mask_kept_side_branch"] = (res["graph_side_branch_replay_plain_ms"]
                                    > 2.5 * res["eager_plain_ms"])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
