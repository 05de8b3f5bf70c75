"""grad_update (elementwise.hip: the fused end-of-step gradient pass 2 + SGD + operand refresh
+ LR decay) alone, timed with HIP events over R back-to-back calls on a model whose deferred
training step left its split-K slabs and bias partials, with ablated launch tables to see
where its time goes:

  full      the production table
  splits1   every deferred layer sums ONE slab (slab traffic / split count)
  nobias    bias and position-bias gradients from the flat gradient (no bias partials)
  nocopy    no operand copies (bf16 / fp8 fragment layouts, bias tables): update only
  noslab    no slabs at all: every layer's gradient from the flat gradient (= the DP form)
  old       the separate launches it replaces: wgrad_reduce(_multi) + sgd + weight_refresh

(Repeated calls keep applying the same gradient; the timing does not depend on the values.)
Usage: python tools/kbench_gu.py [CH] [DTYPE] [R]  -> one JSON line (us per call)"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# refresh-row columns that hold optional operand-copy outputs (elementwise.hip
# parse_refresh_row): wf, wd, pbias_frag, wf8, pbias, wf_frag, wd_frag, wf8_frag, wd8_frag
COPY_COLS = (1, 2, 9, 10, 15, 16, 17, 18, 19)


def main():
    from deep_go_amd.config import get_preset
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet
    from deep_go_amd.ops.native import stream_handle
    ch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
    R = int(sys.argv[3]) if len(sys.argv) > 3 else 50
    B = 256
    cfg = get_preset("12x128-bf16", channelSize=ch, batchSize=B, dtype=dt)
    net = HipGoNet(cfg, B, device="cuda:0")
    pl, py, rk, lb = random_planes(B, seed=1)
    net.set_batch(*(torch.from_numpy(a).cuda() for a in (pl, py, rk, lb)))
    assert net.can_defer(), "needs the deferred (single-GPU, grouped-wgrad) step"
    net.set_defer(True)
    net.forward_backward()          # slabs + bias partials of this step stay in place
    torch.cuda.synchronize()
    h, s = net.h, stream_handle()
    n = net.params.numel()
    hd = net.head
    base = net._gu_table(True).copy()
    flat = net._gu_table(False).copy()
    grads_ok = net.grads.abs().sum().item() >= 0   # (the flat gradient: whatever it holds)
    assert grads_ok

    def gu(table):
        def run():
            h.grad_update(table.ctypes.data, len(table), hd.w_off, n - hd.w_off,
                          net.params.data_ptr(), net.grads.data_ptr(), 0, 0, 0.9, 1.0,
                          net.gate.data_ptr(), net.lr.data_ptr(), 0.0,
                          net.step_count.data_ptr(), net.gu_tickets.data_ptr(),
                          net.bad_steps.data_ptr(), 0, 1, 0, s)
        return run

    variants = {"full": base}
    t = base.copy()
    sl = t[:, 20] != 0
    t[sl, 22] = 1
    variants["splits1"] = t
    t = base.copy()
    t[:, 21] = 0
    variants["nobias"] = t
    t = base.copy()
    t[:, list(COPY_COLS)] = 0
    variants["nocopy"] = t
    variants["noslab"] = flat
    runs = {k: gu(np.ascontiguousarray(v)) for k, v in variants.items()}

    def old():
        for g in net.wgroups:              # the grouped slab reduce(s) the deferral skips
            f, a = net._bwd[g[0]][2]
            f(*a, s)
        h.sgd(net.params.data_ptr(), net.grads.data_ptr(), n, net.lr.data_ptr(), 1.0,
              net.gate.data_ptr(), s)
        rt = net._step_refresh_table()
        h.weight_refresh_decay(rt.ctypes.data, len(rt), net.lr.data_ptr(), 0.0,
                               net.step_count.data_ptr(), s)
    runs["old"] = old

    out = {"config": f"12x{ch}-{dt}", "calls": R}
    for k, fn in runs.items():
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(R):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[k] = round(1000.0 * e0.elapsed_time(e1) / R, 2)
    assert int(net.gu_tickets.abs().sum().item()) == 0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
