"""fp8 training fidelity bisection in the memorisation regime (tests/test_train_gpu.py
test_fp8_stress_vs_bf16_memorisation): the same init and batch stream (a 256-position subset
of the real fixture, cycled) through bf16 and through the fp8 path with each fp8 stage
switched back to bf16 in turn — forward stack (always fp8 with dtype=fp8), e5m2 backward-data
stack (DG_FP8_DGRAD), MX-fp8 weight gradients (DG_FP8_WGRAD) — and the e5m2 gradients rounded
to nearest even instead of stochastically (DG_FP8_SR=0).  Round 4 result (12x128, 800
steps, rate 0.1): nearest-even e5m2 gradients stall near 5.3 nats while bf16 reaches 2.7;
bf16 backward-data recovers it (so the forward is fine): the fix is stochastic rounding.
"ghead" variants: other e5m2 gradient-scale headrooms (hip_model.FP8_G_HEADROOM).  Prints the
100-step window mean losses per variant (and writes gpurun_out/fp8_memo_12x<ch>.json).
Usage: [FP8_MEMO_VARIANTS=name,...] python tools/fp8_memo.py [CH] [STEPS] [RATE]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from deep_go_amd.models import hip_model
    global G_HEAD0
    G_HEAD0 = hip_model.FP8_G_HEADROOM
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    from deep_go_amd.train.backends import HIPBackend
    ch = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 800
    rate = float(sys.argv[3]) if len(sys.argv) > 3 else 0.1
    B = 64
    fix = os.path.join(ROOT, "tests", "fixtures")
    pk = PackedDataset.load(os.path.join(fix, "train.dgpack.npz"))
    ld = BatchLoader(pk, B, threads=2, prefetch=4, seed=9, pin=False)
    subset = [ld.next_numpy() for _ in range(256 // B)]
    ld.close()
    variants = [("bf16", "bf16", {}),
                ("fp8", "fp8", {}),
                ("fp8 rne", "fp8", {"DG_FP8_SR": "0"}),
                ("fp8 bf16-wgrad", "fp8", {"DG_FP8_WGRAD": "0"}),
                ("fp8 bf16-dgrad", "fp8", {"DG_FP8_DGRAD": "0", "DG_FP8_WGRAD": "0"}),
                ("fp8 ghead2", "fp8", {"ghead": 2.0}),
                ("fp8 ghead8", "fp8", {"ghead": 8.0}),
                ]
    only = os.environ.get("FP8_MEMO_VARIANTS")
    if only:
        variants = [v for v in variants if v[0] in only.split(",")]
    out, flat0 = {}, None
    for name, dt, env in variants:
        from deep_go_amd.models import hip_model
        for k in ("DG_FP8_WGRAD", "DG_FP8_DGRAD", "DG_FP8_SR"):
            os.environ.pop(k, None)
        env = dict(env)
        hip_model.FP8_G_HEADROOM = env.pop("ghead", G_HEAD0)
        os.environ.update(env)
        cfg = ExperimentConfig(numLayers=12, channelSize=ch, batchSize=B, rate=rate,
                               rateDecay=1e-5, head_relu=False, useCuda=True, seed=13,
                               dtype=dt, checkpoint_dir="/tmp", data_root=fix)
        be = HIPBackend(cfg, B, flat=flat0)
        if flat0 is None:
            flat0 = be.flat_params().clone()
        ls = []
        for k in range(N):
            be.set_batch(*subset[k % len(subset)])
            be.train_step()
            ls.append(be.loss_sum() / B)
        ls = np.array(ls)
        rec = {"windows": [round(float(ls[w:w + 100].mean()), 4) for w in range(0, N, 100)]}
        if dt == "fp8":
            rec["ghead"] = hip_model.FP8_G_HEADROOM
            rec["sat"] = be.net.fp8_sat.cpu().tolist()
            rec["scales"] = be.net.fp8_scales.cpu().tolist()
            rec["gscales"] = be.net.fp8_gscales.cpu().tolist()
        out[name] = rec
        print(name, rec["windows"], flush=True)
        del be
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"fp8_memo_12x{ch}.json"), "w") as f:
        json.dump(out, f)


if __name__ == "__main__":
    main()
