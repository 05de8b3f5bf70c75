"""HIP trainer vs fp32 oracle on the accuracy half (deep_go_amd/train/accuracy.py
oracle_parity): prints per-split top-1 / NLL of both runs and the loss-curve gaps.
Usage: python tools/acc_parity.py [--steps 500] [--rate 0.05] [--layers 6] [--channels 64]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--rate", type=float, default=0.05)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--channels", type=int, default=64)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seed", type=int, default=5)
    ap.add_argument("--perturb", default="", help="comma-separated relative init perturbations "
                    "of extra fp32 oracle runs (SGD's own sensitivity)")
    a = ap.parse_args()
    import numpy as np
    import torch
    from deep_go_amd.train.accuracy import oracle_parity
    r = oracle_parity(torch.device("cuda", 0), layers=a.layers, channels=a.channels,
                      batch=a.batch, rate=a.rate, steps=a.steps, seed=a.seed,
                      perturb=[float(x) for x in a.perturb.split(",") if x])
    for n in r["runs"][2:]:
        lp = np.array(r.pop(f"loss_{n}"))
        r[f"gap_{n}_vs_cpu"] = {str(k): round(float(abs(lp[k] - np.array(r["loss_cpu"])[k])), 5)
                                for k in (100, 200, 300, 400, len(lp) - 1) if k < len(lp)}
    lc, lg = np.array(r.pop("loss_cpu")), np.array(r.pop("loss_hip"))
    r["loss_first50"] = [round(lc[:50].mean(), 4), round(lg[:50].mean(), 4)]
    r["loss_last50"] = [round(lc[-50:].mean(), 4), round(lg[-50:].mean(), 4)]
    r["loss_max_abs_gap"] = round(float(np.abs(lc - lg).max()), 5)
    r["loss_gap_at"] = {str(k): round(float(abs(lc[k] - lg[k])), 5)
                        for k in (0, 10, 50, 100, 200, 300, 400, len(lc) - 1) if k < len(lc)}
    print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
