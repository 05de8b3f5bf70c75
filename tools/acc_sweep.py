"""Sweep of the bench's accuracy phase (deep_go_amd/train/accuracy.py) over learning rate /
batch / steps with the reference's head ReLU, to pick a configuration that learns.
Usage: python tools/acc_sweep.py [--layers 12] [--channels 128] [--steps 2000]
One JSON line per setting (stdout)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--steps", default="2000")
    ap.add_argument("--rates", default="0.005,0.01,0.02,0.05,0.1")
    ap.add_argument("--batches", default="64,256")
    ap.add_argument("--head-relu", type=int, default=1)
    a = ap.parse_args()
    import torch
    from deep_go_amd.train.accuracy import fixture_accuracy
    dev = torch.device("cuda", 0)
    for steps in [int(x) for x in a.steps.split(",")]:
        for b in [int(x) for x in a.batches.split(",")]:
            for r in [float(x) for x in a.rates.split(",")]:
                out = fixture_accuracy(dev, layers=a.layers, channels=a.channels, steps=steps,
                                       batch=b, rate=r, head_relu=bool(a.head_relu))
                print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
