"""Train on the packed reference fixture and report validation cost/accuracy over time.

Usage: python tools/real_data_run.py [--rates 0.05,0.1] [--iters 1000] [--layers 6] [--ch 64]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="0.05,0.1,0.2")
    ap.add_argument("--iters", type=int, default=1000)
    ap.add_argument("--layers", type=int, default=6)
    ap.add_argument("--ch", type=int, default=64)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--head-relu", type=int, default=0)
    ap.add_argument("--data", default="tests/fixtures")
    a = ap.parse_args()
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.train.experiment import Experiment
    out = []
    for r in [float(x) for x in a.rates.split(",")]:
        cfg = ExperimentConfig(numLayers=a.layers, channelSize=a.ch, batchSize=a.batch,
                               rate=r, rateDecay=1e-7, head_relu=bool(a.head_relu),
                               useCuda=True, data_root=a.data, validationSize=256,
                               validation_interval=max(1, a.iters // 5), log_interval=50,
                               checkpoint_dir="/tmp", nan_policy="skip", seed=11)
        e = Experiment(cfg, id=f"real_r{r}")
        res = e.run(a.iters)
        tc, ta = e.evaluate_split("test", 125)
        out.append({"rate": r, "val_costs": e.validation_costs,
                    "val_acc": e.validation_accuracies, "test_cost": tc, "test_acc": ta,
                    "boards_per_sec": res["samples_per_sec"]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
