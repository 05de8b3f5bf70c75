"""End-to-end training throughput through the real pipeline (C++ loader threads -> pinned
packed slots -> one async H2D copy -> graphed step), on the packed reference fixture, at the
flagship shape (12 layers x 128 channels, batch 256).  Compare with bench.py (synthetic,
device-resident pool) to see what the input pipeline costs.

Usage: python tools/pipeline_bench.py [--iters 400] [--threads 4] [--data tests/fixtures]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--ch", type=int, default=128)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--data", default="tests/fixtures")
    a = ap.parse_args()
    import torch
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.train.experiment import Experiment
    cfg = ExperimentConfig(numLayers=a.layers, channelSize=a.ch, batchSize=a.batch, rate=0.05,
                           rateDecay=1e-7, useCuda=True, data_root=a.data, validationSize=256,
                           validation_interval=10 ** 9, log_interval=100,
                           checkpoint_dir="/tmp", nan_policy="skip", seed=3,
                           loader_threads=a.threads)
    e = Experiment(cfg, id="pipeline")
    e.run(50)  # warmup: graph capture, loader spin-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.run(a.iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "pipeline boards/s (real data, 1 GPU)",
                      "value": a.batch * a.iters / dt, "ms_per_step": 1e3 * dt / a.iters,
                      "threads": a.threads, "config": f"{a.layers}x{a.ch} b{a.batch}"}))


if __name__ == "__main__":
    main()
