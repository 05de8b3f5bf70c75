"""End-to-end training throughput through the real pipeline (C++ loader threads -> pinned
packed slots -> one async H2D copy -> graphed step), on the packed reference fixture, at the
flagship shape (12 layers x 128 channels, batch 256).  Compare with bench.py (synthetic,
device-resident pool) to see what the input pipeline costs.

The Experiment runs with its DEFAULT policies (nan_policy=guard: the device gate, one fused
graph per step; comm=auto), i.e. what `python -m deep_go_amd train` gives a user.
--synthetic: the trainer's synthetic positions (C++ engine games) through the same loader
instead of the fixture (compare with bench.py's device-resident synthetic pool).

Usage: python tools/pipeline_bench.py [--iters 400] [--threads 4] [--data tests/fixtures]
                                      [--ch 256] [--dtype fp8] [--synthetic]"""
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
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--synthetic", action="store_true")
    a = ap.parse_args()
    import torch
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.train.experiment import Experiment
    cfg = ExperimentConfig(numLayers=a.layers, channelSize=a.ch, batchSize=a.batch, rate=0.05,
                           rateDecay=1e-7, useCuda=True, data_root=a.data, validationSize=256,
                           validation_interval=10 ** 9, log_interval=100,
                           checkpoint_dir="/tmp", seed=3, loader_threads=a.threads,
                           dtype=a.dtype, synthetic=a.synthetic)
    e = Experiment(cfg, id="pipeline")
    e.run(50)  # warmup: graph capture, loader spin-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e.run(a.iters)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"metric": "trainer boards/s (" + ("synthetic" if a.synthetic else
                                                          "real fixture") + " data, 1 GPU)",
                      "value": round(a.batch * a.iters / dt, 1),
                      "ms_per_step": round(1e3 * dt / a.iters, 4), "threads": a.threads,
                      "dtype": a.dtype, "nan_policy": cfg.nan_policy,
                      "config": f"{a.layers}x{a.ch} b{a.batch}"}), flush=True)


if __name__ == "__main__":
    main()
