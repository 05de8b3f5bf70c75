"""Command line: ``python -m deep_go_amd <command> ...``

  train     [--preset NAME] [key=value ...] --iters N [--export-t7 PATH] [--auto-resume]
            (localtest.lua / default-experiment.lua / notebook equivalents via presets)
  resume    CKPT --iters N [--reset-optimizer] [--id NAME] [key=value ...]
            (experiments/repeated.lua: -gpu/-num/-iters -> --device/--id/--iters)
  eval      CKPT [--split test] [--n N]          (top-1 / NLL on a split; never done in the ref)
  makedata  scatter SRC DST train=N validation=N test=N | transcribe SRC DST [--threads T] [--ko]
            | count ROOT SPLIT | pack ROOT SPLIT
  export    CKPT OUT.t7        (reference Torch7 experiment table)
  import    IN.t7 OUT.model
  plot      FILE... [--out PNG] (validation/training curves from checkpoints or JSONL; plot.lua)
  bench     [bench.py args]

Multi-GPU: launch with ``python -m torch.distributed.run --nproc-per-node N -m deep_go_amd
train ...`` (one rank per GPU, RCCL); ``batchSize`` is the GLOBAL batch (split across ranks,
like nn.DataParallelTable).
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def _cfg_from(args, base=None):
    from .config import ExperimentConfig, get_preset, parse_overrides
    ov = parse_overrides(args.overrides)
    if base is not None:
        return base.replace(**ov) if ov else base
    if args.preset:
        return get_preset(args.preset, **ov)
    return ExperimentConfig().replace(**ov) if ov else ExperimentConfig()


def cmd_train(args):
    from .train.experiment import Experiment
    cfg = _cfg_from(args)
    if args.device == "cpu":
        cfg = cfg.replace(useCuda=False)
    elif args.device == "gpu":
        cfg = cfg.replace(useCuda=True)
    e = Experiment(cfg)
    iters = args.iters
    if args.auto_resume:
        # restart after a failure: continue <checkpoint_dir>/<id>.model
        # (exact resume: weights, optimizer, iteration, sampler cursor, RNG) up to --iters
        if not cfg.id:
            raise SystemExit("--auto-resume needs a stable experiment id (id=NAME)")
        path = e.checkpoint_path()
        if os.path.exists(path):
            e = Experiment.load(path)
            if args.device == "cpu":
                e.cfg = e.cfg.replace(useCuda=False)
            iters = max(0, args.iters - e.iterations)
            print(json.dumps({"auto_resume": path, "from_iteration": e.iterations}), flush=True)
    try:
        res = e.run(iters) if iters > 0 else {"iterations": e.iterations}
        if e.info.is_main:
            e.save()
            if args.export_t7:
                e.export_t7(args.export_t7)
            print(json.dumps({"id": e.id, "checkpoint": e.checkpoint_path(), **res}))
    finally:
        e.close()
    return 0


def cmd_resume(args):
    from .config import parse_overrides
    from .train.experiment import Experiment
    ov = parse_overrides(args.overrides)
    e = Experiment.load(args.checkpoint, reset_optimizer=args.reset_optimizer, **ov)
    if args.id:
        e.id = args.id
    if args.device == "cpu":
        e.cfg = e.cfg.replace(useCuda=False)
    try:
        res = e.run(args.iters)
        if e.info.is_main:
            e.save()
            print(json.dumps({"id": e.id, "checkpoint": e.checkpoint_path(), **res}))
    finally:
        e.close()
    return 0


def cmd_eval(args):
    from .train.experiment import Experiment
    e = Experiment.load(args.checkpoint)
    if args.device == "cpu":
        e.cfg = e.cfg.replace(useCuda=False)
    try:
        cost, acc = e.evaluate_split(args.split, args.n)
    finally:
        e.close()
    print(json.dumps({"split": args.split, "cost": cost, "accuracy": acc}))
    return 0


def cmd_makedata(args):
    from .data import makedata as md
    a = args.rest
    if not a:
        raise SystemExit("makedata: scatter|transcribe|count|pack")
    op = a[0]
    if op == "scatter":
        cats = dict(x.split("=") for x in a[3:])
        print(json.dumps(md.scatter(a[1], a[2], {k: int(v) for k, v in cats.items()},
                                    seed=args.seed)))
    elif op == "transcribe":
        print(json.dumps(md.transcribe(a[1], a[2], threads=args.threads, mark_ko=args.ko)))
    elif op == "count":
        print(md.count(a[1], a[2]))
    elif op == "pack":
        print(md.pack(a[1], a[2], threads=args.threads))
    else:
        raise SystemExit(f"unknown makedata op {op}")
    return 0


def cmd_export(args):
    from .utils import checkpoint as ck
    cfg, flat, state, opt = ck.load_checkpoint(args.checkpoint)
    ck.export_t7(args.out, cfg, flat, state, float(opt.get("rate", cfg.rate)))
    print(args.out)
    return 0


def cmd_import(args):
    from .utils import checkpoint as ck
    cfg, flat, state, rate = ck.import_t7(args.t7)
    state.setdefault("id", "imported")
    ck.save_checkpoint(args.out, cfg, flat, state,
                       {"kind": "sgd", "rate": rate, "rate_decay": cfg.rateDecay})
    print(args.out)
    return 0


def cmd_plot(args):
    from .utils.plot import plot_files
    print(plot_files(args.files, args.out))
    return 0


def cmd_bench(args):
    import runpy
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.argv = [os.path.join(root, "bench.py")] + args.rest
    runpy.run_path(sys.argv[0], run_name="__main__")
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(prog="deep_go_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train")
    t.add_argument("--preset")
    t.add_argument("--iters", type=int, required=True)
    t.add_argument("--device", choices=["auto", "cpu", "gpu"], default="auto")
    t.add_argument("--export-t7")
    t.add_argument("--auto-resume", action="store_true",
                   help="continue from <checkpoint_dir>/<id>.model if it exists (--iters = total)")
    t.add_argument("overrides", nargs="*")
    t.set_defaults(fn=cmd_train)
    r = sub.add_parser("resume")
    r.add_argument("checkpoint")
    r.add_argument("--iters", type=int, default=100)
    r.add_argument("--reset-optimizer", action="store_true")
    r.add_argument("--id")
    r.add_argument("--device", choices=["auto", "cpu", "gpu"], default="auto")
    r.add_argument("overrides", nargs="*")
    r.set_defaults(fn=cmd_resume)
    e = sub.add_parser("eval")
    e.add_argument("checkpoint")
    e.add_argument("--split", default="test")
    e.add_argument("--n", type=int)
    e.add_argument("--device", choices=["auto", "cpu", "gpu"], default="auto")
    e.set_defaults(fn=cmd_eval)
    m = sub.add_parser("makedata")
    m.add_argument("--threads", type=int, default=32)
    m.add_argument("--ko", action="store_true",
                   help="mark the simple-ko point in the stored liberty plane (for ko_plane=1)")
    m.add_argument("--seed", type=int, default=0)
    m.add_argument("rest", nargs="*")
    m.set_defaults(fn=cmd_makedata)
    x = sub.add_parser("export")
    x.add_argument("checkpoint")
    x.add_argument("out")
    x.set_defaults(fn=cmd_export)
    i = sub.add_parser("import")
    i.add_argument("t7")
    i.add_argument("out")
    i.set_defaults(fn=cmd_import)
    p = sub.add_parser("plot")
    p.add_argument("files", nargs="+")
    p.add_argument("--out", default="curves.png")
    p.set_defaults(fn=cmd_plot)
    b = sub.add_parser("bench")
    b.add_argument("rest", nargs=argparse.REMAINDER)
    b.set_defaults(fn=cmd_bench)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
