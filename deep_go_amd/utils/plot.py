"""Validation / training curves (the reference's plot.lua: plotAll / plotFromFile / plotVal,
which loaded every *.model checkpoint and plotted validation_costs against iterations)."""
from __future__ import annotations

from typing import List


def _series(path: str):
    if path.endswith(".jsonl"):
        from .metrics import read_jsonl
        rows = read_jsonl(path)
        val = [(r["step"], r["val_cost"]) for r in rows if r.get("kind") == "validation"]
        tr = [(r["step"], r["loss_ema"]) for r in rows if r.get("kind") == "train"]
        return val, tr
    from .checkpoint import load_checkpoint
    cfg, _, state, _ = load_checkpoint(path)
    vc = state.get("validation_costs", [])
    it = state.get("iterations", 0)
    step = it / max(1, len(vc))  # plotVal: evenly spaced over the run
    val = [((i + 1) * step, c) for i, c in enumerate(vc)]
    tc = state.get("train_costs", [])
    tr = [((i + 1) * cfg.log_interval, c) for i, c in enumerate(tc)]
    return val, tr


def plot_files(files: List[str], out: str) -> str:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(7, 4))
    for f in files:
        val, tr = _series(f)
        if val:
            ax.plot([v[0] for v in val], [v[1] for v in val], "o-", label=f"val {f}")
        if tr:
            ax.plot([v[0] for v in tr], [v[1] for v in tr], "-", alpha=0.6, label=f"train {f}")
    ax.set_xlabel("iteration")
    ax.set_ylabel("NLL")
    ax.set_title("Validation Cost")
    ax.legend(fontsize=7)
    fig.tight_layout()
    fig.savefig(out)
    return out
