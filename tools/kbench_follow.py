"""Kernel bench of the bias-gradient follower beside the backward-data stack (12x128, B=256).

  python tools/kbench_follow.py [--reps 20]

Times (us, median of --reps, CUDA events): the dgrad stack alone (plain stores), the stack
with the arrival counters (SIG: write-through stores + per-row signals) alone, the follower
alone on ready frames (counters preset), the finish pass computing every task alone, the
previous multi-layer partials launch alone, and the stack + follower concurrently (stack
time on the main stream, the pair's wall time, the follower's own span) for each load cache
policy (0 default, 2 nt, 16 sc1) and poll interval of the follower.  Prints one JSON line."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch
    os.environ["DG_BIAS_FOLLOW"] = "1"
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet
    cfg = ExperimentConfig(numLayers=12, channelSize=128, batchSize=256, seed=7)
    net = HipGoNet(cfg, 256, device="cuda")
    net.set_batch(*[torch.from_numpy(x).cuda() for x in random_planes(256, seed=3)])
    net.forward_backward()
    torch.cuda.synchronize()
    h = net.h
    main_s = torch.cuda.current_stream()
    side = net.side
    (_, sig_args), = [op for op in net._bwd_pre if op[0] is h.conv_stack2_dgrad_sig]
    table, nl, X0, B, sig = sig_args
    f_follow, f_args = net._bf_follow
    _, fin_args = net._bf_finish
    old_op = None
    g = net.wgroups[0]

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        return e

    def timed(fn, reps=a.reps):
        ts = []
        for _ in range(reps + 2):
            e0, e1 = ev(), ev()
            e0.record(main_s)
            fn()
            e1.record(main_s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return round(float(np.median(ts[2:])), 1)

    def reset():
        net._bf_sig.zero_()
        net._bf_done.zero_()

    s = main_s.cuda_stream
    out = {}
    out["stack_plain"] = timed(lambda: h.conv_stack2(h.EPI_DGRAD, table, nl, X0, 0, B, s))

    def stack_sig():
        reset()
        h.conv_stack2_dgrad_sig(table, nl, X0, B, sig, s)
    out["stack_sig_alone(+reset)"] = timed(stack_sig)
    out["reset_only"] = timed(reset)

    def follower_ready():
        reset()
        net._bf_sig.fill_(B)
        f_follow(*f_args, s)
    out["follower_ready_alone(+reset)"] = timed(follower_ready)

    def finish_all():
        reset()
        f_follow(*fin_args, s)
    out["finish_all_tasks(+reset)"] = timed(finish_all)
    # the previous partials launch (DG_BIAS_FOLLOW=0's op)
    bt = net._bf_table
    old_tab = np.ascontiguousarray(np.array([[int(r[0]), int(r[1]), 0] for r in bt], dtype=np.int64))
    out["old_partials_alone"] = timed(lambda: h.bias_grad_partial_multi(
        old_tab.ctypes.data, len(old_tab), B, 128, 1, 0, s))

    for aux in (0, 2, 16):
        for slp in (1, 4, 16):
            h.bias_follow_set_variant(aux, slp)
            spans = []

            def pair():
                reset()
                side.wait_stream(main_s)
                ef0, ef1 = ev(), ev()
                ef0.record(side)
                f_follow(*f_args, side.cuda_stream)
                ef1.record(side)
                es0, es1 = ev(), ev()
                es0.record(main_s)
                h.conv_stack2_dgrad_sig(table, nl, X0, B, sig, s)
                es1.record(main_s)
                main_s.wait_stream(side)
                f_follow(*fin_args, s)
                spans.append((ef0, ef1, es0, es1))
            wall = timed(pair)
            torch.cuda.synchronize()
            st = float(np.median([x[2].elapsed_time(x[3]) * 1e3 for x in spans[2:]]))
            fo = float(np.median([x[0].elapsed_time(x[1]) * 1e3 for x in spans[2:]]))
            out[f"pair_aux{aux}_sleep{slp}"] = {"wall(+reset+finish)": wall, "stack": round(st, 1),
                                               "follower": round(fo, 1)}
    h.bias_follow_set_variant(0, 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
