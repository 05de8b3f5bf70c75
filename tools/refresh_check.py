"""Which plain (non-fragment) weight copies the per-step refresh keeps, per layer, for the
bench configs (HipGoNet._step_refresh_table).  Usage: python tools/refresh_check.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from deep_go_amd.config import get_preset  # noqa: E402
from deep_go_amd.models.hip_model import HipGoNet  # noqa: E402


def main():
    for ch, dt in ((128, "bf16"), (256, "bf16"), (256, "fp8")):
        cfg = get_preset("12x128-bf16", numLayers=12, channelSize=ch, batchSize=256, dtype=dt)
        net = HipGoNet(cfg, 256, device="cuda")
        full, step = net._refresh_table, net._step_refresh_table()
        names = {1: "wf", 2: "wd", 10: "wf8", 16: "wf_frag", 17: "wd_frag", 18: "wf8_frag",
                 19: "wd8_frag"}
        for i in range(len(full)):
            kept = [n for c, n in names.items() if step[i, c]]
            dropped = [n for c, n in names.items() if full[i, c] and not step[i, c]]
            print(f"{ch} {dt} layer {i}: kept {kept} dropped {dropped}", flush=True)
        del net
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
