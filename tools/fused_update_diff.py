"""Which parameters differ between the fused update (grad_update) and the separate SGD +
refresh launches after ONE step (diagnostic for tests/test_model_gpu.py
test_fused_update_matches_separate_launches).  Usage: python tools/fused_update_diff.py L C"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    nets = []
    for fused in ("0", "1"):
        os.environ["DG_FUSED_UPDATE"] = fused
        cfg = ExperimentConfig(numLayers=L, channelSize=C, batchSize=4, seed=2, rateDecay=1e-3)
        net = HipGoNet(cfg, 4, device="cuda")
        pl, py_, rk, lb = random_planes(4, seed=9)
        net.set_batch(*(torch.from_numpy(x).cuda() for x in (pl, py_, rk, lb)))
        net.train_step()
        torch.cuda.synchronize()
        nets.append(net)
    a, b = nets
    print("grads equal", torch.equal(a.grads, b.grads))
    for name, off, n in a.layout.tensor_ranges():
        pa, pb = a.params[off:off + n], b.params[off:off + n]
        d = (pa != pb).nonzero().flatten()
        if d.numel():
            i = int(d[0])
            print(f"{name}: {d.numel()}/{n} differ; first at {i}: {pa[i].item()!r} vs "
                  f"{pb[i].item()!r}; grad {a.grads[off + i].item()!r} {b.grads[off + i].item()!r}")
    print("lr", a.lr.item(), b.lr.item())


if __name__ == "__main__":
    main()
