"""A few training steps of one configuration, for the stream-ordering checks
(tests/test_model_gpu.py::test_stream_handoffs_checked_and_serialized_run_bit_identical).

  python tools/stream_check_run.py OUT.pt [--channels 128] [--dtype bf16] [--steps 3]
                                          [--batch 32] [--mode eager|graph] [--dp]

Runs the fused training step (``SegmentedStep``; ``--dp``: the data-parallel step with the
native RCCL communicator at world 1, buckets on the comm stream) and saves the parameters,
the step's last loss vector and how many cross-stream hand-offs ``DG_CHECK_STREAMS=1``
verified.  The test runs it under DG_CHECK_STREAMS=1, under AMD_SERIALIZE_KERNEL=3 (every
kernel serialized: no two streams overlap) and plainly, and compares the outputs bit for bit.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--layers", type=int, default=12)
    ap.add_argument("--mode", default="eager", choices=["eager", "graph"])
    ap.add_argument("--dp", action="store_true")
    a = ap.parse_args()
    import torch
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp
    cfg = ExperimentConfig(numLayers=a.layers, channelSize=a.channels, batchSize=a.batch,
                           seed=3, dtype=a.dtype, rate=0.05)
    wire = "bf16" if a.dp else "fp32"
    net = HipGoNet(cfg, a.batch, device="cuda", grad_wire=wire)
    bk = None
    comm = None
    if a.dp:
        comm = dp.make_communicator("native", "cuda:0")
        lay = net.layout
        bk = dp.GradBucketer(net.grads, dp.make_buckets(
            [lay.layer_range(i) for i in range(len(lay.layers))], 1 << 20, groups=net.wgroups),
            grad_dtype=wire, comm=comm, shadow=net.grads16)
    batches = [[torch.from_numpy(x).cuda() for x in random_planes(a.batch, seed=40 + k)]
               for k in range(a.steps)]
    net.set_batch(*batches[0])
    step = SegmentedStep(net, bk, use_graphs=a.mode == "graph")
    for k in range(a.steps):
        net.set_batch(*batches[k])
        step()
        net.check_streams()
    torch.cuda.synchronize()
    torch.save({"params": net.params.cpu(), "loss": net.loss.cpu(),
                "checked": net.sc.checked if net.sc else 0, "mode": step.mode}, a.out)
    if comm is not None:
        comm.close()


if __name__ == "__main__":
    main()
