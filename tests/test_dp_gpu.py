"""Data-parallel machinery on the GPU (SURVEY.md §4.3 'Distributed tests').  The 2/4/8-GPU
runs are the driver's; here the RCCL code path runs at world size 1 on one MI355X: the
process group (backend 'nccl' = RCCL), async bucketed all-reduces fired between hipGraph
segments, the bf16 wire format, broadcast — and the gradients must equal the plain step."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def rccl_world1(monkeypatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_segmented_step_with_rccl_buckets(rccl_world1, grad_dtype):
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp
    cfg = ExperimentConfig(numLayers=5, channelSize=128, batchSize=8, seed=2)
    data = [torch.from_numpy(a).cuda() for a in random_planes(8, seed=3)]
    ref = HipGoNet(cfg, 8, device="cuda")
    ref.set_batch(*data)
    ref.forward_backward()
    net = HipGoNet(cfg, 8, device="cuda")
    dp.broadcast_(net.params, 0)
    net.refresh_weights()
    net.set_batch(*data)
    lay = net.layout
    ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
    buckets = dp.make_buckets(ranges, 256 * 1024)  # small buckets: several segments
    assert len(buckets) >= 3
    bk = dp.GradBucketer(net.grads, buckets, grad_dtype=grad_dtype)
    step = SegmentedStep(net, bk, use_graphs=True)
    assert len(step.graphs) >= 3
    step.forward_backward()
    torch.cuda.synchronize()
    tol = dict(rtol=1e-5, atol=1e-8) if grad_dtype == "fp32" else dict(rtol=1e-2, atol=1e-5)
    assert torch.allclose(net.grads, ref.grads, **tol)
    # the optimizer graph runs after the all-reduced gradients
    p0 = net.params.clone()
    step.optimizer()
    torch.cuda.synchronize()
    assert not torch.equal(p0, net.params)
    vals = dp.all_reduce_scalars([1.5, 2.0], device="cuda")
    assert vals == [1.5, 2.0]
