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


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16", "bf16-direct"])
def test_segmented_step_with_rccl_buckets(rccl_world1, grad_dtype):
    """Graph segments between bucket all-reduces (world 1); bf16 wire through a private
    shadow (copies around the collective) or directly on the model's bf16 twin, which the
    gradient reduce kernels write and the optimizer reads (no conversion kernels)."""
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp
    cfg = ExperimentConfig(numLayers=5, channelSize=128, batchSize=8, seed=2)
    data = [torch.from_numpy(a).cuda() for a in random_planes(8, seed=3)]
    ref = HipGoNet(cfg, 8, device="cuda")
    ref.set_batch(*data)
    ref.forward_backward()
    direct = grad_dtype == "bf16-direct"
    net = HipGoNet(cfg, 8, device="cuda", grad_wire="bf16" if direct else "fp32")
    dp.broadcast_(net.params, 0)
    net.refresh_weights()
    net.set_batch(*data)
    lay = net.layout
    ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
    buckets = dp.make_buckets(ranges, 256 * 1024)  # small buckets: several segments
    assert len(buckets) >= 3
    bk = dp.GradBucketer(net.grads, buckets, grad_dtype="bf16" if direct else grad_dtype,
                         shadow=net.grads16)
    assert bk.direct == direct
    step = SegmentedStep(net, bk, use_graphs=True)
    assert len(step.graphs) >= 3
    step.forward_backward()
    torch.cuda.synchronize()
    tol = dict(rtol=1e-5, atol=1e-8) if grad_dtype == "fp32" else dict(rtol=1e-2, atol=1e-5)
    assert torch.allclose(net.grads, ref.grads, **tol)
    if direct:   # the twin is the fp32 gradient rounded once (world 1: the sum of one)
        assert torch.equal(net.grads16, ref.grads.to(torch.bfloat16))
    # the optimizer graph runs after the all-reduced gradients
    p0 = net.params.clone()
    lr = net.lr.item()
    step.optimizer()
    torch.cuda.synchronize()
    assert not torch.equal(p0, net.params)
    if direct:   # SGD read the bf16 twin
        want = p0 - torch.tensor(lr, dtype=torch.float32) * net.grads16.float()
        assert torch.allclose(net.params, want, rtol=1e-6, atol=1e-9)
    vals = dp.all_reduce_scalars([1.5, 2.0], device="cuda")
    assert vals == [1.5, 2.0]


def _gpu_dp_worker(rank, world, port, B, out_path, layers, bucket_kb, wire="fp32"):
    """One rank of a multi-process DP step on the HIP executor; all ranks share cuda:0 and
    all-reduce over gloo (RCCL needs one GPU per rank): the segmented-graph / bucket /
    global-batch-scaling logic is the same code path the 8-GPU RCCL run takes."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from deep_go_amd.config import ExperimentConfig
        from deep_go_amd.data.synthetic import random_planes
        from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
        from deep_go_amd.parallel import dp
        torch.cuda.set_device(0)
        cfg = ExperimentConfig(numLayers=layers, channelSize=128, batchSize=B, seed=21)
        Bl = B // world
        net = HipGoNet(cfg, Bl, device="cuda", global_batch=B, grad_wire=wire)
        if rank != 0:
            net.params.mul_(0.5)  # must be overwritten by the broadcast from rank 0
        dp.broadcast_(net.params, 0)
        net.refresh_weights()
        planes, player, rank_, labels = random_planes(B, seed=22)
        sl = slice(rank * Bl, (rank + 1) * Bl)
        net.set_batch(*(torch.from_numpy(a[sl]).cuda() for a in (planes, player, rank_, labels)))
        lay = net.layout
        ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
        # wire bf16: the trainer's / bench's default DP path — the gradient pass 2 writes the
        # bf16 twin and the buckets are all-reduced ON it (shadow = the twin, no copies)
        bk = dp.GradBucketer(net.grads, dp.make_buckets(ranges, bucket_kb * 1024,
                                                        groups=net.wgroups),
                             grad_dtype=wire, shadow=net.grads16)
        assert bk.direct == (wire == "bf16")
        step = SegmentedStep(net, bk, use_graphs=True)
        step.forward_backward()
        torch.cuda.synchronize()
        if rank == 0:
            g = net.grads16.float() if wire == "bf16" else net.grads
            torch.save({"grads": g.cpu(), "nbuckets": len(bk.buckets),
                        "groups": net.wgroups}, out_path)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,wire", [(2, "fp32"), (4, "fp32"), (2, "bf16"), (4, "bf16")])
def test_multirank_dp_step_matches_single_process(world, wire, tmp_path):
    """DP=k over k processes (per-rank batch B/k, grouped wgrads, segmented graphs, bucketed
    all-reduce) gives the gradients of one process with the whole batch B.  wire bf16 is the
    default DP path (bf16 twin all-reduced directly): within the bf16 wire tolerance of the
    fp32 single-process gradient (k-1 rounded partial sums + the twins' own rounding;
    tests/test_wire_cpu.py bounds the same at world 8)."""
    import torch.multiprocessing as mp
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet
    B, layers = 8, 9
    out = str(tmp_path / "g.pt")
    mp.spawn(_gpu_dp_worker, args=(world, _free_port(), B, out, layers, 600, wire),
             nprocs=world, join=True)
    res = torch.load(out, weights_only=True)
    assert res["nbuckets"] >= 2 and res["groups"]
    cfg = ExperimentConfig(numLayers=layers, channelSize=128, batchSize=B, seed=21)
    ref = HipGoNet(cfg, B, device="cuda")
    ref.set_batch(*(torch.from_numpy(a).cuda() for a in random_planes(B, seed=22)))
    ref.forward_backward()
    torch.cuda.synchronize()
    g = res["grads"].cuda()
    err = (g - ref.grads).norm() / ref.grads.norm()
    assert err < (1e-5 if wire == "fp32" else 1e-2), err.item()


@pytest.mark.parametrize("grad_dtype", ["fp32", "bf16"])
def test_native_comm_one_graph_dp_step(grad_dtype):
    """Native RCCL communicator (csrc/comm/comm.cpp) at world 1: its all-reduces captured
    INSIDE the one-graph DP step (mode dp-graph) give the plain step's gradients; the
    optimizer runs after the join; async_error() reports a healthy communicator."""
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp
    comm = dp.make_communicator("native", "cuda:0")
    assert comm.kind == "native" and comm.world == 1
    dp.selftest_in_graph(comm)
    cfg = ExperimentConfig(numLayers=8, channelSize=128, batchSize=8, seed=2)
    data = [torch.from_numpy(a).cuda() for a in random_planes(8, seed=3)]
    ref = HipGoNet(cfg, 8, device="cuda")
    ref.set_batch(*data)
    ref.forward_backward()
    ref_opt = HipGoNet(cfg, 8, device="cuda")
    ref_opt.set_batch(*data)
    ref_opt.train_step()
    net = HipGoNet(cfg, 8, device="cuda")
    net.set_batch(*data)
    lay = net.layout
    ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
    bk = dp.GradBucketer(net.grads, dp.make_buckets(ranges, 256 * 1024, groups=net.wgroups),
                         grad_dtype=grad_dtype, comm=comm)
    step = SegmentedStep(net, bk, use_graphs=True)
    assert step.mode == "dp-graph" and len(bk.buckets) >= 2
    p0 = net.params.clone()
    step.forward_backward()
    torch.cuda.synchronize()
    tol = dict(rtol=1e-5, atol=1e-8) if grad_dtype == "fp32" else dict(rtol=1e-2, atol=1e-5)
    assert torch.allclose(net.grads, ref.grads, **tol)
    net.params.copy_(p0)
    net.lr.fill_(cfg.rate)
    step()                               # full graph: fwd/bwd + collectives + optimizer
    torch.cuda.synchronize()
    ptol = dict(rtol=1e-6, atol=1e-7) if grad_dtype == "fp32" else dict(rtol=1e-4, atol=1e-6)
    assert torch.allclose(net.params, ref_opt.params, **ptol)
    assert comm.async_error() == ""
    comm.close()
