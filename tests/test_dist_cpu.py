"""Data parallelism without a cluster (SURVEY.md §4.3 'Distributed tests'):

(a) DP=k with per-rank batch B/k gives the same update as DP=1 with batch B;
(b) a CPU gloo world exercises the bucketing / async all-reduce logic;
(c) the bucket scheduler is unit-tested without any communicator."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from deep_go_amd.config import ExperimentConfig
from deep_go_amd.parallel.dp import GradBucketer, make_buckets


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_make_buckets_keeps_groups_whole():
    """Layers whose gradients become final together (a grouped wgrad launch) stay in one
    bucket, which is ready at the group's top layer."""
    ranges = [(0, 100), (100, 200), (200, 300), (300, 400), (400, 500), (500, 520)]
    b = make_buckets(ranges, bucket_bytes=4 * 150, groups=[[4, 3, 2]])
    # walk: layer 5 (20 elems), group 2..4 (300) -> bucket [200, 520) ready at 4; then 1, 0
    assert b[0] == (200, 520, 4)
    assert b[1] == (0, 200, 0)
    assert sum(e - s for s, e, _ in b) == 520
    # without groups: plain per-layer walk
    b2 = make_buckets(ranges, bucket_bytes=4 * 150)
    assert b2[0] == (300, 520, 3)


def test_make_buckets_reverse_order_and_sizes():
    ranges = [(0, 100), (100, 300), (300, 350), (350, 1000)]
    b = make_buckets(ranges, bucket_bytes=4 * 250)
    # walk from the last layer: [350,1000) fills a bucket; then [100,350) (2 layers) ...
    assert b[0] == (350, 1000, 3)
    assert b[1] == (100, 350, 1)
    assert b[-1][0] == 0 and b[-1][2] == 0
    covered = sorted((s, e) for s, e, _ in b)
    assert covered[0][0] == 0 and covered[-1][1] == 1000
    assert all(covered[i][1] == covered[i + 1][0] for i in range(len(covered) - 1))


def _data(B, seed=0):
    from deep_go_amd.data.synthetic import random_planes
    return random_planes(B, seed=seed)


def _dp_worker(rank, world, port, B, out_path, grad_dtype):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deep_go_amd.models.gocnn import ParamLayout
    from deep_go_amd.train.backends import CPUBackend
    cfg = ExperimentConfig(numLayers=3, channelSize=16, rate=0.1, seed=5, bucket_mb=0.01)
    be = CPUBackend(cfg, B // world, world=world, bucket_mb=0.01)
    planes, player, rank_, labels = _data(B)
    sl = slice(rank * (B // world), (rank + 1) * (B // world))
    for step in range(3):
        be.set_batch(planes[sl], player[sl], rank_[sl], labels[sl])
        be.forward_backward()
        be.optimizer_step()
    # GradBucketer (async buckets + optional bf16 wire format) on the same world
    g = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    bk = GradBucketer(g, make_buckets([(0, 400), (400, 1000)], 4 * 300), grad_dtype=grad_dtype)
    for i in range(len(bk.buckets)):
        bk.fire(i)
    bk.wait()
    if rank == 0:
        torch.save({"params": be.flat_params().clone(), "g": g.clone()}, out_path)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,grad_dtype", [(2, "fp32"), (2, "bf16"), (4, "fp32"),
                                              (8, "fp32")])
def test_dp_equals_dp1(tmp_path, world, grad_dtype):
    """DP=k with per-rank batch B/k gives the update of DP=1 with batch B
    (world 2, 4 and 8 gloo ranks on the CPU; 8 = one rank per MI355X of a node)."""
    B = 8
    outk = str(tmp_path / f"dp{world}.pt")
    mp.spawn(_dp_worker, args=(world, _free_port(), B, outk, grad_dtype), nprocs=world,
             join=True)
    out1 = str(tmp_path / "dp1.pt")
    mp.spawn(_dp_worker, args=(1, _free_port(), B, out1, grad_dtype), nprocs=1, join=True)
    a = torch.load(outk, weights_only=True)
    b = torch.load(out1, weights_only=True)
    assert torch.allclose(a["params"], b["params"], atol=1e-6, rtol=1e-5)
    # sum over ranks of (rank + 1) * i
    ref = torch.arange(1000, dtype=torch.float32) * (world * (world + 1) // 2)
    if grad_dtype == "fp32":
        assert torch.equal(a["g"], ref)
    else:
        assert torch.allclose(a["g"], ref, rtol=1e-2)


def _exp_worker(rank, world, port, ref_data, ckdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from deep_go_amd.train.experiment import Experiment
    cfg = ExperimentConfig(numLayers=2, channelSize=16, batchSize=4, validationSize=12,
                           validation_interval=3, log_interval=3, useCuda=False,
                           data_root=ref_data, checkpoint_dir=ckdir, loader_threads=1,
                           prefetch=2, seed=1)
    e = Experiment(cfg, id="dist")
    res = e.run(6)
    assert e.iterations == 6 and len(e.validation_costs) == 2
    dist.barrier()
    dist.destroy_process_group()


def test_experiment_runs_under_gloo_world2(tmp_path, ref_data):
    mp.spawn(_exp_worker, args=(2, _free_port(), ref_data, str(tmp_path)), nprocs=2, join=True)
    assert os.path.exists(tmp_path / "dist.model")  # rank 0 checkpoint only


# ---------------------------------------------------------------- native communicator set-up
class _StubDgcomm:
    """Stands in for the ``_dgcomm`` module (csrc/comm/comm.cpp) on the CPU: unique ids are
    random bytes, ``Comm`` records what it was built with."""
    aborted = []

    @staticmethod
    def unique_id():
        return os.urandom(128)

    @staticmethod
    def version():
        return 21801

    class Comm:
        def __init__(self, uid, world, rank, device):
            self.uid, self.world, self.rank, self.device = uid, world, rank, device

        def abort(self):
            _StubDgcomm.aborted.append(self.rank)


def _native_worker(rank, world, port, out_path, mode):
    import json
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from deep_go_amd.parallel import dp

    def load():
        if mode == "no-module" and rank == 1:
            raise ImportError("_dgcomm missing on this rank")
        return _StubDgcomm

    def selftest(c):
        if mode == "bad-selftest" and rank == 1:
            raise RuntimeError("native all-reduce self-test: wrong in-graph sum")

    factory = lambda mod: dp.NativeComm("cpu", mod=mod, stream="comm-stream")  # noqa: E731
    made = []

    def counting_factory(mod):
        made.append(1)
        return factory(mod)
    comms = [dp.make_communicator("auto", "cpu", selftest=selftest, load_module=load,
                                  native_factory=counting_factory) for _ in range(2)]
    rec = {"kinds": [c.kind for c in comms], "made": len(made),
           "aborted": list(_StubDgcomm.aborted),
           "uids": [c.uid.hex() if c.kind == "native" else None for c in comms],
           "keys": [getattr(c, "key", None) for c in comms]}
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(rec, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["ok", "bad-selftest", "no-module"])
def test_native_comm_rendezvous_and_collective_fallback(tmp_path, mode):
    """World 2 over gloo with a stub _dgcomm: every rank's n-th communicator meets under the
    same store key and gets rank 0's unique id; if ANY rank fails its module load or
    self-test, EVERY rank falls back to torch.distributed (and the ranks whose native
    communicator came up abort it) — never a split decision."""
    import json
    out = str(tmp_path / "rec")
    mp.spawn(_native_worker, args=(2, _free_port(), out, mode), nprocs=2, join=True)
    recs = [json.load(open(f"{out}.{r}")) for r in (0, 1)]
    if mode == "ok":
        for r in recs:
            assert r["kinds"] == ["native", "native"]
            assert r["keys"] == ["dg_rccl_uid_0", "dg_rccl_uid_1"]
        assert recs[0]["uids"] == recs[1]["uids"]          # rank 0's id reached rank 1
        assert recs[0]["uids"][0] != recs[0]["uids"][1]    # a fresh id per communicator
    else:
        for r in recs:
            assert r["kinds"] == ["torch", "torch"]
        if mode == "bad-selftest":
            # both ranks built a native comm (init is collective); both aborted it
            assert recs[0]["made"] == recs[1]["made"] == 2
            assert recs[0]["aborted"] == [0, 0] and recs[1]["aborted"] == [1, 1]
        else:
            # agreed BEFORE the collective init: no rank entered ncclCommInitRank
            assert recs[0]["made"] == recs[1]["made"] == 0
