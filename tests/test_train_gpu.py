"""Experiment on the HIP backend (graphs, checkpoint/resume, CPU-vs-GPU parity, real data)."""
import os

import numpy as np
import pytest
import torch

from deep_go_amd.config import ExperimentConfig

pytestmark = pytest.mark.gpu

# the reference's bundled data, packed by our t7 reader and committed (tests/fixtures)
FIXTURE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "tests", "fixtures")


def _cfg(tmp_path, **kw):
    base = dict(numLayers=4, channelSize=64, batchSize=32, validationSize=64,
                validation_interval=10, log_interval=5, useCuda=True, synthetic=True,
                checkpoint_dir=str(tmp_path), seed=2, loader_threads=4, prefetch=3)
    base.update(kw)
    return ExperimentConfig(**base)


def test_gpu_experiment_run_and_resume(tmp_path):
    from deep_go_amd.train.experiment import Experiment
    e = Experiment(_cfg(tmp_path), id="g")
    res = e.run(20)
    assert np.isfinite(res["train_cost"]) and len(e.validation_costs) == 2
    p = e.save()
    r = Experiment.load(p)
    r.id = "g2"
    r.run(10)
    assert r.iterations == 30
    assert torch.isfinite(r.backend.net.params).all()


def test_fused_trainer_step_matches_unfused(tmp_path):
    """nan_policy='skip' runs the non-validation iterations as the fused one-graph step
    (forward/backward + SGD + refresh, experiment.py); 'raise' never does.  Same init, same
    data stream across two validation points: the same parameters and validation costs up to
    last-bit reduction-order effects (the graphs differ in stream placement), the same rate
    (read before the step on both paths)."""
    from deep_go_amd.train.experiment import Experiment
    runs = {}
    for pol in ("skip", "raise"):
        e = Experiment(_cfg(tmp_path / pol, nan_policy=pol), id=pol)
        e.run(25)
        runs[pol] = e
    a, b = runs["skip"], runs["raise"]
    assert len(a.validation_costs) == 2
    pa, pb = a.backend.net.params, b.backend.net.params
    assert ((pa - pb).norm() / pb.norm()).item() < 1e-5
    assert a.validation_costs == pytest.approx(b.validation_costs, rel=1e-4)
    assert a.backend.rate == b.backend.rate


def test_gpu_step_matches_cpu_step(tmp_path):
    """One SGD step through the HIP kernels vs the fp32 PyTorch oracle from the same init."""
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.train.backends import CPUBackend, HIPBackend
    cfg = _cfg(tmp_path, rate=0.05, head_relu=False)
    cpu_be = CPUBackend(cfg, 16)
    gpu_be = HIPBackend(cfg, 16, flat=cpu_be.flat_params().clone())
    batch = random_planes(16, seed=4)
    for be in (cpu_be, gpu_be):
        be.set_batch(*batch)
        be.forward_backward()
        be.optimizer_step()
    a = cpu_be.flat_params()
    b = gpu_be.flat_params()
    p0 = CPUBackend(cfg, 16).flat_params()
    da, db = a - p0, b - p0
    rel = (da - db).norm() / da.norm()
    assert rel < 0.05, rel.item()
    assert gpu_be.rate == pytest.approx(cpu_be.rate, rel=1e-12)


def test_real_data_training_reduces_loss(tmp_path):
    from deep_go_amd.train.experiment import Experiment
    cfg = _cfg(tmp_path, synthetic=False, data_root=FIXTURE, numLayers=6, channelSize=64,
               batchSize=64, rate=0.1, head_relu=False, validation_interval=300,
               validationSize=256, log_interval=20)
    # default-experiment.lua shape (6 layers, d=64, B=64). Without the head ReLU the reference
    # rate .512 diverges on this tiny fixture; the tools/real_data_run.py sweep
    # (profiles/r1_real_data_lr_sweep.json) puts 0.1 at val cost ~4.1 after 600 steps.
    e = Experiment(cfg, id="real")
    e.run(600)
    assert e.train_costs[-1] < e.train_costs[0] - 0.3, e.train_costs  # EMA(0.95): lags
    assert e.validation_costs[-1] < 5.0, e.validation_costs
    cost, acc = e.evaluate_split("test", 125)
    assert np.isfinite(cost) and acc > 0.0


def test_200_step_training_curve_matches_fp32_oracle(tmp_path):
    """200 SGD steps on the real fixture from the same init and the same batch stream: the
    HIP trainer (bf16 operands, fp32 master weights, one-graph step) against the fp32
    PyTorch oracle (CPUBackend), rate 0.05.  Stated tolerances: per-step loss within 0.01
    nats at every step (measured max 4.7e-4), the mean loss of each 50-step window within
    0.1% of the oracle's, and the parameter update (p_200 - p_0) within 10% relative norm.
    (At rate 0.1 this tiny fixture's SGD is chaotic — a 1e-5 difference at step 1 grew to
    0.77 nats by step 200 — so the rate is kept in the stable regime.)  The reference's
    semantics: train.lua:4-12, optimizer.lua:16-27."""
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    from deep_go_amd.train.backends import CPUBackend, HIPBackend
    torch.set_num_threads(min(16, os.cpu_count() or 4))
    cfg = _cfg(tmp_path, numLayers=6, channelSize=64, batchSize=32, rate=0.05, rateDecay=1e-4,
               head_relu=False, synthetic=False, data_root=FIXTURE)
    pk = PackedDataset.load(os.path.join(FIXTURE, "train.dgpack.npz"))
    ld = BatchLoader(pk, 32, threads=2, prefetch=3, seed=5, pin=False)
    cpu_be = CPUBackend(cfg, 32)
    p0 = cpu_be.flat_params().clone()
    gpu_be = HIPBackend(cfg, 32, flat=p0.clone())
    lc, lg = [], []
    for _ in range(200):
        batch = ld.next_numpy()
        for be, out in ((cpu_be, lc), (gpu_be, lg)):
            be.set_batch(*batch)
            be.train_step()
            out.append(be.loss_sum() / 32)
    ld.close()
    lc, lg = np.array(lc), np.array(lg)
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/curve_200.json", "w") as f:
        json.dump({"cpu_fp32": lc.tolist(), "hip_bf16": lg.tolist()}, f)
    assert np.isfinite(lg).all()
    assert np.abs(lc - lg).max() < 0.01, np.abs(lc - lg).max()
    for w in range(4):
        a, b = lc[50 * w:50 * (w + 1)].mean(), lg[50 * w:50 * (w + 1)].mean()
        assert abs(a - b) < 1e-3 * a, (w, a, b)
    assert lc[-50:].mean() < lc[:50].mean() - 0.02     # it is learning
    da = cpu_be.flat_params() - p0
    db = gpu_be.flat_params() - p0
    assert ((da - db).norm() / da.norm()).item() < 0.10
    assert gpu_be.rate == pytest.approx(cpu_be.rate, rel=1e-9)


def test_bf16_gradient_wire_world8_memorisation_curve(tmp_path):
    """The data-parallel bf16 gradient wire at WORLD 8, emulated on one GPU, against the fp32
    wire, in a regime with a real learning signal.  Every step's global
    batch of 64 (cycling a 256-position subset of the real fixture: memorisation; 12x128, rate
    0.07, no head ReLU, 1200 steps) is split into 8 rank shards of 8 boards; each shard's backward runs on
    the HIP executor with the global-batch gradient scale, exactly as a rank would.  The bf16
    arm takes each shard's bf16 twin (what the gradient pass 2 writes) and sums them with a
    ring all-reduce's per-hop bf16 rounding (parallel.dp.ring_allreduce_emulate: 7 roundings
    per element — RCCL's worst case); the fp32 arm sums the fp32 shard gradients in fp32 (the
    reference's DataParallelTable reduce).  Both optimizers then run from those reduced
    gradients (the bf16 arm reads the twin, as under DP).  Bounds: every loss finite; both
    arms fall by more than 1 nat; the first 100-step windows agree within 2%; afterwards the
    bf16 arm lags by at most one window (the fp8 stress test's one-sided rule: SGD at this
    rate is chaotic, so the trajectories separate and either may learn faster)."""
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    from deep_go_amd.parallel import dp
    B, R, N, W = 64, 8, 1200, 100
    pk = PackedDataset.load(os.path.join(FIXTURE, "train.dgpack.npz"))
    ld = BatchLoader(pk, B, threads=2, prefetch=4, seed=9, pin=False)
    subset = [[np.asarray(x) for x in ld.next_numpy()] for _ in range(256 // B)]
    ld.close()
    cfg = _cfg(tmp_path, numLayers=12, channelSize=128, batchSize=B, rate=0.07,
               rateDecay=1e-5, head_relu=False, synthetic=False, data_root=FIXTURE, seed=13)
    nets = {w: HipGoNet(cfg, B // R, device="cuda", global_batch=B, grad_wire=w)
            for w in ("fp32", "bf16")}
    nets["bf16"].load_params(nets["fp32"].params.clone())
    steps = {w: SegmentedStep(n, None, use_graphs=True) for w, n in nets.items()}
    lay = nets["fp32"].layout
    buckets = dp.make_buckets([lay.layer_range(i) for i in range(len(lay.layers))],
                              int(cfg.bucket_mb * 2 ** 20), groups=nets["bf16"].wgroups)
    curves = {"fp32": [], "bf16": []}
    for k in range(N):
        bt = subset[k % len(subset)]
        for w, net in nets.items():
            parts, loss = [], 0.0
            for r in range(R):
                sl = slice(r * (B // R), (r + 1) * (B // R))
                net.set_batch(*(torch.from_numpy(x[sl]).cuda() for x in bt))
                steps[w].forward_backward()
                parts.append((net.grads16 if w == "bf16" else net.grads).clone())
                loss += net.loss.sum().item()
            if w == "bf16":
                net.grads16.copy_(dp.ring_allreduce_emulate(parts, buckets))
            else:
                net.grads.copy_(dp.ring_allreduce_emulate(parts, buckets, wire=torch.float32))
            steps[w].optimizer()
            curves[w].append(loss / B)
    l32, l16 = np.array(curves["fp32"]), np.array(curves["bf16"])
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/curve_world8_bf16_wire.json", "w") as f:
        json.dump({"fp32_wire": l32.tolist(), "bf16_wire_world8": l16.tolist()}, f)
    assert np.isfinite(l16).all() and np.isfinite(l32).all()
    assert l32[-W:].mean() < l32[:W].mean() - 1.0, (l32[:W].mean(), l32[-W:].mean())
    assert l16[-W:].mean() < l16[:W].mean() - 1.0, (l16[:W].mean(), l16[-W:].mean())
    assert abs(l16[:W].mean() - l32[:W].mean()) < 0.02 * l32[:W].mean()
    for w in range(W, N, W):
        m32, m16 = l32[w:w + W].mean(), l16[w:w + W].mean()
        ref = max(m32, l32[w - W:w].mean())
        assert m16 < ref + max(0.15, 0.10 * ref), (w, m32, m16)


@pytest.mark.parametrize("ch", [128, 256])
def test_fp8_stress_vs_bf16_memorisation(tmp_path, ch):
    """Mixed-precision stress of the whole fp8 path (e4m3 forward stack, e5m2 backward-data
    stack, MX-fp8 weight gradients, delayed power-of-two scaling) against bf16 from the same
    init on the same batch stream, in a regime with a real learning signal: 1200 SGD steps
    cycling a 256-position subset of the real fixture (memorisation; 12 x ch, batch 64,
    rate 0.07, no head ReLU: both fall from 5.9 nats to ~0 — rate 0.1 sits on the edge of
    stability, where one fp8 run of six diverged, tools/fp8_memo.py).  Bounds: every loss finite; bf16
    AND fp8 each drop by more than 1 nat; fp8 lags bf16 by at most one 100-step window: in
    every window its mean loss is no worse than the better of bf16's same and previous window
    by more than 0.15 nats or 10% (one-sided, with a lag: the loss collapses within ~200
    steps and SGD at this rate is chaotic, so the trajectories separate and either may
    learn faster — with nearest-even e5m2 gradients fp8 stalled near 5.3 nats while bf16
    reached 2.7, tools/fp8_memo.py; stochastic rounding fixed it); fewer than 1%
    saturation events (a layer-step whose observed amax exceeded the range of the delayed
    scale) over the weight + activation tensors, and separately over the e5m2 gradients.
    (BASELINE config 5 is 12x256; the 12x128 fp8 secondary is checked the same way.)"""
    import json
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    from deep_go_amd.train.backends import HIPBackend
    B, N, W = 64, 1200, 100
    pk = PackedDataset.load(os.path.join(FIXTURE, "train.dgpack.npz"))
    ld = BatchLoader(pk, B, threads=2, prefetch=4, seed=9, pin=False)
    subset = [ld.next_numpy() for _ in range(256 // B)]
    ld.close()
    losses, sat = {}, None
    flat0 = None
    for dt in ("bf16", "fp8"):
        cfg = _cfg(tmp_path, numLayers=12, channelSize=ch, batchSize=B, rate=0.07,
                   rateDecay=1e-5, head_relu=False, synthetic=False, data_root=FIXTURE,
                   dtype=dt, seed=13)
        be = HIPBackend(cfg, B, flat=flat0)
        if flat0 is None:
            flat0 = be.flat_params().clone()
        out = []
        for k in range(N):
            be.set_batch(*subset[k % len(subset)])
            be.train_step()
            out.append(be.loss_sum() / B)
        losses[dt] = np.array(out)
        if dt == "fp8":
            assert be.net.stack_fp8 and be.net.win8_groups
            sat = be.net.fp8_sat.cpu().numpy()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/fp8_stress_memo_12x{ch}.json", "w") as f:
        json.dump({k: v.tolist() for k, v in losses.items()} | {"sat": sat.tolist()}, f)
    lb, l8 = losses["bf16"], losses["fp8"]
    assert np.isfinite(lb).all() and np.isfinite(l8).all()
    assert lb[-W:].mean() < lb[:W].mean() - 1.0, (lb[:W].mean(), lb[-W:].mean())
    assert l8[-W:].mean() < l8[:W].mean() - 1.0, (l8[:W].mean(), l8[-W:].mean())
    for w in range(0, N, W):
        mb, m8 = lb[w:w + W].mean(), l8[w:w + W].mean()
        prev = lb[max(0, w - W):max(W, w)].mean()
        ref = max(mb, prev)
        assert m8 < ref + max(0.15, 0.10 * ref), (w, mb, prev, m8)
    L = sat.size // 3
    wa, g = sat[:2 * L], sat[2 * L:]        # weights + activations | e5m2 gradients
    assert wa.sum() < 0.01 * N * wa.size, sat
    assert g.sum() < 0.01 * N * g.size, sat


@pytest.mark.timeout(300)
def test_accuracy_half_matches_fp32_oracle_with_head_relu():
    """The metric's accuracy half through the HIP trainer against the fp32 PyTorch oracle
    (VERDICT r5 item 5), at the reference's default-experiment shape WITH its head ReLU
    (default-experiment.lua: 6 layers, d = 64, batch 64; experiments.lua:133-153): HIPBackend
    and CPUBackend from the same init on the same game-uniform batch stream of the fixture's
    training games, 500 SGD steps at rate 0.05 (where this shape learns with the head ReLU:
    tools/acc_sweep.py; the reference's own .512 pins the loss at ln 361), then both scored
    on EVERY held-out validation (134) and test (125) position and on the 4139 training
    positions (train.lua:14-45).

    SGD here is chaotic once the network leaves the ln 361 plateau (~step 250): two fp32
    oracle runs whose inits differ by a relative 1e-5 separate by 0.1-0.4 nats per step and
    end 2-5 validation positions apart (profiles/r6_accuracy_parity.txt).  So the
    tolerances are stated against the oracle's own sensitivity, measured in the same test
    (oracle runs from the init perturbed by 1e-5 and 1e-3):
      * before the plateau escape the curves agree: |loss difference| < 1e-3 nats on every
        one of the first 150 steps (measured <= 7e-5);
      * both learn: the training loss falls by more than 1 nat;
      * per split, the HIP run is no further from the oracle than the perturbed oracle runs
        are, plus 2 positions (held-out games; train: + 0.5% of 4139) in top-1, and plus 1%
        of the oracle's NLL in NLL.
    Paper-level top-1 stays parity unpinned (one held-out game per split)."""
    from deep_go_amd.train.accuracy import oracle_parity
    r = oracle_parity(torch.device("cuda", 0), layers=6, channels=64, batch=64, rate=0.05,
                      steps=500, head_relu=True, seed=5, perturb=(1e-5, 1e-3))
    assert r is not None, "packed fixture missing"
    import json
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/accuracy_parity_6x64_relu.json", "w") as f:
        json.dump(r, f)
    lc, lg = np.array(r["loss_cpu"]), np.array(r["loss_hip"])
    assert np.isfinite(lg).all()
    assert np.abs(lc[:150] - lg[:150]).max() < 1e-3, np.abs(lc[:150] - lg[:150]).max()
    assert lc[-50:].mean() < lc[:50].mean() - 1.0, (lc[:50].mean(), lc[-50:].mean())
    assert lg[-50:].mean() < lg[:50].mean() - 1.0, (lg[:50].mean(), lg[-50:].mean())
    pert = [n for n in r["runs"] if n.startswith("cpu~")]
    for split in ("validation", "test", "train"):
        sc = r[split]
        c, g = sc["cpu"], sc["hip"]
        env_top1 = max(abs(sc[n]["correct"] - c["correct"]) for n in pert)
        env_nll = max(abs(sc[n]["nll"] - c["nll"]) for n in pert)
        slack = 2 if split != "train" else int(0.005 * c["positions"])
        assert abs(g["correct"] - c["correct"]) <= env_top1 + slack, (split, sc)
        assert abs(g["nll"] - c["nll"]) <= env_nll + 0.01 * c["nll"], (split, sc)


@pytest.mark.parametrize("shape", [(6, 64), (12, 128)])
def test_hip_training_is_bit_reproducible(shape):
    """Two HIP trainer runs from the same init on the same batch stream end with bit-identical
    parameters and losses (every reduction has a fixed order: split-K slabs, bias partials,
    head reduce, the standalone head's per-board weight gradient — whose LDS atomicAdd over
    the waves made d = 64 runs differ in the last bits, found by the accuracy-half parity runs
    in round 6).  With the head ReLU (the reference's), 60 steps."""
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    from deep_go_amd.train.backends import HIPBackend
    L, C = shape
    B = 32
    pk = PackedDataset.load(os.path.join(FIXTURE, "train.dgpack.npz"))
    ld = BatchLoader(pk, B, threads=2, prefetch=3, seed=21, pin=False)
    batches = [ld.next_numpy() for _ in range(60)]
    ld.close()
    cfg = ExperimentConfig(numLayers=L, channelSize=C, batchSize=B, rate=0.05, seed=8,
                           head_relu=True, useCuda=True)
    out = []
    for _ in range(2):
        be = HIPBackend(cfg, B)
        losses = []
        for bt in batches:
            be.set_batch(*bt)
            be.train_step()
            losses.append(be.loss_sum())
        out.append((be.flat_params().clone(), losses))
        del be
    assert out[0][1] == out[1][1]
    assert torch.equal(out[0][0], out[1][0])
