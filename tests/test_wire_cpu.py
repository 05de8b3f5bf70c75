"""The data-parallel bf16 gradient wire at world 8, bounded on the CPU.

Under DP every rank's gradient pass 2 writes a bf16 twin of its gradient and the bucket
all-reduces sum those twins on the wire; RCCL's reduction kernels round every partial sum
back to bf16, so an 8-rank ring rounds each element up to 7 times (plus the twin's own
rounding).  The reference reduces fp32 gradients (``/root/reference/experiments.lua:155-168``).
These tests take REAL per-rank gradients — the fp32 oracle model on eight different
game-uniform shards of the reference's bundled training games — emulate the ring's per-hop
rounding (``parallel.dp.ring_allreduce_emulate``), and bound the result against the fp32 sum
three ways:
  * elementwise, by the recursive-summation theorem (gamma_7 * sum |twin_i|);
  * normwise, by an absolute relative-error budget;
  * against the sampling noise of the global-batch gradient itself (the error a different
    draw of the same-size batch makes), which the wire error must be far below.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from deep_go_amd.config import ExperimentConfig
from deep_go_amd.parallel import dp

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures")
WORLD = 8


def _rank_gradients(cfg, per_rank, seed):
    """fp32 gradients of the mean-NLL over the global batch (WORLD x per_rank boards), one per
    rank (each rank's share of the sum, as the HIP head scales by 1 / global batch)."""
    from deep_go_amd.data.dataset import PackedDataset, sample_reference
    from deep_go_amd.models.gocnn import ParamLayout, init_params, reference_forward
    from deep_go_amd.ops.native import cpu
    pk = PackedDataset.load(os.path.join(FIXTURE, "train.dgpack.npz"))
    rng = np.random.default_rng(seed)
    g, mv = sample_reference(list(pk.game_count), WORLD * per_rank, rng)
    idx = pk.game_start[g] + mv - 1
    lay = ParamLayout(cfg)
    flat = init_params(lay, cfg.seed)
    x = torch.from_numpy(cpu().expand(pk.planes[idx], pk.player[idx], pk.rank[idx], False))
    y = torch.from_numpy(pk.label[idx].astype(np.int64))
    grads = []
    for r in range(WORLD):
        sl = slice(r * per_rank, (r + 1) * per_rank)
        p = flat.clone().requires_grad_(True)
        logp = reference_forward(lay, p, x[sl], head_relu=cfg.head_relu)
        loss = F.nll_loss(logp, y[sl], reduction="sum") / (WORLD * per_rank)
        loss.backward()
        grads.append(p.grad.detach().clone())
    return lay, grads


@pytest.fixture(scope="module")
def world8_grads():
    torch.manual_seed(0)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    # default-experiment shape (default-experiment.lua:16-19: 6 layers, d = 64), the
    # reference's own architecture; 8 ranks x 8 boards
    cfg = ExperimentConfig(numLayers=6, channelSize=64, head_relu=False, seed=5)
    return _rank_gradients(cfg, per_rank=8, seed=17)


def test_ring_emulation_matches_exact_sum_at_world_1_and_fp32():
    """The emulator itself: one rank is the identity; an fp32 wire sums to fp32 precision."""
    x = [torch.randn(1000, dtype=torch.float64) for _ in range(4)]
    one = dp.ring_allreduce_emulate([x[0]], wire=torch.bfloat16)
    assert torch.equal(one, x[0].to(torch.bfloat16))
    s32 = dp.ring_allreduce_emulate(x, wire=torch.float32).double()
    exact = torch.stack(x).sum(0)
    assert ((s32 - exact).abs() <= 3 * 2.0 ** -24 * torch.stack(x).abs().sum(0) + 1e-30).all()


def test_bf16_ring_world8_bounded_against_fp32_sum(world8_grads):
    lay, grads = world8_grads
    ranges = [lay.layer_range(i) for i in range(len(lay.layers))]
    # the buckets the trainer uses (config bucket_mb), and small ones (more chunk seams)
    for bucket_bytes in (int(6.0 * 2 ** 20), 64 * 1024):
        buckets = dp.make_buckets(ranges, bucket_bytes)
        twins = [g.to(torch.bfloat16) for g in grads]           # what pass 2 writes
        wire = dp.ring_allreduce_emulate(twins, buckets).double()
        exact = torch.stack([g.double() for g in grads]).sum(0)  # the fp32 wire, exactly
        twin_sum = torch.stack([t.double() for t in twins]).sum(0)
        # (1) theorem: the 7 hop roundings stay within gamma_7 * sum |twin_i| (+ the final
        # store's rounding is one of them); each twin's own rounding within u |g_i|
        hop = (wire - twin_sum).abs()
        assert (hop <= dp.recursive_sum_bound(twins) + 1e-38).all()
        tw = (twin_sum - exact).abs()
        assert (tw <= dp.BF16_UNIT_ROUNDOFF * torch.stack(
            [g.double().abs() for g in grads]).sum(0) + 1e-38).all()
        # (2) normwise: the world-8 bf16 wire error of the reduced gradient
        nrm = exact.norm()
        err = ((wire - exact).norm() / nrm).item()
        err1 = ((twin_sum.to(torch.bfloat16).double() - exact).norm() / nrm).item()
        # (measured: 6.6e-3 vs 2.2e-3 for ONE rounding of the exact sum — the hop errors add
        # like a random walk, ~sqrt(7)x, not 7x)
        assert err < 1e-2, err
        assert err < 4.0 * max(err1, 1e-6), (err, err1)
        # (3) against the sampling noise of the global-batch gradient: the standard error of
        # the mean over the 8 shards' estimates (per-rank mean gradient = 8 x its share);
        # measured: the wire error is 0.65% of it
        est = torch.stack([WORLD * g.double() for g in grads])
        se = ((est - exact).pow(2).sum(1).sum() / (WORLD * (WORLD - 1))).sqrt().item()
        assert (wire - exact).norm().item() < 0.02 * se, ((wire - exact).norm().item(), se)
        # per-layer: no layer's gradient (weights, biases, per-position biases) is an
        # outlier — every range within 1.5% relative (measured <= 0.7%)
        for s, e in ranges:
            r = ((wire[s:e] - exact[s:e]).norm() / exact[s:e].norm().clamp_min(1e-30)).item()
            assert r < 1.5e-2, (s, e, r)


def test_sgd_update_under_world8_bf16_wire_close_to_fp32(world8_grads):
    """The quantity training sees: one SGD update with the world-8 bf16 wire vs the fp32 wire
    (the fused update reads the all-reduced twin): relative difference of the updates."""
    lay, grads = world8_grads
    twins = [g.to(torch.bfloat16) for g in grads]
    wire = dp.ring_allreduce_emulate(twins).float()
    exact = torch.stack(grads).sum(0)
    lr = 0.05
    d16, d32 = -lr * wire, -lr * exact
    assert ((d16 - d32).norm() / d32.norm()).item() < 1e-2
