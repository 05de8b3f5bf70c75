"""Dataset index, packed dataset and threaded loader."""
import os

import numpy as np
import pytest

from deep_go_amd.data.dataset import (GameIndex, PackedDataset, load_index, sample_reference,
                                      write_counts)
from deep_go_amd.data.loader import BatchLoader


@pytest.fixture(scope="module")
def train_index(ref_data):
    return load_index(ref_data, "train", build_missing=False)


def test_index_parsing(ref_data, train_index):
    # 21 listed games, one with count 0 and no directory -> 20 usable, 4139 positions
    assert len(train_index) == 20
    assert train_index.num_positions == 4139
    assert load_index(ref_data, "validation").num_positions == 134
    assert load_index(ref_data, "test").num_positions == 125


def test_write_counts_matches_reference_index(ref_data, tmp_path):
    import shutil
    root = tmp_path / "data"
    shutil.copytree(f"{ref_data}/test", root / "test")
    write_counts(str(root), "test")
    idx = load_index(str(root), "test")
    assert [n for _, n in idx.games] == [125]


def test_packed_matches_files(train_index):
    pk = PackedDataset.from_index(train_index)
    assert len(pk) == 4139 and pk.num_games == 20
    lf = BatchLoader(train_index, 16, threads=3, prefetch=3, seed=7, pin=False)
    lp = BatchLoader(pk, 16, threads=2, prefetch=2, seed=7, pin=False)
    for _ in range(5):
        a, b = lf.next_numpy(), lp.next_numpy()
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    assert lf.errors() == 0
    lf.close()
    lp.close()


def test_loader_deterministic_across_thread_counts(train_index):
    pk = PackedDataset.from_index(train_index)
    runs = []
    for threads in (1, 5):
        ld = BatchLoader(pk, 32, threads=threads, prefetch=4, seed=123, pin=False)
        runs.append([ld.next_numpy()[3] for _ in range(6)])
        ld.close()
    assert all(np.array_equal(a, b) for a, b in zip(*runs))


def test_game_uniform_sampling_bias():
    """The reference samples a game uniformly then a move uniformly (data.lua:29-37): a
    game with 10 positions is drawn as often as one with 1000."""
    counts = [10, 1000]
    pk = PackedDataset.from_arrays(np.zeros((1010, 9, 19, 19), np.uint8), np.ones(1010),
                                   np.ones(1010), np.arange(1010) % 361, game_size=10)
    pk.game_start = np.array([0, 10])
    pk.game_count = np.array(counts, np.int32)
    ld = BatchLoader(pk, 256, threads=2, prefetch=2, seed=1, pin=False)
    small = 0
    n = 0
    impl = ld._impl
    for k in range(40):
        s = impl.sample_batch(k)
        small += sum(1 for g, _ in s if g == 0)
        n += len(s)
    ld.close()
    assert 0.4 < small / n < 0.6
    g, m = sample_reference(counts, 20000, np.random.default_rng(0))
    assert 0.45 < (g == 0).mean() < 0.55 and m.min() >= 1


def test_position_uniform_sampling():
    pk = PackedDataset.from_arrays(np.zeros((1010, 9, 19, 19), np.uint8), np.ones(1010),
                                   np.ones(1010), np.arange(1010) % 361)
    pk.game_start = np.array([0, 10])
    pk.game_count = np.array([10, 1000], np.int32)
    ld = BatchLoader(pk, 256, threads=1, prefetch=2, seed=1, sampling="position", pin=False)
    s = [g for k in range(20) for g, _ in ld._impl.sample_batch(k)]
    ld.close()
    assert np.mean(np.array(s) == 0) < 0.03


def test_packed_save_load(tmp_path, train_index):
    pk = PackedDataset.from_index(train_index)
    p = str(tmp_path / "t.npz")
    pk.save(p)
    q = PackedDataset.load(p)
    assert np.array_equal(pk.planes, q.planes) and np.array_equal(pk.label, q.label)
    assert np.array_equal(pk.game_count, q.game_count)


@pytest.mark.parametrize("B", [1, 5, 8])
def test_pack_batch_roundtrip(B):
    """HipGoNet's single-copy input layout (planes | player | rank | int32 labels)."""
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import pack_batch, packed_batch_bytes, unpack_views
    pl, py, rk, lb = random_planes(B, seed=2)
    buf = pack_batch(pl, py, rk, lb)
    assert buf.numel() == packed_batch_bytes(B)
    a, b, c, d = unpack_views(buf, B)
    assert (a.numpy() == pl.reshape(B, 9, 361)).all() and (b.numpy() == py).all()
    assert (c.numpy() == rk).all() and (d.numpy() == lb).all()


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_packed_slot_copy_matches_numpy(packed_fixture, device):
    """next_packed_to (one copy of the pinned packed slot) carries the same batches as
    next_numpy, and many more batches than slots go through without a stall."""
    import torch
    from deep_go_amd.data.batch import packed_batch_bytes, unpack_views
    pk = PackedDataset.load(os.path.join(packed_fixture, "train.dgpack.npz"))
    B = 24
    la = BatchLoader(pk, B, threads=2, prefetch=3, seed=11, pin=(device == "cuda"))
    lb = BatchLoader(pk, B, threads=2, prefetch=3, seed=11, pin=False)
    dst = torch.zeros(packed_batch_bytes(B), dtype=torch.uint8, device=device)
    for _ in range(12):
        la.next_packed_to(dst)
        want = lb.next_numpy()
        got = unpack_views(dst.cpu(), B)
        assert np.array_equal(got[0].numpy().reshape(B, 9, 19, 19), want[0])
        for g, w in zip(got[1:], want[1:]):
            assert np.array_equal(g.numpy(), w)
    la.close()
    lb.close()


@pytest.mark.parametrize("split", ["train", "validation", "test"])
def test_committed_packed_fixture_matches_reference(ref_data, packed_fixture, split):
    """tests/fixtures/<split>.dgpack.npz is exactly what our t7 reader makes of the
    reference's bundled data (so GPU-box tests on it test the real fixture)."""
    a = PackedDataset.from_index(load_index(ref_data, split, build_missing=False))
    b = PackedDataset.load(os.path.join(packed_fixture, f"{split}.dgpack.npz"))
    assert len(a) == len(b) and a.num_games == b.num_games
    for f in ("planes", "player", "rank", "label", "game_start", "game_count"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f


def _rank_stream(args):
    r, path, n = args
    from deep_go_amd.data.dataset import PackedDataset
    from deep_go_amd.data.loader import BatchLoader
    pk = PackedDataset.load(path)
    ld = BatchLoader(pk, 16, threads=2, prefetch=3, seed=1000 + r, pin=False)
    out = [ld.next_numpy() for _ in range(n)]
    ld.close()
    return [np.concatenate([a.reshape(-1).astype(np.int64) for a in b]) for b in out]


def test_concurrent_rank_loaders_are_deterministic(packed_fixture):
    """8-rank input pipeline: one loader process per rank (seed 1000 + rank), running
    concurrently, yields exactly the stream the same seed gives in-process; ranks differ."""
    import multiprocessing as mp
    path = os.path.join(packed_fixture, "train.dgpack.npz")
    with mp.get_context("spawn").Pool(4) as pool:
        got = pool.map(_rank_stream, [(r, path, 6) for r in range(4)])
    for r in (0, 3):
        want = _rank_stream((r, path, 6))
        assert all(np.array_equal(a, b) for a, b in zip(got[r], want))
    assert not np.array_equal(got[0][0], got[1][0])


def test_stack_frag_linear_indexing():
    """layouts.stack_frag_linear (conv_stack2's fused first layer): A[row][col] lands at
    [s][wm][kk][i][lane][e] with row = wm*64 + i*16 + (lane & 15), col = s*64 + kk*32 +
    (lane >> 4)*8 + e (a CPU check of the index algebra the kernel and weight_refresh use)."""
    import torch
    from deep_go_amd.ops import layouts as LY
    A = torch.arange(128 * 1024, dtype=torch.int64).reshape(128, 1024)
    f = LY.stack_frag_linear(A).reshape(16, 2, 2, 4, 64, 8)
    rng = np.random.default_rng(0)
    for _ in range(200):
        s_, wm, kk, i, lane, e = (int(rng.integers(n)) for n in (16, 2, 2, 4, 64, 8))
        row = wm * 64 + i * 16 + (lane & 15)
        col = s_ * 64 + kk * 32 + (lane >> 4) * 8 + e
        assert f[s_, wm, kk, i, lane, e].item() == A[row, col].item()


def test_stack_frag_linear_multi_pass_and_pbias_indexing():
    """conv_l1_frag's operands (conv_l1.hip): the first layer's [256][1024] weights as two
    128-channel passes [h][s][wm][kk][i][lane][e] (pass 0 = the 128-channel layout), and the
    stack-order bias table [h][24][wm][i][lane][4] = bf16(bias + posb) of pixel
    jg*16 + (lane & 15) (clamped to 360), channels 128h + wm*64 + i*16 + (lane >> 4)*4 + e —
    the order weight_refresh writes (CPU check of the index algebra)."""
    import torch
    from deep_go_amd.ops import layouts as LY
    A = torch.arange(256 * 1024, dtype=torch.int64).reshape(256, 1024)
    f = LY.stack_frag_linear(A, 256).reshape(2, 16, 2, 2, 4, 64, 8)
    assert torch.equal(f[0].reshape(-1), LY.stack_frag_linear(A[:128]))
    rng = np.random.default_rng(1)
    for _ in range(200):
        h, s_, wm, kk, i, lane, e = (int(rng.integers(n)) for n in (2, 16, 2, 2, 4, 64, 8))
        row = 128 * h + wm * 64 + i * 16 + (lane & 15)
        col = s_ * 64 + kk * 32 + (lane >> 4) * 8 + e
        assert f[h, s_, wm, kk, i, lane, e].item() == A[row, col].item()
    C = 256
    bias = torch.randn(C)
    posb = torch.randn(361, C)
    tab = (posb + bias[None, :]).to(torch.bfloat16)
    pf = LY.stack_pbias_frag(bias, posb).reshape(2, 24, 2, 4, 64, 4)
    for _ in range(200):
        h, jg, wm, i, lane, e = (int(rng.integers(n)) for n in (2, 24, 2, 4, 64, 4))
        p = min(jg * 16 + (lane & 15), 360)
        c = 128 * h + wm * 64 + i * 16 + (lane >> 4) * 4 + e
        assert pf[h, jg, wm, i, lane, e].item() == tab[p, c].item()


def test_stack_frag_layout_indexing():
    """layouts.stack_frag puts A[row][col] at the conv_stack2 fragment index (CPU check of the
    permutation the kernel and weight_refresh assume)."""
    import torch
    from deep_go_amd.ops import layouts as LY
    A = torch.arange(128 * 1152, dtype=torch.float64).reshape(128, 1152)
    f = LY.stack_frag(A)
    rng = np.random.default_rng(0)
    for _ in range(200):
        s, wm, kk, i, lane, e = (int(rng.integers(n)) for n in (18, 2, 2, 4, 64, 8))
        chunk, tap = divmod(s, 9)
        row = wm * 64 + i * 16 + (lane & 15)
        col = tap * 128 + chunk * 64 + kk * 32 + (lane >> 4) * 8 + e
        idx = ((((s * 2 + wm) * 2 + kk) * 4 + i) * 64 + lane) * 8 + e
        assert f[idx].item() == A[row, col].item()


def test_stack_frag_f8_layout_indexing():
    """layouts.stack_frag_f8 puts byte w8[co][tap][ci] where conv_stack_f8 loads it."""
    import torch
    from deep_go_amd.ops import layouts as LY
    w = torch.arange(128 * 9 * 128, dtype=torch.int64).reshape(128, 9, 128)
    f = LY.stack_frag_f8(w)
    rng = np.random.default_rng(1)
    # 128 channels: half-major K-steps [st][wm][i][half][lane][e]: lane group g = 2p + q holds
    # unit n = 2 st + p = 9 kh + tap, channels 64 kh + 32 q + 16 half + e
    for _ in range(200):
        st, wm, i, half, lane, e = (int(rng.integers(n)) for n in (9, 2, 4, 2, 64, 16))
        g = lane >> 4
        kh, t = divmod(2 * st + (g >> 1), 9)
        co = wm * 64 + i * 16 + (lane & 15)
        ci = 64 * kh + 32 * (g & 1) + 16 * half + e
        idx = ((((st * 2 + wm) * 4 + i) * 2 + half) * 64 + lane) * 16 + e
        assert f[idx].item() == w[co, t, ci].item()
    # every (co, tap, ci) exactly once
    assert torch.equal(torch.sort(f).values, torch.arange(128 * 9 * 128))
    # 256 channels: [h][tap][c][wm][i][half][lane][e]
    w = torch.arange(256 * 9 * 256, dtype=torch.int64).reshape(256, 9, 256)
    f = LY.stack_frag_f8(w)
    for _ in range(200):
        h, t, c, wm, i, half, lane, e = (int(rng.integers(n)) for n in (2, 9, 2, 2, 4, 2, 64, 16))
        co = 128 * h + wm * 64 + i * 16 + (lane & 15)
        ci = 128 * c + 32 * (lane >> 4) + 16 * half + e
        idx = ((((((h * 9 + t) * 2 + c) * 2 + wm) * 4 + i) * 2 + half) * 64 + lane) * 16 + e
        assert f[idx].item() == w[co, t, ci].item()
