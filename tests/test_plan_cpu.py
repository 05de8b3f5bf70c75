"""CPU checks of HipGoNet launch-plan rewrites that need no GPU: the merge of consecutive
conv_layer2 launches into conv_layer2_multi runs (hip_model.HipGoNet._merge_layer2_runs)."""
import numpy as np

from deep_go_amd.models.hip_model import HipGoNet


class _H:
    EPI_FWD, EPI_DGRAD = 1, 2

    @staticmethod
    def conv_layer2(*a):
        pass

    @staticmethod
    def conv_layer2_multi(*a):
        pass

    @staticmethod
    def other(*a):
        pass


def _net():
    n = HipGoNet.__new__(HipGoNet)
    n.h = _H
    n._l2_tables = []
    return n


def _l2(epi, x, y, a=1000, pb=2000, mk=3000, C=256, B=8):
    # conv_layer2 args: (epi, A, pbias, X, Y, mask, C, B)
    return (_H.conv_layer2, (epi, a + x, pb + x, x, y, mk + x, C, B))


def test_chained_run_becomes_one_multi_launch(monkeypatch):
    monkeypatch.delenv("DG_LAYER2_MULTI", raising=False)
    n = _net()
    ops = [(_H.other, (0,))] + [_l2(1, 10 + i, 11 + i) for i in range(10)] + [(_H.other, (1,))]
    out, own = n._merge_layer2_runs(ops, list(range(len(ops))))
    assert [f for f, _ in out] == [_H.other, _H.conv_layer2_multi, _H.other]
    assert own == [0, 1, 11]
    epi, tab_ptr, nl, C, B = out[1][1]
    assert (epi, nl, C, B) == (1, 10, 256, 8)
    tab = n._l2_tables[0]
    assert tab.ctypes.data == tab_ptr and tab.shape == (10, 5)
    # rows {A, pbias, X, Y, mask}; each row's X is the previous row's Y
    assert np.array_equal(tab[:, 2][1:], tab[:, 3][:-1])
    assert tab[0].tolist() == [1010, 2010, 10, 11, 3010]


def test_runs_split_on_chain_break_kind_and_16_layers(monkeypatch):
    monkeypatch.delenv("DG_LAYER2_MULTI", raising=False)
    n = _net()
    ops = [_l2(1, 0, 1), _l2(1, 1, 2),          # run A (2 layers)
           _l2(1, 50, 51),                     # chain break: single launch kept as is
           _l2(2, 51, 52), _l2(2, 52, 53)]     # kind change: run B (dgrad)
    ops += [_l2(2, 100 + i, 101 + i) for i in range(20)]   # 20 chained: 16 + 4
    out, _ = n._merge_layer2_runs(ops)
    kinds = [(f.__name__, a[2] if f is _H.conv_layer2_multi else None) for f, a in out]
    assert kinds == [("conv_layer2_multi", 2), ("conv_layer2", None),
                     ("conv_layer2_multi", 2), ("conv_layer2_multi", 16),
                     ("conv_layer2_multi", 4)]


def test_disabled_keeps_per_layer_launches(monkeypatch):
    monkeypatch.setenv("DG_LAYER2_MULTI", "0")
    n = _net()
    ops = [_l2(1, i, i + 1) for i in range(4)]
    out, _ = n._merge_layer2_runs(ops)
    assert out == ops
