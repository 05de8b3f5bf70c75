"""HIP kernel numerics vs plain PyTorch fp32 oracles (SURVEY.md §4.3 'Kernel unit tests').

Inputs are rounded to bf16 first so the oracle sees exactly what the MFMA sees; the
remaining error is fp32-accumulation order + the bf16 rounding of the output.  The conv
oracle itself is computed on the CPU (conv_ref).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def bf(x):
    return x.to(torch.bfloat16).float()


def rel_err(a, b):
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def conv_ref(x, w_ohwi, k):
    """The fp32 oracle runs on the CPU (a CPU F.conv2d, not a GPU library
    conv); the result comes back to x's device.  Differentiable through the device moves,
    so autograd gives the CPU dgrad / wgrad oracles too."""
    y = F.conv2d(x.cpu().float(), w_ohwi.cpu().float().permute(0, 3, 1, 2),
                 padding=(k - 1) // 2)
    return y.to(x.device)


@pytest.mark.parametrize("B,cin,cout,k,tiles", [
    (2, 64, 64, 3, None), (7, 128, 128, 3, None), (3, 40, 128, 5, None), (1, 16, 16, 3, None),
    (5, 128, 128, 3, (128, 128)), (5, 128, 128, 3, (128, 192)), (4, 256, 256, 3, None),
    (3, 64, 64, 3, (64, 256)), (2, 128, 128, 1, None)])
def test_conv_forward_linear(B, cin, cout, k, tiles):
    torch.manual_seed(0)
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) / (k * (cin ** 0.5)))
    from deep_go_amd.ops import functional as Fn
    y = Fn.conv_forward(x, w, epi="linear", tiles=tiles)
    ref = conv_ref(x, w, k)
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("B,cin,cout,k", [(3, 64, 64, 3), (2, 40, 128, 5), (6, 128, 128, 3)])
def test_conv_forward_bias_relu(B, cin, cout, k):
    torch.manual_seed(1)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5))
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y = Fn.conv_forward(x, w, b, pb, epi="fwd")
    ref = F.relu(conv_ref(x, w, k) + b.view(1, -1, 1, 1) + pb.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("B,cin,cout,k", [(3, 64, 64, 3), (7, 128, 128, 3), (2, 256, 256, 3),
                                          (2, 16, 16, 3), (4, 128, 64, 3)])
def test_conv_dgrad(B, cin, cout, k):
    torch.manual_seed(2)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5))
    dz = bf(torch.randn(B, cout, 19, 19, device=DEV))
    aux = bf(torch.relu(torch.randn(B, cin, 19, 19, device=DEV)))
    got = Fn.conv_dgrad(dz, w, aux)
    xr = x.clone().requires_grad_(True)
    y = conv_ref(xr, w, k)
    (gx,) = torch.autograd.grad(y, xr, dz)
    ref = gx * (aux > 0)
    assert rel_err(got, ref) < 1e-2


@pytest.mark.parametrize("B,cin,cout,k", [(3, 64, 64, 3), (5, 128, 128, 3), (2, 256, 256, 3),
                                          (3, 128, 64, 3), (2, 64, 128, 1), (1, 192, 128, 3),
                                          (2, 64, 128, 5)])
@pytest.mark.parametrize("bm", ["64", "128"])
def test_conv_board_forward(B, cin, cout, k, bm, monkeypatch):
    monkeypatch.setenv("DG_BOARD_BM", bm)  # 64: single halo / 2 WGs per CU; 128: double halo
    torch.manual_seed(5)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5))
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y = Fn.conv_board(x, w, epi="linear")
    assert rel_err(y, conv_ref(x, w, k)) < 1e-2
    y = Fn.conv_board(x, w, b, pb, epi="fwd")
    ref = F.relu(conv_ref(x, w, k) + b.view(1, -1, 1, 1) + pb.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref) < 1e-2


@pytest.mark.parametrize("B,cin,cout,k", [(3, 40, 128, 5), (2, 37, 64, 5), (5, 64, 128, 3)])
def test_conv_nt_relu_mask(B, cin, cout, k):
    """The pixel-tiled forward (first layer) writes the same ReLU bitmask layout as the
    board kernels: bit = bf16 output != 0."""
    torch.manual_seed(8)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5)
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y, mask = Fn.conv_nt_mask(x, w, b, pb)
    assert torch.equal(y, Fn.conv_forward(x, w, b, pb, tiles=None))
    bits = torch.stack([(mask >> e) & 1 for e in range(8)], -1).reshape(B, 361, cout)
    ref = (y.permute(0, 2, 3, 1).reshape(B, 361, cout) != 0).to(bits.dtype)
    assert torch.equal(bits, ref)


@pytest.mark.parametrize("bm", [64, 128])
def test_conv_board_pbias_and_relu_mask(bm):
    """Forward with the combined bf16 bias table writes the ReLU bitmask; dgrad gated by the
    bitmask equals dgrad gated by the activation frame."""
    torch.manual_seed(9)
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    B, C, k = 3, 128, 3
    x = bf(torch.relu(torch.randn(B, C, 19, 19, device=DEV)))
    w = bf(torch.randn(C, k, k, C, device=DEV) / (k * C ** 0.5))
    b = torch.randn(C, device=DEV) * 0.1
    pb = torch.randn(361, C, device=DEV) * 0.1
    KP, _, Mpad = LY.conv_dims(k, C, C, bm)
    A = LY.fwd_weight(w.float(), C, KP, Mpad)
    xf = LY.to_frame(x, 1, C)
    y = LY.alloc_frame(B, C, 1, DEV)
    pbias = (b.view(1, C) + pb).to(torch.bfloat16).contiguous()
    mask = torch.zeros(B, 361, C // 8, dtype=torch.uint8, device=DEV)
    s = stream_handle()
    h.conv_board_ex(h.EPI_FWD, k, bm, A.data_ptr(), KP, C, Mpad, xf.data_ptr(), 1, C, B,
                    y.data_ptr(), 1, 0, 0, pbias.data_ptr(), 0, 0, mask.data_ptr(), s)
    yv = LY.from_frame(y, 1, C)
    ref = F.relu(conv_ref(x, w, k) + pbias.float().t().reshape(1, C, 19, 19))
    assert rel_err(yv, ref) < 1e-2
    bits = torch.stack([(mask >> e) & 1 for e in range(8)], -1).reshape(B, 361, C)
    assert torch.equal(bits.bool(), (yv > 0).reshape(B, C, 361).transpose(1, 2))
    # dgrad: mask vs aux frame
    dz = bf(torch.randn(B, C, 19, 19, device=DEV))
    Ad = LY.dgrad_weight(w.float(), KP, Mpad)
    dzf = LY.to_frame(dz, 1)
    o1 = LY.alloc_frame(B, C, 1, DEV)
    o2 = LY.alloc_frame(B, C, 1, DEV)
    h.conv_board_ex(h.EPI_DGRAD, k, bm, Ad.data_ptr(), KP, C, Mpad, dzf.data_ptr(), 1, C, B,
                    o1.data_ptr(), 1, 0, 0, 0, y.data_ptr(), 1, 0, s)
    h.conv_board_ex(h.EPI_DGRAD, k, bm, Ad.data_ptr(), KP, C, Mpad, dzf.data_ptr(), 1, C, B,
                    o2.data_ptr(), 1, 0, 0, 0, 0, 1, mask.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)


@pytest.mark.parametrize("B,cin,cout,k,bm", [(3, 128, 128, 3, 64), (2, 256, 128, 3, 64),
                                             (2, 128, 256, 3, 128), (2, 128, 64, 1, 64)])
def test_conv_board_fp8_forward(B, cin, cout, k, bm):
    """FP8 (e4m3, MX-scaled MFMA) forward vs the fp32 reference of the same op: error at the
    e4m3 quantization level (3 mantissa bits), bf16 + fp8 outputs, amax tracking."""
    torch.manual_seed(8)
    from deep_go_amd.ops import functional as Fn
    x = torch.relu(torch.randn(B, cin, 19, 19, device=DEV))
    w = torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5)
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y, y8, s_y, amax = Fn.conv_board_fp8(x, w, b, pb, bm=bm)
    ref = F.relu(conv_ref(x, w, k) + b.view(1, -1, 1, 1) + pb.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref) < 0.08   # e4m3 operands: ~4-5% expected (CPU simulation)
    # exact-semantics check: the same op on e4m3-rounded operands (torch's OCP e4m3fn cast)
    q = lambda t, sc: ((t.cpu() / sc).to(torch.float8_e4m3fn).float() * sc).to(DEV)
    xb = bf(x)  # the kernel quantizes the bf16 activation frame, with its amax
    sx = xb.abs().max().item() / 448
    sw = w.abs().max().item() / 448
    ref_q = F.relu(conv_ref(q(xb, sx), q(w, sw), k) + b.view(1, -1, 1, 1)
                   + pb.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref_q) < 1e-2
    assert abs(amax - y.max().item()) < 1e-2 * y.max().item() + 1e-6
    assert rel_err(y8, ref) < 0.15  # second quantization (fp8 shadow for the next layer)


@pytest.mark.parametrize("B,cin,cout,k", [(3, 64, 64, 3), (4, 128, 128, 3), (2, 256, 256, 3),
                                          (2, 64, 128, 3)])
@pytest.mark.parametrize("bm", ["64", "128"])
def test_conv_board_dgrad(B, cin, cout, k, bm, monkeypatch):
    monkeypatch.setenv("DG_BOARD_BM", bm)
    torch.manual_seed(6)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) / (k * cin ** 0.5))
    dz = bf(torch.randn(B, cout, 19, 19, device=DEV))
    aux = bf(torch.relu(torch.randn(B, cin, 19, 19, device=DEV)))
    got = Fn.conv_board(dz, w, epi="dgrad", aux=aux)
    xr = x.clone().requires_grad_(True)
    (gx,) = torch.autograd.grad(conv_ref(xr, w, k), xr, dz)
    assert rel_err(got, gx * (aux > 0)) < 1e-2


@pytest.mark.parametrize("B,cin,cout,k,splits", [(3, 64, 64, 3, None), (7, 128, 128, 3, None),
                                                 (2, 40, 128, 5, 3), (5, 256, 256, 3, None),
                                                 (1, 16, 16, 3, 1), (2, 128, 128, 1, 2),
                                                 (3, 128, 128, 3, 7), (2, 128, 256, 3, None)])
def test_conv_wgrad(B, cin, cout, k, splits):
    """im2col wgrad: the three-slice 128x384 tiles where K % 384 == 0 (9 x 128 / 256), else
    the 2-stage 128x128 kernel (the first layer's 5 x 5 x 40, d = 64 / 16 layers, 1 x 1)."""
    torch.manual_seed(3)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    dz = bf(torch.randn(B, cout, 19, 19, device=DEV))
    got, gp, gb = Fn.conv_wgrad(dz, x, k, splits=splits, with_bias=True, algo="im2col")
    w0 = torch.zeros(cout, k, k, cin, device=DEV, requires_grad=True)
    y = conv_ref(x, w0, k)
    (gw,) = torch.autograd.grad(y, w0, dz)
    assert rel_err(got, gw) < 1e-3
    # fused bias grads (column sums of dZ)
    assert rel_err(gp, dz.sum(0).reshape(cout, 361).t()) < 1e-4
    assert rel_err(gb, dz.sum((0, 2, 3))) < 1e-4


@pytest.mark.parametrize("B,cout,splits", [(2, 128, 3), (7, 128, None), (256, 128, 64),
                                           (5, 256, 4)])
def test_conv_wgrad5_pipe_bit_identical(B, cout, splits):
    """The first layer's 5x5 weight gradient on conv_wgrad_pipe_kernel (32-pixel K-steps,
    four LDS-DMA stages) vs conv_wgrad_kernel (two 64-pixel stages): the same
    tiles and the same MFMA summation order, so BIT-identical gradients (B = 256: the
    flagship shape, 64 splits) — and both against the fp32 reference."""
    torch.manual_seed(5)
    from deep_go_amd.ops import functional as Fn
    from deep_go_amd.ops.native import hip
    x = bf(torch.relu(torch.randn(B, 37, 19, 19, device=DEV)))
    dz = bf(torch.randn(B, cout, 19, 19, device=DEV))
    res = {}
    try:
        for ns in (0, 4):
            hip().conv_wgrad5_set_ns(ns)
            res[ns] = Fn.conv_wgrad(dz, x, 5, splits=splits, cinp=40, algo="im2col")
            torch.cuda.synchronize()
    finally:
        hip().conv_wgrad5_set_ns(int(os.environ.get("DG_WGRAD5_NS", "4")))
    assert torch.equal(res[0], res[4])
    w0 = torch.zeros(cout, 5, 5, 37, device=DEV, requires_grad=True)
    (gw,) = torch.autograd.grad(conv_ref(x, w0, 5), w0, dz)
    assert rel_err(res[4], gw) < 1e-3


@pytest.mark.parametrize("B,cin,cout,k", [(3, 37, 128, 5), (2, 40, 256, 5), (1, 37, 96, 5),
                                         (4, 64, 128, 3), (5, 16, 128, 5)])
def test_conv_l1(B, cin, cout, k):
    """Board-resident first-layer forward (conv_l1.hip: whole input frame in LDS, K over
    8-channel (tap, chunk) groups; half-board 4-wave workgroups, or whole-board 8-wave ones
    where two do not fit on a CU — the 64-channel 3x3 shape) vs the fp32 reference."""
    torch.manual_seed(8)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, k, k, cin, device=DEV) * 0.1)
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y, mask = Fn.conv_l1(x, w, b, pb, with_mask=cout % 8 == 0)
    ref = torch.relu(conv_ref(x, w, k) + b[None, :, None, None]
                     + pb.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref) < 1e-2
    # bitmask: bit k of byte q = channel 8q + k of the stored bf16 output is nonzero
    bits = (mask.unsqueeze(-1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1
    nz = (y.to(torch.bfloat16) != 0).permute(0, 2, 3, 1).reshape(B, 361, cout)
    assert torch.equal(bits.reshape(B, 361, cout).bool(), nz)


@pytest.mark.parametrize("B,cin,cout", [(3, 37, 128), (2, 40, 256), (5, 37, 384), (1, 16, 128)])
def test_conv_l1_frag(B, cin, cout):
    """First layer on conv_l1_frag (conv_l1.hip: one board per workgroup, the input frame in
    conflict-free planes, fragment-ordered weights, 1-3 128-channel passes) vs the fp32
    reference with the same bf16-rounded bias table, and its ReLU bitmask."""
    torch.manual_seed(9)
    from deep_go_amd.ops import functional as Fn
    from deep_go_amd.ops.native import hip
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    w = bf(torch.randn(cout, 5, 5, cin, device=DEV) * 0.1)
    b = torch.randn(cout, device=DEV) * 0.1
    pb = torch.randn(361, cout, device=DEV) * 0.1
    y, mask = Fn.conv_l1_frag(x, w, b, pb)
    torch.cuda.synchronize()
    tab = (pb + b[None, :]).to(torch.bfloat16).float()
    ref = torch.relu(conv_ref(x, w, 5) + tab.t().reshape(1, cout, 19, 19))
    assert rel_err(y, ref) < 1e-2
    bits = (mask.unsqueeze(-1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1
    nz = (y.to(torch.bfloat16) != 0).permute(0, 2, 3, 1).reshape(B, 361, cout)
    assert torch.equal(bits.reshape(B, 361, cout).bool(), nz)


@pytest.mark.parametrize("B,cin,cout,splits", [
    (3, 128, 128, None), (1, 128, 128, 1), (2, 128, 128, 26), (5, 256, 256, None),
    (4, 64, 128, 7), (3, 192, 256, 2), (6, 128, 128, 5), (3, 128, 64, None)])
def test_conv_wgrad_win(B, cin, cout, splits):
    """Sliding-window 3x3 wgrad (conv_wgrad_win.hip: frame-linear K, one X window for all 9
    taps, split ranges that start / end inside a board) vs the fp32 reference."""
    torch.manual_seed(6)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.randn(B, cin, 19, 19, device=DEV))
    dz = bf(torch.randn(B, cout, 19, 19, device=DEV))
    got = Fn.conv_wgrad(dz, x, 3, splits=splits, algo="win")
    w0 = torch.zeros(cout, 3, 3, cin, device=DEV, requires_grad=True)
    (gw,) = torch.autograd.grad(conv_ref(x, w0, 3), w0, dz)
    assert rel_err(got, gw) < 1e-3


@pytest.mark.parametrize("B,C,k,relu", [(3, 64, 3, True), (7, 128, 3, True),
                                        (5, 128, 3, False), (2, 32, 1, False), (4, 256, 3, True),
                                        (5, 256, 3, False)])
def test_head(B, C, k, relu):
    """Fused head (3x3/128 and /256: the MFMA kernel; other shapes: the VALU kernel) vs fp32
    autograd."""
    torch.manual_seed(4)
    from deep_go_amd.ops import functional as Fn
    x = bf(torch.relu(torch.randn(B, C, 19, 19, device=DEV)))
    w = bf(torch.randn(1, k, k, C, device=DEV) * 0.05)  # fwd dots use bf16 weights
    b = torch.randn(1, device=DEV) * 0.1
    pb = torch.randn(361, device=DEV) * 0.1
    labels = torch.randint(0, 361, (B,), device=DEV)
    out = Fn.head(x, w, b, pb, labels, head_relu=relu)
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    pr = pb.clone().requires_grad_(True)
    z = conv_ref(xr, wr, k) + br.view(1, 1, 1, 1) + pr.view(1, 1, 19, 19)
    if relu:
        z = torch.relu(z)
    logp = F.log_softmax(z.reshape(B, 361), 1)
    loss = F.nll_loss(logp, labels)
    gx, gw, gb, gp = torch.autograd.grad(loss, [xr, wr, br, pr])
    assert rel_err(out["logp"], logp) < 1e-4
    assert torch.allclose(out["loss"].mean(), loss, rtol=1e-4, atol=1e-5)
    assert (out["pred"].long() == logp.argmax(1)).float().mean() > 0.99
    assert rel_err(out["dz"], gx * (x > 0)) < 1e-2
    assert rel_err(out["gw"], gw) < 1e-3
    assert (out["gbias"] - gb.view(1)).abs().item() < 1e-3 * max(1.0, gb.abs().item())
    assert rel_err(out["gposb"], gp.view(-1)) < 1e-3


def test_expand_features():
    from deep_go_amd.data.features import expand_batch
    from deep_go_amd.ops import functional as Fn
    rng = np.random.default_rng(0)
    B = 9
    planes = np.zeros((B, 9, 19, 19), np.uint8)
    planes[:, 0] = rng.integers(0, 3, (B, 19, 19))
    for c in range(1, 9):
        planes[:, c] = rng.integers(0, 12, (B, 19, 19))
    # simple-ko marks at a few empty points (liberty plane = KO_MARK; data/features.py)
    for b in range(B):
        e = np.flatnonzero(planes[b, 0].reshape(-1) == 0)[b % 3]
        planes[b, 1].reshape(-1)[e] = 255
    player = rng.integers(1, 3, B).astype(np.uint8)
    rank = rng.integers(1, 10, B).astype(np.uint8)
    got = Fn.expand_features(torch.from_numpy(planes), torch.from_numpy(player),
                             torch.from_numpy(rank))
    ref = expand_batch(planes, player, rank, ko=True)
    assert torch.equal(got[:, :38].cpu(), torch.from_numpy(ref))
    assert got[:, 37].sum().item() == B
    assert got[:, 38:].abs().sum().item() == 0


def test_bias_grad():
    from deep_go_amd.ops import functional as Fn
    dz = bf(torch.randn(13, 128, 19, 19, device=DEV))
    gp, gb = Fn.bias_grad(dz)
    ref_p = dz.sum(0).reshape(128, 361).t()
    assert rel_err(gp, ref_p) < 1e-5
    assert rel_err(gb, dz.sum((0, 2, 3))) < 1e-4


@pytest.mark.parametrize("C", [128, 256])
def test_bias_grad_multi(C):
    """Multi-layer bias partials (elementwise.hip bias_grad_partial_kernel<2>, the launch
    beside the window weight gradient) vs the fp32 per-chunk sums of the same bf16 frames."""
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    torch.manual_seed(C)
    B, nl, P = 128, 2, 361
    dz = [bf(torch.randn(B, C, 19, 19, device=DEV)) for _ in range(nl)]
    frames = [LY.to_frame(d, 1) for d in dz]
    nch = h.bias_chunks_multi(B)
    parts = [torch.full((nch * (P + 19) * C,), float("nan"), device=DEV) for _ in range(nl)]
    tab = np.array([[f.data_ptr(), q.data_ptr(), 0] for f, q in zip(frames, parts)],
                   dtype=np.int64)
    h.bias_grad_partial_multi(tab.ctypes.data, nl, B, C, 1, 0, stream_handle())
    torch.cuda.synchronize()
    for i in range(nl):
        ref = dz[i].view(nch, B // nch, C, P).sum(1).transpose(1, 2)     # [chunk][p][C]
        ref_r = ref.reshape(nch, 19, 19, C).sum(2)                       # [chunk][h][C]
        got = parts[i]
        assert rel_err(got[:nch * P * C].view(nch, P, C), ref) < 1e-5, i
        assert rel_err(got[nch * P * C:].view(nch, 19, C), ref_r) < 1e-5, i


def test_sgd_and_lr_decay():
    from deep_go_amd.ops import functional as Fn
    p = torch.randn(1001, device=DEV)
    g = torch.randn(1001, device=DEV)
    p0 = p.clone()
    lr = Fn.sgd_(p, g, 0.5, 0.1, steps=3)
    lrs = [0.5, 0.45, 0.405]
    ref = p0 - sum(lrs) * g
    assert torch.allclose(p, ref, atol=1e-5)
    assert abs(lr.item() - 0.5 * 0.9 ** 3) < 1e-12


def test_weight_refresh():
    from deep_go_amd.ops import functional as Fn
    from deep_go_amd.ops import layouts as LY
    w = torch.randn(64, 3, 3, 32, device=DEV)
    KP, _, Mpad = LY.conv_dims(3, 32, 64, 64)
    KPd, _, Mpad_d = LY.conv_dims(3, 64, 32, 64)
    wf, wd = Fn.weight_refresh(w, 32, KP, Mpad, KPd, Mpad_d)
    assert torch.equal(wf, LY.fwd_weight(w, 32, KP, Mpad))
    assert torch.equal(wd, LY.dgrad_weight(w, KPd, Mpad_d))


def test_weight_refresh_stack_fragments():
    """conv_stack2's fragment-ordered A operands (written by weight_refresh from the fp32
    master) are the plain forward / dgrad operand matrices permuted by layouts.stack_frag."""
    from deep_go_amd.ops import functional as Fn
    from deep_go_amd.ops import layouts as LY
    w = torch.randn(128, 3, 3, 128, device=DEV)
    KP, _, Mpad = LY.conv_dims(3, 128, 128, 128)
    wf, wd, ff, fd = Fn.weight_refresh(w, 128, KP, Mpad, KP, Mpad, frag=True)
    assert torch.equal(ff, LY.stack_frag(wf))
    assert torch.equal(fd, LY.stack_frag(wd))
    assert torch.equal(ff, LY.stack_frag(LY.fwd_weight(w, 128, KP, Mpad)))


def test_fp8_scale_update_ignores_non_finite_amax():
    """Delayed fp8 scaling never adopts a non-finite amax (an inf |dz| or a NaN activation):
    the previous scale stays and the event counts as a saturation (otherwise exp2f(inf)
    would zero every later quantized tensor and freeze the scales of the layers below)."""
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    n = 3
    f = lambda vals: torch.tensor(vals, dtype=torch.float32, device=DEV)  # noqa: E731
    bits = lambda vals: f(vals).view(torch.int32).clone()                 # noqa: E731
    scales = f([0.5, 2.0, 0.25, 4.0, 1.0, 8.0])       # [2l] = s_w, [2l + 1] = s_y
    gscales = f([16.0, 32.0, 64.0])
    amax_w = bits([100.0, float("inf"), 10.0])
    amax_y = bits([float("nan"), 64.0, 5.0])
    gamax = bits([float("inf"), 1000.0, float("nan")])
    sat = torch.zeros(3 * n, dtype=torch.int32, device=DEV)
    s0, g0 = scales.clone(), gscales.clone()
    h.fp8_update_scales(n, scales.data_ptr(), amax_w.data_ptr(), 1, amax_y.data_ptr(), 1.05,
                        8.0, sat.data_ptr(), gscales.data_ptr(), gamax.data_ptr(), 0,
                        stream_handle())
    torch.cuda.synchronize()
    assert torch.isfinite(scales).all() and torch.isfinite(gscales).all()
    assert scales[2].item() == s0[2].item()          # layer 1 s_w: amax_w inf -> unchanged
    H = 2.0                                          # conv_fp8.hip FP8_HEADROOM
    assert scales[3].item() == 2.0 ** np.ceil(np.log2(H * 64.0 / 448.0))   # 2^-1
    assert scales[1].item() == s0[1].item()          # layer 0 s_y: amax_y NaN -> unchanged
    assert gscales[0].item() == g0[0].item() and gscales[2].item() == g0[2].item()
    assert abs(scales[0].item() - 100.0 * 1.05 / 448.0) < 1e-6      # finite ones update
    HG = 8.0                                         # g_headroom passed above
    assert gscales[1].item() == 2.0 ** np.ceil(np.log2(HG * 1000.0 / 57344.0))
    s = sat.tolist()
    assert s[2 * 1] == 1 and s[2 * 0 + 1] == 1        # weights l1, activations l0
    assert s[2 * n + 0] == 1 and s[2 * n + 2] == 1    # gradients l0 (inf), l2 (NaN)
    assert (amax_w == 0).all() and (amax_y == 0).all() and (gamax == 0).all()


def test_fp8_gradient_scale_uses_amax_history():
    """The e5m2 gradient scale comes from the max of the last 16 observed gradient amaxes
    (conv_fp8.hip FP8_GHIST): a step with a small amax after a large one keeps the large
    one's range; non-finite amaxes never enter the history; after 16 small steps the scale
    follows the small amax."""
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    n = 2
    f = lambda vals: torch.tensor(vals, dtype=torch.float32, device=DEV)  # noqa: E731
    scales = f([1.0] * (2 * n))
    gscales = f([1.0] * n)
    ghist = torch.zeros((n, 16), dtype=torch.float32, device=DEV)
    sat = torch.zeros(3 * n, dtype=torch.int32, device=DEV)
    amax_w = torch.zeros(n, dtype=torch.int32, device=DEV)
    amax_y = torch.zeros(n, dtype=torch.int32, device=DEV)
    HG = 4.0
    want = lambda a: 2.0 ** np.ceil(np.log2(HG * a / 57344.0))   # noqa: E731

    def step(g0, g1):
        gamax = f([g0, g1]).view(torch.int32).clone()
        h.fp8_update_scales(n, scales.data_ptr(), amax_w.data_ptr(), 1, amax_y.data_ptr(), 1.25,
                            HG, sat.data_ptr(), gscales.data_ptr(), gamax.data_ptr(),
                            ghist.data_ptr(), stream_handle())
        torch.cuda.synchronize()
        return gscales.tolist()

    assert step(1000.0, 5.0) == [want(1000.0), want(5.0)]
    assert step(10.0, float("nan")) == [want(1000.0), want(5.0)]   # history max; NaN skipped
    for _ in range(14):
        g = step(10.0, 7.0)
    assert g == [want(1000.0), want(7.0)]          # 1000 is 15 entries old: still inside
    assert step(10.0, 7.0) == [want(10.0), want(7.0)]   # 16 newer entries: 1000 left
    assert ghist[0].tolist() == [10.0] * 16
