"""Functional (allocate-and-call) wrappers around the HIP kernels.

Used by the kernel unit tests and by ad-hoc tools; the training executor
(``models/hip_model.py``) calls the same kernels with pre-planned static buffers.
Inputs/outputs here are ordinary NCHW / OHWI tensors so each op can be compared with a
plain PyTorch fp32 oracle.
"""
from __future__ import annotations

import numpy as np
import torch

from . import layouts as LY
from .native import hip, stream_handle

NPTS = 361


def _ptr(t):
    return 0 if t is None else t.data_ptr()


def conv_forward(x: torch.Tensor, w: torch.Tensor, bias=None, posb=None, epi: str = "fwd",
                 tiles=None, cinp: int | None = None) -> torch.Tensor:
    """x [B,Cin,19,19] (any float), w OHWI fp32 [Cout,k,k,Cin] -> fp32 NCHW output.

    epi='fwd': relu(conv + bias[co] + posb[p][co]);  epi='linear': conv only."""
    h = hip()
    dev = w.device
    B, cin = x.shape[:2]
    cout, k, _, _ = w.shape
    pad = (k - 1) // 2
    cinp = cinp or LY.round_up(cin, 8)
    npix = B * NPTS
    bm, bn = tiles or LY.pick_tiles(npix, cout)
    KP, _, Mpad = LY.conv_dims(k, cinp, cout, bm)
    xf = LY.to_frame(x.to(dev), pad, cinp)
    yf = LY.alloc_frame(B, cout, 1, dev)
    A = LY.fwd_weight(w.float(), cinp, KP, Mpad)
    e = {"fwd": h.EPI_FWD, "linear": h.EPI_LINEAR}[epi]
    if e == h.EPI_FWD:
        bias = bias.float().contiguous().to(dev)
        posb = posb.float().contiguous().to(dev)
    h.conv_nt(e, k, bm, bn, A.data_ptr(), KP, cout, Mpad, xf.data_ptr(), pad, cinp, npix,
              yf.data_ptr(), 1, _ptr(bias), _ptr(posb), 0, 0, stream_handle())
    return LY.from_frame(yf, 1, cout)


def conv_l1(x: torch.Tensor, w: torch.Tensor, bias, posb, with_mask: bool = False):
    """Board-resident first-layer forward (conv_l1.hip): relu(conv + bias + posb), fp32 NCHW
    (and the ReLU bitmask [B][361][Cout/8] with with_mask)."""
    h = hip()
    dev = w.device
    B, cin = x.shape[:2]
    cout, k, _, _ = w.shape
    pad = (k - 1) // 2
    cinp = LY.round_up(cin, 8)
    KP, _, Mpad = LY.conv_dims(k, cinp, cout, 128)
    assert h.conv_l1_ok(k, pad, cinp, Mpad, KP)
    xf = LY.to_frame(x.to(dev), pad, cinp)
    yf = LY.alloc_frame(B, cout, 1, dev)
    A = LY.fwd_weight(w.float(), cinp, KP, Mpad)
    bias = bias.float().contiguous().to(dev)
    posb = posb.float().contiguous().to(dev)
    mask = torch.zeros(B, NPTS, cout // 8, dtype=torch.uint8, device=dev) if with_mask else None
    h.conv_l1(k, A.data_ptr(), KP, cout, Mpad, xf.data_ptr(), pad, cinp, B, yf.data_ptr(), 1,
              bias.data_ptr(), posb.data_ptr(), _ptr(mask), 0, stream_handle())
    if with_mask:
        return LY.from_frame(yf, 1, cout), mask
    return LY.from_frame(yf, 1, cout)


def conv_l1_frag(x: torch.Tensor, w: torch.Tensor, bias, posb):
    """First-layer forward on conv_l1_frag (conv_l1.hip: one board per workgroup, plane-staged
    input, fragment-ordered weights, stack-order bf16 bias table) for the 5x5 / 37-40 channel
    layer: relu(conv + bf16(bias + posb)) as fp32 NCHW, and the ReLU bitmask [B][361][Cout/8]."""
    h = hip()
    dev = w.device
    B, cin = x.shape[:2]
    cout, k, _, _ = w.shape
    assert k == 5 and cin <= 40 and h.conv_l1_frag_ok(k, 2, 40, cout, 1)
    KP, _, Mpad = LY.conv_dims(k, 40, cout, 128)
    xf = LY.to_frame(x.to(dev), 2, 40)
    yf = LY.alloc_frame(B, cout, 1, dev)
    A = LY.stack_frag_linear(LY.fwd_weight(w.float(), 40, KP, Mpad), cout)
    pbf = LY.stack_pbias_frag(bias.to(dev), posb.to(dev))
    mask = torch.zeros(B, NPTS, cout // 8, dtype=torch.uint8, device=dev)
    h.conv_l1_frag(A.data_ptr(), pbf.data_ptr(), xf.data_ptr(), B, cout, yf.data_ptr(),
                   mask.data_ptr(), 0, 0, 0, stream_handle())
    return LY.from_frame(yf, 1, cout), mask


def conv_nt_mask(x: torch.Tensor, w: torch.Tensor, bias, posb):
    """Pixel-tiled forward that also writes the ReLU bitmask [B][361][Cout/8] (bit k of
    byte q = channel 8q + k > 0).  Returns (NCHW output, mask)."""
    h = hip()
    dev = w.device
    B, cin = x.shape[:2]
    cout, k, _, _ = w.shape
    pad = (k - 1) // 2
    cinp = LY.round_up(cin, 8)
    npix = B * NPTS
    bm, bn = LY.pick_tiles(npix, cout)
    KP, _, Mpad = LY.conv_dims(k, cinp, cout, bm)
    xf = LY.to_frame(x.to(dev), pad, cinp)
    yf = LY.alloc_frame(B, cout, 1, dev)
    mask = torch.zeros(B, NPTS, cout // 8, dtype=torch.uint8, device=dev)
    A = LY.fwd_weight(w.float(), cinp, KP, Mpad)
    bias = bias.float().contiguous().to(dev)
    posb = posb.float().contiguous().to(dev)
    h.conv_nt_ex(h.EPI_FWD, k, bm, bn, A.data_ptr(), KP, cout, Mpad, xf.data_ptr(), pad, cinp,
                 npix, yf.data_ptr(), 1, bias.data_ptr(), posb.data_ptr(), 0, 0,
                 mask.data_ptr(), stream_handle())
    return LY.from_frame(yf, 1, cout), mask


def conv_board(x: torch.Tensor, w: torch.Tensor, bias=None, posb=None, epi: str = "fwd",
               aux=None) -> torch.Tensor:
    """Board-tiled kernel (1x1/3x3, Cin % 64 == 0).  epi='fwd'|'linear' as conv_forward;
    epi='dgrad': x is dZ [B,Cout,19,19], w is the forward OHWI weight [Cout,k,k,Cin],
    aux [B,Cin,19,19] gates the result (ReLU backward)."""
    h = hip()
    dev = w.device
    B = x.shape[0]
    cout, k, _, cin = w.shape
    pad = (k - 1) // 2
    if epi == "dgrad":
        M, xc = cin, cout
        bm = LY.board_bm(M)
        KP, _, Mpad = LY.conv_dims(k, xc, M, bm)
        A = LY.dgrad_weight(w.float(), KP, Mpad)
        xf = LY.to_frame(x.to(dev), max(1, pad))
        auxf = LY.to_frame(aux.to(dev), pad)
        out = LY.alloc_frame(B, M, 1, dev)
        h.conv_board(h.EPI_DGRAD, k, bm, A.data_ptr(), KP, M, Mpad, xf.data_ptr(), max(1, pad),
                     xc, B, out.data_ptr(), 1, 0, 0, auxf.data_ptr(), pad, stream_handle())
        return LY.from_frame(out, 1, M)
    M, xc = cout, cin
    bm = LY.board_bm(M)
    KP, _, Mpad = LY.conv_dims(k, xc, M, bm)
    A = LY.fwd_weight(w.float(), xc, KP, Mpad)
    xf = LY.to_frame(x.to(dev), pad, xc)
    out = LY.alloc_frame(B, M, 1, dev)
    e = {"fwd": h.EPI_FWD, "linear": h.EPI_LINEAR}[epi]
    if e == h.EPI_FWD:
        bias = bias.float().contiguous().to(dev)
        posb = posb.float().contiguous().to(dev)
    h.conv_board(e, k, bm, A.data_ptr(), KP, M, Mpad, xf.data_ptr(), pad, xc, B, out.data_ptr(),
                 1, _ptr(bias), _ptr(posb), 0, 0, stream_handle())
    return LY.from_frame(out, 1, M)


def conv_board_fp8(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, posb: torch.Tensor,
                   bm: int | None = None):
    """FP8 forward (conv_fp8.hip): x [B,Cin,19,19] (Cin % 128 == 0), OHWI w, fp32 bias/posb.
    Quantizes x / w with per-tensor scales (amax / 448) through the same device kernels the
    model uses; returns (y bf16-frame interior as fp32 NCHW, y8 dequantized, s_y, amax_y)."""
    h = hip()
    dev = w.device
    B = x.shape[0]
    cout, k, _, cin = w.shape
    pad = (k - 1) // 2
    bm = bm or LY.board_bm(cout)
    KP, _, Mpad = LY.conv_dims(k, cin, cout, bm)
    s = stream_handle()
    wflat = w.float().contiguous().to(dev)
    scales = (wflat.abs().max() / 448.0).clamp_min(1e-12).reshape(1)  # s_w
    A8 = torch.zeros((Mpad, KP), dtype=torch.uint8, device=dev)
    h.weight_fp8(wflat.data_ptr(), A8.data_ptr(), cout, cin, k * k, cin, KP, scales.data_ptr(), s)
    xf = LY.to_frame(x.to(dev), pad, cin)
    s_x = (xf.float().abs().max() / 448.0).clamp_min(1e-12).reshape(1)
    x8 = torch.zeros(xf.numel(), dtype=torch.uint8, device=dev)
    h.frame_to_fp8(xf.data_ptr(), x8.data_ptr(), xf.numel(), s_x.data_ptr(), 0, s)
    y = LY.alloc_frame(B, cout, 1, dev)
    y8 = torch.zeros(y.numel(), dtype=torch.uint8, device=dev)
    s_y = torch.full((1,), 1.0 / 64, device=dev)
    amax_y = torch.zeros(1, dtype=torch.int32, device=dev)
    h.conv_board_fp8(k, bm, A8.data_ptr(), KP, cout, Mpad, x8.data_ptr(), pad, cin, B,
                     y.data_ptr(), y8.data_ptr(), 1, bias.float().contiguous().to(dev).data_ptr(),
                     posb.float().contiguous().to(dev).data_ptr(), s_x.data_ptr(),
                     scales.data_ptr(), s_y.data_ptr(), amax_y.data_ptr(), 0, s)
    y8f = (y8.view(torch.float8_e4m3fn).float() * s_y).reshape(y.shape).to(torch.bfloat16)
    return (LY.from_frame(y, 1, cout), LY.from_frame(y8f, 1, cout), s_y.item(),
            amax_y.view(torch.float32).item())


def conv_dgrad(dz: torch.Tensor, w: torch.Tensor, aux: torch.Tensor, tiles=None) -> torch.Tensor:
    """dz [B,Cout,19,19], w OHWI [Cout,k,k,Cin], aux [B,Cin,19,19] (activation whose >0
    mask gates the result) -> dX*(aux>0) fp32 NCHW [B,Cin,19,19]."""
    h = hip()
    dev = w.device
    B, cout = dz.shape[:2]
    _, k, _, cin = w.shape
    pad = (k - 1) // 2
    npix = B * NPTS
    bm, bn = tiles or LY.pick_tiles(npix, cin)
    KPd, _, Mpad = LY.conv_dims(k, cout, cin, bm)
    dzf = LY.to_frame(dz.to(dev), max(1, pad))
    auxf = LY.to_frame(aux.to(dev), pad)
    out = LY.alloc_frame(B, cin, 1, dev)
    A = LY.dgrad_weight(w.float(), KPd, Mpad)
    h.conv_nt(h.EPI_DGRAD, k, bm, bn, A.data_ptr(), KPd, cin, Mpad, dzf.data_ptr(), max(1, pad),
              cout, npix, out.data_ptr(), 1, 0, 0, auxf.data_ptr(), pad, stream_handle())
    return LY.from_frame(out, 1, cin)


def conv_wgrad(dz: torch.Tensor, x: torch.Tensor, k: int, splits: int | None = None,
               cinp: int | None = None, with_bias: bool = False, algo: str = "auto"):
    """dW[co][kh][kw][ci] = sum_{b,p} dz[b,co,p] * x[b,ci,p+off] (fp32 OHWI).

    with_bias=True also returns the fused bias grads (gposb [361][co], gbias [co])."""
    h = hip()
    dev = dz.device
    B, cout = dz.shape[:2]
    cin = x.shape[1]
    cinp = cinp or LY.round_up(cin, 8)
    pad = (k - 1) // 2
    npix = B * NPTS
    _, KPw, _ = LY.conv_dims(k, cinp, cout, 128)
    Mpad = LY.round_up(cout, 128)
    if algo == "win":
        # sliding-window kernel (conv_wgrad_win.hip): 3x3, pad-1 frames, 64-co / 64-ci chunks
        assert k == 3 and cout % 64 == 0 and cinp % 64 == 0 and KPw >= 9 * cinp
        splits = splits or h.conv_wgrad_win_splits(
            1, cout, cinp, B, torch.cuda.get_device_properties(dev).multi_processor_count)
        dzf = LY.to_frame(dz, 1)
        xf = LY.to_frame(x.to(dev), 1, cinp)
        slab = torch.empty(splits * Mpad * KPw, dtype=torch.float32, device=dev)
        out = torch.empty((cout, k, k, cin), dtype=torch.float32, device=dev)
        table = torch.tensor([[dzf.data_ptr(), xf.data_ptr(), slab.data_ptr()]], dtype=torch.int64)
        s = stream_handle()
        h.conv_wgrad_win(table.data_ptr(), 1, cout, Mpad, cinp, B, KPw, splits, 0, s)
        h.wgrad_reduce(slab.data_ptr(), out.data_ptr(), splits, cout, Mpad, KPw, 9, cin, cinp,
                       0, 0, 0, 0, 0, s)
        torch.cuda.synchronize(dev)
        return out
    splits = splits or LY.pick_wgrad_splits(npix, KPw, Mpad,
                                             wgs_per_cu=h.conv_wgrad_wgs_per_cu_for(KPw),
                                             ktile=h.conv_wgrad_ktile(KPw))
    dzf = LY.to_frame(dz, max(1, pad))
    xf = LY.to_frame(x.to(dev), pad, cinp)
    slab = torch.empty(splits * Mpad * KPw, dtype=torch.float32, device=dev)
    out = torch.empty((cout, k, k, cin), dtype=torch.float32, device=dev)
    gp = torch.zeros((NPTS, cout), dtype=torch.float32, device=dev)
    gb = torch.zeros(cout, dtype=torch.float32, device=dev)
    nch = h.bias_chunks(B)
    bpart = torch.empty(nch * (NPTS + 19) * cout, dtype=torch.float32, device=dev)
    s = stream_handle()
    h.bias_grad_partial(dzf.data_ptr(), B, cout, max(1, pad), bpart.data_ptr(), s)
    h.conv_wgrad(k, dzf.data_ptr(), max(1, pad), cout, Mpad, xf.data_ptr(), pad, cinp, B,
                 KPw, splits, slab.data_ptr(), s)
    h.wgrad_reduce(slab.data_ptr(), out.data_ptr(), splits, cout, Mpad, KPw, k * k, cin, cinp,
                   bpart.data_ptr(), nch, gp.data_ptr(), gb.data_ptr(), 0, s)
    if with_bias:
        return out, gp, gb
    return out


def head(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor, posb: torch.Tensor,
         labels: torch.Tensor | None, head_relu: bool = True, train: bool = True,
         grad_scale: float | None = None):
    """Fused head.  x [B,C,19,19]; w [1,k,k,C].  Returns dict with loss[B], pred[B],
    logp[B,361] and (train) dz [B,C,19,19] (masked by x>0), gw, gbias, gposb."""
    h = hip()
    dev = w.device
    B, C = x.shape[:2]
    k = w.shape[1]
    pad = (k - 1) // 2
    xf = LY.to_frame(x.to(dev), pad)
    loss = torch.zeros(B, dtype=torch.float32, device=dev)
    pred = torch.zeros(B, dtype=torch.int32, device=dev)
    logp = torch.zeros((B, NPTS), dtype=torch.float32, device=dev)
    lab = labels.to(dev, torch.int32).contiguous() if labels is not None else None
    out = {"loss": loss, "pred": pred, "logp": logp}
    dzf = gw = gb = gp = gwp = dzb = None
    if train:
        dzf = LY.alloc_frame(B, C, 1, dev)
        gw = torch.zeros(k * k * C, dtype=torch.float32, device=dev)
        gb = torch.zeros(1, dtype=torch.float32, device=dev)
        gp = torch.zeros(NPTS, dtype=torch.float32, device=dev)
        gwp = torch.zeros((B, k * k * C), dtype=torch.float32, device=dev)
        dzb = torch.zeros((B, NPTS), dtype=torch.float32, device=dev)
    s = stream_handle()
    wc = w.float().contiguous()
    bc = bias.float().contiguous()
    pc = posb.float().contiguous()
    h.head(k, xf.data_ptr(), pad, C, B, wc.data_ptr(), bc.data_ptr(), pc.data_ptr(), _ptr(lab),
           loss.data_ptr(), pred.data_ptr(), logp.data_ptr(), _ptr(dzf), 1, _ptr(gwp), 0,
           _ptr(dzb), int(head_relu), float(grad_scale if grad_scale is not None else 1.0 / B), s)
    if train:
        h.head_reduce(dzb.data_ptr(), gwp.data_ptr(), B, k * k * C, gw.data_ptr(), gb.data_ptr(),
                      gp.data_ptr(), 0, s)
    if train:
        out.update(dz=LY.from_frame(dzf, 1, C), gw=gw.view(1, k, k, C), gbias=gb, gposb=gp)
    return out


def expand_features(planes: torch.Tensor, player: torch.Tensor, rank: torch.Tensor,
                    pad: int = 2, CP: int = 40) -> torch.Tensor:
    """planes uint8 [B,9,19,19] -> float NCHW [B,CP,19,19] via the GPU expansion kernel."""
    h = hip()
    dev = torch.device("cuda")
    B = planes.shape[0]
    pl = planes.to(dev, torch.uint8).contiguous()
    py = player.to(dev, torch.uint8).contiguous()
    rk = rank.to(dev, torch.uint8).contiguous()
    out = LY.alloc_frame(B, CP, pad, dev)
    h.expand_features(pl.data_ptr(), py.data_ptr(), rk.data_ptr(), out.data_ptr(), B, pad, CP,
                      stream_handle())
    return LY.from_frame(out, pad, CP)


def bias_grad(dz: torch.Tensor):
    """Pass 1 of the bias grads on the GPU, pass 2 summed here: (gposb [361][C], gbias [C])."""
    h = hip()
    B, C = dz.shape[:2]
    dzf = LY.to_frame(dz, 1)
    nch = h.bias_chunks(B)
    part = torch.empty(nch * (NPTS + 19) * C, dtype=torch.float32, device=dz.device)
    h.bias_grad_partial(dzf.data_ptr(), B, C, 1, part.data_ptr(), stream_handle())
    gp = part[:nch * NPTS * C].view(nch, NPTS, C).sum(0)
    gb = part[nch * NPTS * C:].view(nch * 19, C).sum(0)
    return gp, gb


def sgd_(p: torch.Tensor, g: torch.Tensor, lr: float, decay: float, steps: int = 1):
    h = hip()
    lrt = torch.tensor([lr], dtype=torch.float64, device=p.device)
    s = stream_handle()
    for _ in range(steps):
        h.sgd(p.data_ptr(), g.data_ptr(), p.numel(), lrt.data_ptr(), 1.0, 0, s)
        h.lr_decay(lrt.data_ptr(), decay, 0, s)
    return lrt


def weight_refresh(w: torch.Tensor, cinp: int, KP: int, Mpad: int, KPd: int = 0, Mpad_d: int = 0,
                   frag: bool = False):
    """bf16 operand layouts of OHWI weights w (weight_refresh_kernel).  frag=True (3x3,
    128 -> 128 only) also returns the conv_stack2 fragment-ordered forward / dgrad operands."""
    h = hip()
    cout, k, _, cin = w.shape
    wf = torch.zeros((Mpad, KP), dtype=torch.bfloat16, device=w.device)
    wd = torch.zeros((Mpad_d, KPd), dtype=torch.bfloat16, device=w.device) if KPd else None
    ff = fd = None
    if frag:
        ff = torch.zeros(cout * k * k * cin, dtype=torch.bfloat16, device=w.device)
        fd = torch.zeros_like(ff)
    tbl = np.array([[w.data_ptr(), wf.data_ptr(), _ptr(wd), cout, cin, k * k, cinp, KP, KPd, 0,
                     0, 0, 0, 0, 0, 0, _ptr(ff), _ptr(fd), 0, 0]],
                   dtype=np.int64)
    h.weight_refresh(tbl.ctypes.data, 1, stream_handle())
    torch.cuda.synchronize()
    if frag:
        return wf, wd, ff, fd
    return wf, wd
