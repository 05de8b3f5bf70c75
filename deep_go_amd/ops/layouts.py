"""Tensor layouts shared by the HIP kernels and their tests.

* Activation frames: zero-bordered NHWC bf16 ``[B][19+2p][19+2p][C]``.  The border is
  the conv zero padding (the reference's ``nn.SpatialZeroPadding``,
  ``experiments.lua:137``); kernels only ever write the 19x19 interior.
* Forward weights (MFMA A operand): bf16 ``[Mpad][KP]`` with ``k = tap*cinp + ci``.
* Dgrad weights: bf16 ``[CinPad][KPd]`` with ``k = (T-1-tap)*cout + co`` (flipped taps).
"""
from __future__ import annotations

import os

import math

import torch

BOARD = 19


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


def frame_dim(pad: int) -> int:
    return BOARD + 2 * pad


def alloc_frame(B: int, C: int, pad: int, device, dtype=torch.bfloat16) -> torch.Tensor:
    F = frame_dim(pad)
    return torch.zeros((B, F, F, C), dtype=dtype, device=device)


def frame_interior(frame: torch.Tensor, pad: int) -> torch.Tensor:
    return frame[:, pad:pad + BOARD, pad:pad + BOARD, :]


def to_frame(x_nchw: torch.Tensor, pad: int, C: int | None = None, device=None) -> torch.Tensor:
    B, c = x_nchw.shape[:2]
    C = C or c
    fr = alloc_frame(B, C, pad, device or x_nchw.device)
    frame_interior(fr, pad)[..., :c] = x_nchw.permute(0, 2, 3, 1).to(fr.dtype)
    return fr


def from_frame(frame: torch.Tensor, pad: int, C: int) -> torch.Tensor:
    return frame_interior(frame, pad)[..., :C].permute(0, 3, 1, 2).float()


def fwd_weight(w_ohwi: torch.Tensor, cinp: int, KP: int, Mpad: int) -> torch.Tensor:
    cout, kh, kw, cin = w_ohwi.shape
    out = torch.zeros((Mpad, KP), dtype=torch.bfloat16, device=w_ohwi.device)
    tmp = torch.zeros((cout, kh * kw, cinp), dtype=torch.float32, device=w_ohwi.device)
    tmp[:, :, :cin] = w_ohwi.reshape(cout, kh * kw, cin)
    out[:cout, :kh * kw * cinp] = tmp.reshape(cout, -1).to(torch.bfloat16)
    return out


def dgrad_weight(w_ohwi: torch.Tensor, KPd: int, Mpad: int) -> torch.Tensor:
    cout, kh, kw, cin = w_ohwi.shape
    T = kh * kw
    out = torch.zeros((Mpad, KPd), dtype=torch.bfloat16, device=w_ohwi.device)
    # [ci][T-1-t][co]
    t = w_ohwi.reshape(cout, T, cin).flip(1).permute(2, 1, 0).reshape(cin, T * cout)
    out[:cin, :T * cout] = t.to(torch.bfloat16)
    return out


def stack_frag(A: torch.Tensor) -> torch.Tensor:
    """conv_stack2 A-operand order of a [128][1152] operand matrix (fwd_weight / dgrad_weight
    of a 3x3 128 -> 128 layer, k = tap*128 + channel): K-step s = chunk*9 + tap covers columns
    tap*128 + chunk*64 .. +64; flat [s 18][wm 2][kk 2][i 4][lane 64][e 8] with row
    wm*64 + i*16 + (lane & 15), column base + kk*32 + (lane >> 4)*8 + e."""
    assert A.shape[0] >= 128 and A.shape[1] >= 1152
    a = A[:128, :1152].reshape(2, 4, 16, 9, 2, 2, 4, 8)   # wm i lr | tap chunk kk lq e
    # -> chunk tap | wm | kk | i | lq lr | e
    return a.permute(4, 3, 0, 5, 1, 6, 2, 7).reshape(-1).contiguous()


def stack_frag_linear(A: torch.Tensor, cout: int = 128) -> torch.Tensor:
    """conv_stack2's fused-first-layer A order (l1 mode; also conv_l1_frag) of a
    [cout][1024] operand matrix with LINEAR k (fwd_weight of the 5x5 40-channel first layer,
    k = tap*40 + c, zero-padded from 1000): flat [h cout/128][s 16][wm 2][kk 2][i 4][lane 64]
    [e 8] with row 128h + wm*64 + i*16 + (lane & 15), column s*64 + kk*32 + (lane >> 4)*8 + e."""
    assert cout % 128 == 0 and A.shape[0] >= cout and A.shape[1] >= 1024
    a = A[:cout, :1024].reshape(cout // 128, 2, 4, 16, 16, 2, 4, 8)   # h wm i lr | s kk lq e
    return a.permute(0, 4, 1, 5, 2, 6, 3, 7).reshape(-1).contiguous()


def stack_pbias_frag(bias: torch.Tensor, posb: torch.Tensor) -> torch.Tensor:
    """The forward stacks' epilogue table (weight_refresh pbias_frag): bf16(bias + posb) of
    [361][cout] (cout = 128h) as flat [h][24 px frags][wm 2][i 4][lane 64][4] with pixel
    jg*16 + (lane & 15) (clamped to 360) and channels 128h + wm*64 + i*16 + (lane >> 4)*4 + e."""
    cout = bias.numel()
    t = (posb.float() + bias.float()[None, :]).to(torch.bfloat16)            # [361][cout]
    p = torch.arange(24 * 16, device=t.device).clamp(max=360)
    t = t[p]                                                                 # [384][cout]
    a = t.reshape(24, 16, cout // 128, 2, 4, 4, 4)       # jg lr | h wm i lq e
    return a.permute(2, 0, 3, 4, 5, 1, 6).reshape(-1).contiguous()


def stack_frag_f8(w8: torch.Tensor) -> torch.Tensor:
    """conv_stack_f8 A-operand order of e4m3 forward weights ``w8`` [C co][9 taps][C ci]
    (uint8 bytes, C = 128 | 256).
    C = 256: flat [h 2][tap 9][c 2][wm 2][i 4][half 2][lane 64][e 16] with co = 128h + wm*64 +
    i*16 + (lane & 15), ci = 128c + 32*(lane >> 4) + 16*half + e (the MX-MFMA lane group g
    holds k = 32g .. 32g + 31; h = output pass, c = K chunk).
    C = 128 (half-major K-steps, the staggered schedule's order): unit n = 9*kh + tap (64
    channels kh of one tap) is K-step n // 2 in lane groups 2*(n % 2), +1: flat [st 9][wm 2]
    [i 4][half 2][lane 64][e 16] with lane group g = 2p + q holding unit 2*st + p, ci = 64*kh +
    32*q + 16*half + e."""
    C = w8.shape[0]
    assert C in (128, 256) and tuple(w8.shape) == (C, 9, C)
    if C == 128:
        a = w8.reshape(128, 9, 2, 2, 2, 16)                 # co | tap | kh q half e
        a = a.permute(0, 2, 1, 3, 4, 5).reshape(128, 18, 2, 2, 16)   # co | n = 9kh+tap | q..
        a = a.reshape(2, 4, 16, 9, 2, 2, 2, 16)             # wm i lr | st p | q half e
        return a.permute(3, 0, 1, 6, 4, 5, 2, 7).reshape(-1).contiguous()
    n = C // 128
    a = w8.reshape(n, 2, 4, 16, 9, n, 4, 2, 16)         # h wm i lr | tap | c lq half e
    return a.permute(0, 4, 5, 1, 2, 7, 6, 3, 8).reshape(-1).contiguous()


def conv_dims(k: int, cin_frame: int, cout: int, bm: int):
    """K/M padding for a conv whose input frame has ``cin_frame`` channels."""
    ngroups = k * k * cin_frame // 8
    KP = round_up(ngroups * 8, 64)
    KPw = round_up(ngroups * 8, 128)
    Mpad = round_up(cout, bm)
    return KP, KPw, Mpad


def gpt_magic(d: int) -> int:
    return (1 << 32) // d + 1


def pick_tiles(npix: int, cout: int, num_cus: int = 256) -> tuple[int, int]:
    """Choose (BM, BN) for the NT conv kernel: minimise quantised rounds x tile cost.

    2 workgroups fit per CU (64-80 KiB LDS each); a partially filled last round costs a
    whole round.  Larger tiles have better arithmetic intensity (eff factor)."""
    cands = [(128, 128, 1.0), (128, 192, 1.06), (64, 128, 0.8), (64, 256, 0.9)]
    best, best_cost = None, math.inf
    for bm, bn, eff in cands:
        if cout > 64 and bm == 64:
            continue
        if cout <= 64 and bm == 128:
            continue
        tiles = math.ceil(npix / bn) * math.ceil(cout / bm)
        rounds = math.ceil(tiles / (2 * num_cus))
        cost = rounds * bm * bn / eff
        if cost < best_cost:
            best, best_cost = (bm, bn), cost
    return best


def pick_wgrad_splits(npix: int, KPw: int, Mpad: int, num_cus: int = 256,
                      wgs_per_cu: int = 2, ktile: int = 128) -> int:
    """Split-K count for the im2col wgrad: one dispatch round of (k-tiles x m-tiles x
    splits) workgroups at ``wgs_per_cu`` resident workgroups per CU (hip().
    conv_wgrad_wgs_per_cu(): 2 for the 2-stage kernel)."""
    tiles = (KPw // ktile) * (Mpad // 128)
    target = max(1, (wgs_per_cu * num_cus) // tiles)
    max_split = max(1, npix // 256)
    return max(1, min(target, max_split))


def board_ok(k: int, cin_frame: int) -> bool:
    """The board-tiled kernel (conv_board.hip) handles 1x1/3x3 layers whose input frame
    has a multiple of 64 channels; everything else uses the pixel-tiled conv_nt kernel."""
    return k in (1, 3) and cin_frame % 64 == 0


def board_bm(cout: int) -> int:
    """M tile of the board kernel: 64 -> single halo image, two workgroups per CU (the
    epilogue of one overlaps the other's MFMAs); 128 -> one workgroup per CU.  DG_BOARD_BM
    overrides (A/B benchmarking)."""
    env = os.environ.get("DG_BOARD_BM")
    if env:
        return int(env)
    return 64