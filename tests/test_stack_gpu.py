"""The board-resident layer stack (csrc/kernels/conv_stack2.hip) against a plain
PyTorch fp32 oracle, layer by layer (teacher-forced: each layer's oracle input is the
kernel's own bf16 output of the layer below, so errors do not compound).

The stack computes, per layer l with operand matrix A_l [128][9*128] (k = tap*128 + c):
  out[r][p] = sum_{tap, c} A_l[r][tap*128 + c] * X[p + off(tap)][c]   (zero padded 19x19)
  EPI_FWD  : Y = relu(out + pbias)          (pbias = 0 here) and the ReLU bitmask
  EPI_DGRAD: Y = out * mask bit(r)          (mask = the random bitmask supplied)
Both epilogues see the same A, so one oracle covers the forward and the dgrad stack (for the
dgrad A holds the flipped, transposed weights).  Reference ops: experiments.lua:137-147.
"""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
C = 128


def _oracle(A, x_frame, mask, epi):
    """A [128][1152] bf16, x_frame [B][21][21][128] bf16 -> fp32 [B][19][19][128]."""
    from deep_go_amd.ops import layouts as LY
    x = LY.frame_interior(x_frame, 1).float().permute(0, 3, 1, 2)          # B C 19 19
    w = A[:C, :9 * C].float().reshape(C, 3, 3, C).permute(0, 3, 1, 2)    # r c kh kw
    out = F.conv2d(x.cpu(), w.cpu(), padding=1).to(DEV).permute(0, 2, 3, 1)  # CPU fp32 oracle
    if epi == "fwd":
        return out.relu()
    bits = ((mask.long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1)  # B 361 16 8
    return out * bits.reshape(out.shape[0], 19, 19, C).float()


@pytest.mark.parametrize("epi", ["fwd", "dgrad"])
def test_stack_layers_match_fp32_oracle(epi):
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    torch.manual_seed(3)
    B, NL = 6, 3
    KP = 9 * C
    x = LY.alloc_frame(B, C, 1, DEV)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=DEV).relu())
    As, ys, ms = [], [], []
    for _ in range(NL):
        As.append((torch.randn(C, KP, device=DEV) / (3 * C ** 0.5)).to(torch.bfloat16))
        ys.append(LY.alloc_frame(B, C, 1, DEV))
        ms.append(torch.randint(0, 256, (B, 361, 16), dtype=torch.uint8, device=DEV))
    pb = torch.zeros(24 * 2 * 4 * 64 * 4, dtype=torch.bfloat16, device=DEV)
    ops = [LY.stack_frag(a) for a in As]
    tab = np.array([[ops[i].data_ptr(), pb.data_ptr() if epi == "fwd" else 0, ys[i].data_ptr(),
                     ms[i].data_ptr()] for i in range(NL)], dtype=np.int64)
    masks_in = [m.clone() for m in ms]
    e = h.EPI_FWD if epi == "fwd" else h.EPI_DGRAD
    h.conv_stack2(e, tab.ctypes.data, NL, x.data_ptr(), 0, B, stream_handle())
    torch.cuda.synchronize()
    xin = x
    for l in range(NL):
        ref = _oracle(As[l], xin, masks_in[l], epi)
        got = LY.frame_interior(ys[l], 1).float()
        err = ((got - ref).abs().max() / (ref.abs().max() + 1e-6)).item()
        assert err < 1e-2, f"{epi} layer {l}: rel err {err:.3g}"
        # zero border untouched
        assert ys[l][:, 0].abs().sum().item() == 0 and ys[l][:, :, 0].abs().sum().item() == 0
        if epi == "fwd":  # bitmask written = nonzero of the bf16 output
            nz = (LY.frame_interior(ys[l], 1) != 0).reshape(B, 361, C // 8, 8).long()
            packed = (nz << torch.arange(8, device=DEV)).sum(-1).to(torch.uint8)
            assert torch.equal(packed, ms[l]), f"fwd layer {l}: mask"
        xin = ys[l]


def _q8(x):
    """e4m3 (OCP, RNE) rounding of x (|x| <= 448) as float32."""
    return x.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


def _q5(x):
    """e5m2 (RNE) rounding of x (|x| <= 57344) as float32."""
    return x.clamp(-57344.0, 57344.0).to(torch.float8_e5m2).float()


@pytest.mark.parametrize("C,nl,epi", [(128, 2, "fwd"), (128, 4, "fwd"), (256, 2, "fwd"),
                                      (256, 3, "fwd"), (128, 3, "dgrad"), (256, 2, "dgrad")])
def test_fp8_stack_matches_emulated_oracle(C, nl, epi):
    """conv_stack_f8 vs a PyTorch fp32 oracle that applies the same quantization.  Forward:
    layer l's input = e4m3(Y_{l-1} / s_x) (teacher-forced on the kernel's own dequantized bf16
    output, which re-quantizes to the exact bytes), weights e4m3(W / s_w),
    y = relu(s_x s_w acc + bias); non-last layers output bf16(e4m3(y / s_y) s_y), the last
    bf16(y); ReLU bits = nonzero outputs.  Backward-data (EPI_DGRAD): e5m2 gradients,
    y = s_x s_w acc * ReLU bit of the layer below, no bias.  Also: the |x| max of every
    quantized tensor is folded in, borders stay zero."""
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    torch.manual_seed(11)
    B = 5
    q = _q8 if epi == "fwd" else _q5
    qmax = 448.0 if epi == "fwd" else 57344.0
    npb = (C // 128) * 24 * 2 * 4 * 64 * 4
    x = LY.alloc_frame(B, C, 1, DEV)
    xi = torch.randn(B, 19, 19, C, device=DEV)
    LY.frame_interior(x, 1).copy_(xi.relu() if epi == "fwd" else 1e-3 * xi)
    # scales: s[0] = input, s[1 + l] = output of layer l (powers of two, as fp8_update_scales
    # guarantees: the kernel's scaled conversions rely on it); ws[l] = weight scales
    s = torch.empty(nl + 1, device=DEV)
    s[0] = 2.0 ** math.ceil(math.log2(x.float().abs().max().item() / qmax))
    ws = torch.empty(nl, device=DEV)
    amax = torch.zeros(nl + 1, dtype=torch.int32, device=DEV)
    W8, ys, ms, pbs = [], [], [], []
    for l in range(nl):
        w = torch.randn(C, 9, C, device=DEV) / (3 * C ** 0.5)
        ws[l] = w.abs().max() / 448.0
        s[1 + l] = 2.0 ** (-4 - l) if epi == "fwd" else 2.0 ** (-20 - l)
        W8.append((w / ws[l]).clamp(-448, 448).to(torch.float8_e4m3fn))
        ys.append(LY.alloc_frame(B, C, 1, DEV))
        ms.append(torch.zeros(B, 361, C // 8, dtype=torch.uint8, device=DEV) if epi == "fwd"
                  else torch.randint(0, 256, (B, 361, C // 8), dtype=torch.uint8, device=DEV))
        pbs.append(torch.zeros(npb, dtype=torch.bfloat16, device=DEV))
    frags = [LY.stack_frag_f8(w8.view(torch.uint8)) for w8 in W8]
    masks_in = [m.clone() for m in ms]
    f4 = 4
    tab = np.array([[frags[i].data_ptr(), pbs[i].data_ptr() if epi == "fwd" else 0,
                     ys[i].data_ptr(), ms[i].data_ptr(), s.data_ptr() + f4 * i,
                     ws.data_ptr() + f4 * i, s.data_ptr() + f4 * (i + 1),
                     amax.data_ptr() + f4 * (i + 1)] for i in range(nl)], dtype=np.int64)
    e = h.EPI_FWD if epi == "fwd" else h.EPI_DGRAD
    h.conv_stack_f8(C, e, tab.ctypes.data, nl, x.data_ptr(), s.data_ptr(), amax.data_ptr(), B,
                    stream_handle())
    torch.cuda.synchronize()
    amax_f = amax.view(torch.float32)
    assert abs(amax_f[0].item() - x.float().abs().max().item()) < 1e-6 * qmax
    xin = x
    for l in range(nl):
        s_x, s_w, s_y = s[l], ws[l], s[l + 1]
        xq = q(LY.frame_interior(xin, 1).float() / s_x).permute(0, 3, 1, 2)
        wq = W8[l].float().reshape(C, 3, 3, C).permute(0, 3, 1, 2)
        v = (F.conv2d(xq.cpu(), wq.cpu(), padding=1).to(DEV)            # CPU fp32 oracle
             * (s_x * s_w)).permute(0, 2, 3, 1)
        if epi == "fwd":
            v = v.relu()
        else:
            bits = (masks_in[l].long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1
            v = v * bits.reshape(B, 19, 19, C).float()
        got = LY.frame_interior(ys[l], 1).float()
        last = l == nl - 1
        ref = v if last else q(v / s_y) * s_y
        err = ((got - ref).abs().max() / (ref.abs().max() + 1e-30)).item()
        # accumulation-order differences may move a value across an fp8 rounding boundary
        # (one e4m3 step = 1/16 .. 1/8 relative, e5m2 1/8 .. 1/4); the bulk must match to
        # bf16 rounding
        close = ((got - ref).abs() <= 1e-2 * ref.abs() + 1e-30).float().mean().item()
        tol = 1e-2 if last else (0.07 if epi == "fwd" else 0.14)
        assert err < tol and close > 0.99, (l, err, close)
        if not last:
            assert abs(amax_f[l + 1].item() - v.abs().max().item()) <= 1e-3 * v.abs().max().item()
        if epi == "fwd":
            nz = (LY.frame_interior(ys[l], 1) != 0).reshape(B, 361, C // 8, 8).long()
            assert torch.equal((nz << torch.arange(8, device=DEV)).sum(-1).to(torch.uint8), ms[l])
        assert ys[l][:, 0].abs().sum().item() == 0 and ys[l][:, :, 0].abs().sum().item() == 0
        xin = ys[l]


@pytest.mark.parametrize("C", [128, 256])
def test_fp8_dgrad_stochastic_rounding_is_unbiased(C):
    """The e5m2 backward-data stack with stochastic rounding (conv_stack_f8_dgrad, sr_step =
    the device step counter): deterministic for one step, different across steps, and
    unbiased — the mean over 32 steps of the last layer's output approaches the unquantized
    fp32 chain far closer than round-to-nearest-even does (whose error is systematic)."""
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    torch.manual_seed(5)
    B, nl = 4, 2
    x = LY.alloc_frame(B, C, 1, DEV)
    LY.frame_interior(x, 1).copy_(1e-3 * torch.randn(B, 19, 19, C, device=DEV))
    s = torch.empty(nl + 1, device=DEV)
    s[0] = 2.0 ** math.ceil(math.log2(x.float().abs().max().item() / 57344.0))
    ws = torch.empty(nl, device=DEV)
    amax = torch.zeros(nl + 1, dtype=torch.int32, device=DEV)
    W8, ys, ms = [], [], []
    for l in range(nl):
        w = torch.randn(C, 9, C, device=DEV) / (3 * C ** 0.5)
        ws[l] = w.abs().max() / 448.0
        s[1 + l] = 2.0 ** (-20 - l)
        W8.append((w / ws[l]).clamp(-448, 448).to(torch.float8_e4m3fn))
        ys.append(LY.alloc_frame(B, C, 1, DEV))
        ms.append(torch.randint(0, 256, (B, 361, C // 8), dtype=torch.uint8, device=DEV))
    frags = [LY.stack_frag_f8(w8.view(torch.uint8)) for w8 in W8]
    f4 = 4
    tab = np.array([[frags[i].data_ptr(), 0, ys[i].data_ptr(), ms[i].data_ptr(),
                     s.data_ptr() + f4 * i, ws.data_ptr() + f4 * i, s.data_ptr() + f4 * (i + 1),
                     amax.data_ptr() + f4 * (i + 1)] for i in range(nl)], dtype=np.int64)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)

    def run(sr):
        h.conv_stack_f8_dgrad(C, tab.ctypes.data, nl, x.data_ptr(), s.data_ptr(),
                              amax.data_ptr(), B, 0, step.data_ptr() if sr else 0,
                              stream_handle())
        torch.cuda.synchronize()
        return LY.frame_interior(ys[-1], 1).float().clone()

    # unquantized fp32 chain with the same e4m3 weights and masks
    v = LY.frame_interior(x, 1).float()
    for l in range(nl):
        wq = W8[l].float().reshape(C, 3, 3, C).permute(0, 3, 1, 2) * ws[l].item()
        v = F.conv2d(v.permute(0, 3, 1, 2).cpu(), wq.cpu(), padding=1).to(DEV).permute(0, 2, 3, 1)
        bits = (ms[l].long().unsqueeze(-1) >> torch.arange(8, device=DEV)) & 1
        v = v * bits.reshape(B, 19, 19, C).float()
    ref = v
    rel = lambda a: ((a - ref).norm() / ref.norm()).item()  # noqa: E731
    rne = run(False)
    step.fill_(7)
    a, b = run(True), run(True)
    assert torch.equal(a, b)                    # one step: deterministic
    step.fill_(8)
    assert not torch.equal(run(True), a)        # another step: other rounding
    acc = torch.zeros_like(ref)
    errs = []
    for k in range(32):
        step.fill_(100 + k)
        y = run(True)
        errs.append(rel(y))
        acc += y
    e_rne, e_mean = rel(rne), rel(acc / 32)
    print(f"C={C}: rne {e_rne:.4f} single-SR {np.mean(errs):.4f} mean-of-32 {e_mean:.4f}")
    assert max(errs) < 3 * e_rne               # one SR draw: same order as nearest-even
    assert e_mean < 0.4 * e_rne                 # the mean converges: unbiased


@pytest.mark.parametrize("kind", ["bf16", "fp8"])
def test_staggered_schedules_bit_identical(kind):
    """The staggered two-group schedules (conv_stack2.hip / conv_stack_f8.hip STAG: LDS
    counters instead of the per-layer barriers; fp8 C = 128 with a double-buffered image) give
    exactly the barrier schedules' outputs: every layer's frame, the forward's ReLU bits and
    (fp8) the |y| maxima, forward and backward-data (e5m2 with stochastic rounding)."""
    from deep_go_amd.ops import layouts as LY
    from deep_go_amd.ops.native import hip, stream_handle
    h = hip()
    torch.manual_seed(21)
    B, NL = 8, 4
    x = LY.alloc_frame(B, C, 1, DEV)
    LY.frame_interior(x, 1).copy_(torch.randn(B, 19, 19, C, device=DEV).relu())
    ys = [LY.alloc_frame(B, C, 1, DEV) for _ in range(NL)]
    ms = [torch.randint(0, 256, (B, 361, C // 8), dtype=torch.uint8, device=DEV)
          for _ in range(NL)]
    md = [m.clone() for m in ms]
    pbs = [(0.01 * torch.randn(24 * 2 * 4 * 64 * 4, device=DEV)).to(torch.bfloat16)
           for _ in range(NL)]
    s = stream_handle()
    if kind == "bf16":
        ops = [LY.stack_frag((torch.randn(C, 9 * C, device=DEV) / (3 * C ** 0.5))
                             .to(torch.bfloat16)) for _ in range(NL)]

        def run(fwd, stag):
            h.conv_stack2_set_sched(stag, 1, 0)
            tab = np.array([[ops[i].data_ptr(), pbs[i].data_ptr() if fwd else 0,
                             ys[i].data_ptr(), (ms if fwd else md)[i].data_ptr()]
                            for i in range(NL)], dtype=np.int64)
            h.conv_stack2(h.EPI_FWD if fwd else h.EPI_DGRAD, tab.ctypes.data, NL,
                          x.data_ptr(), 0, B, s)
        default = (2, 1, 0)
        outs = lambda fwd: ys + (ms if fwd else [])  # noqa: E731
    else:
        w8 = [LY.stack_frag_f8(torch.randint(0, 0x78, (C, 9, C), dtype=torch.uint8,
                                             device=DEV)) for _ in range(NL)]
        sc = torch.full((NL + 1,), 2.0 ** -6, device=DEV)
        amax = torch.zeros(NL + 1, dtype=torch.int32, device=DEV)
        step = torch.full((1,), 5, dtype=torch.int64, device=DEV)
        # the production variants (as the training step): fp8 copies of every non-last output
        # (y8), the last layer's bf16 frame only
        x8 = [torch.zeros(B * 448 * C, dtype=torch.uint8, device=DEV) for _ in range(NL)]
        y8 = np.array([x8[0].data_ptr()] + [x8[i + 1].data_ptr() if i + 1 < NL else 0
                                            for i in range(NL)], dtype=np.int64)

        def run(fwd, stag):
            h.conv_stack_f8_set_sched(stag, 0)
            tab = np.array([[w8[i].data_ptr(), pbs[i].data_ptr() if fwd else 0,
                             ys[i].data_ptr() if i == NL - 1 else 0,
                             (ms if fwd else md)[i].data_ptr(), sc.data_ptr() + 4 * i,
                             sc.data_ptr() + 4 * i, sc.data_ptr() + 4 * (i + 1),
                             amax.data_ptr() + 4 * (i + 1)] for i in range(NL)], dtype=np.int64)
            if fwd:
                h.conv_stack_f8_y8(C, h.EPI_FWD, tab.ctypes.data, NL, x.data_ptr(),
                                   sc.data_ptr(), amax.data_ptr(), B, y8.ctypes.data, s)
            else:
                h.conv_stack_f8_dgrad(C, tab.ctypes.data, NL, x.data_ptr(), sc.data_ptr(),
                                      amax.data_ptr(), B, y8.ctypes.data, step.data_ptr(), s)
        default = (1, 0)
        outs = lambda fwd: x8 + [ys[-1], amax] + (ms if fwd else [])  # noqa: E731
    try:
        for fwd in (True, False):
            got = []
            for stag in (0, 1):
                for t in outs(fwd):
                    t.zero_()
                run(fwd, stag)
                torch.cuda.synchronize()
                got.append([t.clone() for t in outs(fwd)])
            for k, (a, b) in enumerate(zip(*got)):
                assert torch.equal(a, b), (kind, "fwd" if fwd else "dgrad", k)
            assert any(t.abs().sum().item() > 0 for t in got[0][:NL])
    finally:
        if kind == "bf16":
            h.conv_stack2_set_sched(*default)
        else:
            h.conv_stack_f8_set_sched(*default)
