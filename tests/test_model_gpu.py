"""Whole-model checks on the GPU: HipGoNet fwd/bwd vs the fp32 PyTorch oracle with the
same weights, graph replay == eager, and loss decreasing (SURVEY.md §4.3 model-level)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _setup(layers=4, ch=64, B=5, seed=0, **kw):
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet
    cfg = ExperimentConfig(numLayers=layers, channelSize=ch, batchSize=B, seed=seed, **kw)
    net = HipGoNet(cfg, B, device="cuda")
    planes, player, rank, labels = random_planes(B, seed=seed + 7)
    net.set_batch(torch.from_numpy(planes).cuda(), torch.from_numpy(player).cuda(),
                  torch.from_numpy(rank).cuda(), torch.from_numpy(labels).cuda())
    return cfg, net, (planes, player, rank, labels)


def _oracle(net, data):
    from deep_go_amd.data.features import expand_batch
    from deep_go_amd.models.gocnn import reference_forward
    planes, player, rank, labels = data
    x = torch.from_numpy(expand_batch(planes, player, rank, ko=net.cfg.ko_plane))
    # oracle sees the bf16-rounded weights the kernels use
    flat = net.params.detach().cpu().clone()
    for spec in net.layout.layers[:-1]:
        w = flat[spec.w_off:spec.w_off + spec.w_numel]
        w.copy_(w.to(torch.bfloat16).float())
    flat.requires_grad_(True)
    logp = reference_forward(net.layout, flat, x, head_relu=net.cfg.head_relu)
    loss = F.nll_loss(logp, torch.from_numpy(labels).long())
    (g,) = torch.autograd.grad(loss, flat)
    return loss.item(), logp.argmax(1), g


class _RoundBF16(torch.autograd.Function):
    """bf16 rounding of a stored tensor: the activation frame in the forward AND the dZ frame
    flowing back through it (the kernels store both in bf16)."""
    @staticmethod
    def forward(ctx, x):
        return x.to(torch.bfloat16).float()

    @staticmethod
    def backward(ctx, g):
        return g.to(torch.bfloat16).float()


def _oracle_bf16(net, data):
    """fp32 oracle that stores what the kernels store in bf16: hidden weights, activations
    and dZ frames in bf16, and bias + position bias as ONE bf16 table where the layer's
    epilogue reads that table (net.pbias).  What remains is accumulation order (fp32 MFMA
    sums), so the error should not grow with depth."""
    from deep_go_amd.config import NUM_POINTS
    from deep_go_amd.data.features import expand_batch
    planes, player, rank, labels = data
    lay = net.layout
    x = torch.from_numpy(expand_batch(planes, player, rank)).to(torch.bfloat16).float()
    flat = net.params.detach().cpu().clone().requires_grad_(True)
    n = len(lay.layers)
    h = x
    for L in lay.layers:
        head = L.index == n - 1
        w = lay.weight(flat, L.index).permute(0, 3, 1, 2)
        if not head:
            w = w + (w.detach().to(torch.bfloat16).float() - w.detach())
        z = F.conv2d(h, w, padding=L.pad)
        bias = lay.bias(flat, L.index).reshape(1, L.cout, 1, 1) + \
            lay.pos_bias(flat, L.index).t().reshape(1, L.cout, 19, 19)
        if not head and net.pbias[L.index] is not None:
            bias = bias + (bias.detach().to(torch.bfloat16).float() - bias.detach())
        z = z + bias
        if not head or net.cfg.head_relu:
            z = F.relu(z)
        h = z if head else _RoundBF16.apply(z)
    logp = F.log_softmax(h.reshape(h.shape[0], NUM_POINTS), dim=1)
    loss = F.nll_loss(logp, torch.from_numpy(labels).long())
    (g,) = torch.autograd.grad(loss, flat)
    return loss.item(), logp.argmax(1), g


@pytest.mark.parametrize("layers,ch,B", [(4, 128, 3), (12, 128, 2), (12, 256, 2)])
def test_model_matches_bf16_storage_oracle(layers, ch, B):
    """Flagship shapes (12x128, 12x256) end to end against the bf16-storage oracle.  The
    oracle rounds where the kernels round but cannot round the SAME values (its fp32 sums
    differ in order), so a few ReLU gates near zero flip and the difference compounds down the
    backward: measured max per-tensor gradient error 6.4% (12x128, since the first layer also
    reads the bf16 bias table: the same flips, different ones) / 4.7% (12x256), 0.17% at 4
    layers.  The error grows with the distance from the output (12x128: the last two layers
    0.0002-0.2%, layers 9-10 ~2.7%, layers 1-8 5-6%, median 5.3%), so: the last two layers'
    tensors — no compounding yet — within 1e-2 (a kernel bug shows there), and at 12 layers
    the rest bounded by the measured spread (worst 0.15, median 0.08: a benign reorder of a
    reduction moves the flips); at 4 layers everything within 1e-2.  The per-layer,
    depth-independent bound is test_layerwise_teacher_forced."""
    cfg, net, data = _setup(layers, ch, B, seed=4)
    net.forward_backward()
    torch.cuda.synchronize()
    loss_ref, pred_ref, g_ref = _oracle_bf16(net, data)
    assert abs(net.mean_loss().item() - loss_ref) < 2e-3 * max(1.0, abs(loss_ref))
    g = net.grads.cpu()
    errs = {}
    for name, off, n in net.layout.tensor_ranges():
        a, b = g[off:off + n], g_ref[off:off + n]
        errs[name] = ((a - b).norm() / (b.norm() + 1e-12)).item()
    worst = max(errs, key=errs.get)
    print("max per-tensor grad rel err", worst, errs[worst])
    import json
    import os
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/oracle_errs_{layers}x{ch}.json", "w") as f:
        json.dump(errs, f, indent=0)
    assert errs[worst] < (1e-2 if layers <= 4 else 0.15), errs
    assert float(np.median(list(errs.values()))) < (1e-2 if layers <= 4 else 0.08), errs
    # (names conv<i>.weight / conv<i>.bias / pos_bias<i>, i = 1..layers)
    tail = {k: v for k, v in errs.items()
            if int("".join(c for c in k.split(".")[0] if c.isdigit())) >= layers - 1}
    assert tail and max(tail.values()) < 1e-2, tail


def _interior(frame, pad):
    return frame[:, pad:pad + 19, pad:pad + 19, :].float().permute(0, 3, 1, 2).cpu()


@pytest.mark.parametrize("layers,ch,B", [(12, 128, 4), (12, 256, 2), (6, 64, 4)])
def test_layerwise_teacher_forced(layers, ch, B):
    """Every layer's kernels against an fp32 oracle fed with the kernels' OWN stored inputs
    (activation, dZ and mask frames), so nothing compounds: forward output, weight / bias /
    position-bias gradients and the dgrad of each layer of the flagship shapes within a
    depth-independent bound (bf16 output rounding: 2^-8 relative per element)."""
    from deep_go_amd.data.features import expand_batch
    cfg, net, data = _setup(layers, ch, B, seed=9)
    net.forward_backward()
    # (the training launch with the fused head does not write the last hidden layer's
    # activation frame; the evaluation forward does, with the same kernel arithmetic)
    net.forward()
    torch.cuda.synchronize()
    planes, player, rank, labels = data
    lay = net.layout
    flat = net.params.detach().cpu()
    g = net.grads.cpu()
    x0 = torch.from_numpy(expand_batch(planes, player, rank)).to(torch.bfloat16).float()
    n = len(lay.layers)

    def rel(a, b):
        return ((a - b).norm() / (b.norm() + 1e-20)).item()
    worst = {}
    for L in lay.layers[:-1]:
        i = L.index
        xin = (x0 if i == 0 else _interior(net.act[i - 1], lay.layers[i].pad)).requires_grad_(True)
        w = lay.weight(flat, i).permute(0, 3, 1, 2).to(torch.bfloat16).float().requires_grad_(True)
        bias = lay.bias(flat, i).reshape(1, -1, 1, 1) + lay.pos_bias(flat, i).t().reshape(1, -1, 19, 19)
        if net.pbias[i] is not None:
            bias = bias.to(torch.bfloat16).float()
        bias.requires_grad_(True)
        z = F.conv2d(xin, w, padding=L.pad) + bias
        y = F.relu(z)
        y_gpu = _interior(net.act[i], lay.layers[i + 1].pad)
        e_fwd = rel(y_gpu, y.detach())
        dz = _interior(net.dz[i], net.dzp[i])
        gx, gw, gb = torch.autograd.grad(z, (xin, w, bias), dz)
        e_w = rel(g[L.w_off:L.w_off + L.w_numel].view(L.cout, L.k, L.k, L.cin).permute(0, 3, 1, 2), gw)
        e_b = rel(g[L.b_off:L.b_off + L.cout], gb.sum((0, 2, 3)))
        e_pb = rel(g[L.pos_off:L.pos_off + 361 * L.cout].view(361, L.cout).t().reshape(L.cout, 19, 19), gb.sum(0))
        e_dx = 0.0
        if i > 0:
            mask = (_interior(net.act[i - 1], lay.layers[i].pad) > 0).float()
            e_dx = rel(_interior(net.dz[i - 1], net.dzp[i - 1]), gx * mask)
        worst[i] = (e_fwd, e_w, e_b, e_pb, e_dx)
    print({i: tuple(round(v, 5) for v in e) for i, e in worst.items()})
    for i, (e_fwd, e_w, e_b, e_pb, e_dx) in worst.items():
        assert e_fwd < 4e-3, (i, "fwd", e_fwd)
        assert max(e_w, e_b, e_pb) < 2e-3, (i, "wgrad", e_w, e_b, e_pb)
        assert e_dx < 4e-3, (i, "dgrad", e_dx)


@pytest.mark.parametrize("layers,ch,B", [(3, 64, 5), (4, 128, 3), (6, 64, 8)])
def test_model_matches_oracle(layers, ch, B):
    cfg, net, data = _setup(layers, ch, B)
    net.forward_backward()
    torch.cuda.synchronize()
    loss_ref, pred_ref, g_ref = _oracle(net, data)
    assert abs(net.mean_loss().item() - loss_ref) < 2e-2 * max(1.0, abs(loss_ref))
    g = net.grads.cpu()
    lay = net.layout
    for name, off, n in lay.tensor_ranges():
        a, b = g[off:off + n], g_ref[off:off + n]
        err = (a - b).norm() / (b.norm() + 1e-12)
        assert err < 0.08, (name, err.item())


def _mark_ko(data):
    """A simple-ko mark (liberty plane = KO_MARK) at one empty point per board."""
    planes = data[0].copy()
    for b in range(planes.shape[0]):
        e = np.flatnonzero(planes[b, 0].reshape(-1) == 0)[3 * b + 1]
        planes[b, 1].reshape(-1)[e] = 255
    return (planes,) + tuple(data[1:])


def _set(net, data):
    net.set_batch(*(torch.from_numpy(a).cuda() for a in data))


@pytest.mark.parametrize("layers,ch,B", [(3, 64, 5), (4, 128, 3)])
def test_ko_plane_model_matches_oracle(layers, ch, B):
    """ko_plane=1: a 38-plane first layer whose plane 37 is the ko mark, through the same
    kernels (the mark is expanded into padded input channel 37)."""
    cfg, net, data = _setup(layers, ch, B, ko_plane=True)
    assert net.layout.layers[0].cin == 38
    data = _mark_ko(data)
    _set(net, data)
    net.forward_backward()
    torch.cuda.synchronize()
    loss_ref, _, g_ref = _oracle(net, data)
    assert abs(net.mean_loss().item() - loss_ref) < 2e-2 * max(1.0, abs(loss_ref))
    g = net.grads.cpu()
    for name, off, n in net.layout.tensor_ranges():
        a, b = g[off:off + n], g_ref[off:off + n]
        err = (a - b).norm() / (b.norm() + 1e-12)
        assert err < 0.08, (name, err.item())
    # the ko-plane weights get a real gradient
    L0 = net.layout.layers[0]
    w0 = g[L0.w_off:L0.w_off + L0.w_numel].view(L0.cout, -1, 38)  # [cout][k*k][cin]
    assert w0[:, :, 37].abs().sum().item() > 0


@pytest.mark.parametrize("ch", [64, 128])
def test_37_plane_model_ignores_ko_mark(ch):
    """Without ko_plane the mark changes nothing: bit-identical loss and gradients (d = 64:
    the VALU head's LDS float atomics sum in a varying order — within 1e-5 then)."""
    cfg, net, data = _setup(4, ch, 4)
    net.forward_backward()
    torch.cuda.synchronize()
    loss0, g0 = net.mean_loss().item(), net.grads.clone()
    _set(net, _mark_ko(data))
    net.forward_backward()
    torch.cuda.synchronize()
    if ch >= 128:
        assert net.mean_loss().item() == loss0
        assert torch.equal(net.grads, g0)
    else:
        assert abs(net.mean_loss().item() - loss0) < 1e-6
        assert torch.allclose(net.grads, g0, rtol=1e-5, atol=1e-7)


def test_every_gradient_is_written_each_step():
    """The step does not zero the gradient buffer: all entries must be (over)written."""
    cfg, net, data = _setup(4, 64, 5)
    net.forward_backward()
    torch.cuda.synchronize()
    g0 = net.grads.clone()
    # poison every real gradient entry (the alignment padding between tensors is zero from
    # allocation and never touched)
    for _, off, n in net.layout.tensor_ranges():
        net.grads[off:off + n] = float("nan")
    net.forward_backward()
    torch.cuda.synchronize()
    assert torch.isfinite(net.grads).all()
    assert torch.allclose(net.grads, g0, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("layers,ch,B", [(4, 64, 6), (6, 128, 4), (12, 128, 3)])
def test_graph_replay_matches_eager(layers, ch, B):
    """SegmentedStep.__call__ without buckets replays backward + optimizer as ONE graph
    (full_graph); parameters and the decayed LR match the eager train_step."""
    from deep_go_amd.models.hip_model import SegmentedStep
    cfg, net, data = _setup(layers, ch, B)
    p0 = net.params.clone()
    net.train_step()
    torch.cuda.synchronize()
    p_eager = net.params.clone()
    lr_eager = net.lr.item()
    # reset and replay through graphs
    net.params.copy_(p0)
    net.lr.fill_(cfg.rate)
    net.refresh_weights()
    step = SegmentedStep(net, None, use_graphs=True)
    assert step.full_graph is not None
    net.params.copy_(p0)
    net.lr.fill_(cfg.rate)
    net.refresh_weights()
    step()
    torch.cuda.synchronize()
    # the graph replays the eager launch sequence; every reduction in the default path is
    # deterministic (slab reduces, two-pass bias sums, the MFMA head's reduce), so the
    # updates are expected bit-identical — the tolerance only admits last-bit differences
    d = (net.params - p_eager).abs().max().item()
    assert d < 1e-5, d
    assert abs(net.lr.item() - lr_eager) < 1e-15


@pytest.mark.parametrize("layers,ch,B", [(4, 128, 6), (6, 128, 3)])
def test_side_stream_backward_matches_single_stream(layers, ch, B, monkeypatch):
    """The weight-gradient chain on a side stream (HipGoNet.backward_layer) must give the
    same gradients as the single-stream order, eager and inside a segmented graph with a
    DP-style bucket boundary."""
    from deep_go_amd.models.hip_model import SegmentedStep
    monkeypatch.setenv("DG_SIDE_STREAM", "0")
    _, net0, _ = _setup(layers, ch, B)
    net0.forward_backward()
    torch.cuda.synchronize()
    g0 = net0.grads.clone()
    monkeypatch.setenv("DG_SIDE_STREAM", "bias")
    _, net1, _ = _setup(layers, ch, B)
    assert net1.side is not None
    net1.forward_backward()
    torch.cuda.synchronize()
    assert torch.allclose(net1.grads, g0, rtol=1e-5, atol=1e-7)

    class _Buckets:  # fake bucketer: two buckets, no communication
        buckets = [(0, 0, 2), (0, 0, 0)]

        def fire(self, b):
            pass

        def wait(self):
            pass
    step = SegmentedStep(net1, _Buckets(), use_graphs=True)
    assert len(step.graphs) >= 2
    # segments whose launches were all grouped away are not captured (no empty graphs)
    assert all((g is None) == (n == 0) for g, n in zip(step.graphs, step.seg_launches))
    step.forward_backward()
    torch.cuda.synchronize()
    assert torch.allclose(net1.grads, g0, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("layers", [4, 6])
def test_fused_forward_stack_matches_per_layer(layers, monkeypatch):
    """conv_stack2_fwd (board-resident multi-layer forward) computes the per-layer board
    kernels' exact MFMA sequence: activations, masks and loss are bit-identical."""
    monkeypatch.setenv("DG_STACK", "0")
    _, n0, _ = _setup(layers, 128, 5, seed=6)
    monkeypatch.setenv("DG_STACK", "1")
    _, n1, _ = _setup(layers, 128, 5, seed=6)
    assert len(n1.stack) == layers - 2 and not n0.stack
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    # (the training launch with the fused head skips the last hidden layer's frame: nothing
    # in training reads it; the evaluation forward writes it)
    for a0, a1 in zip(n0.act[:-1], n1.act[:-1]):
        assert torch.equal(a0, a1)
    for m0, m1 in zip(n0.relu_mask, n1.relu_mask):
        if m0 is not None:
            assert torch.equal(m0, m1)
    assert torch.equal(n0.loss, n1.loss)
    g0, g1 = n0.grads.clone(), n1.grads.clone()
    n0.forward()
    n1.forward()
    torch.cuda.synchronize()
    assert torch.equal(n0.act[-1], n1.act[-1])
    # (the two paths group the weight-gradient split-K partials differently: fp32 summation
    # order only)
    assert torch.allclose(g0, g1, rtol=1e-5, atol=1e-8)


def test_layer2_matches_board_kernel_at_256(monkeypatch):
    """d = 256 bf16 hidden layers on conv_layer2.hip (fragment-ordered weights in VGPRs, chunk
    images double-buffered in LDS) run the board kernel's exact MFMA sequence, bias table and
    ReLU-mask gating: activations, masks, every dZ and the gradients are bit-identical to
    DG_LAYER2=0 (conv_board.hip), forward and backward-data."""
    monkeypatch.setenv("DG_LAYER2", "0")
    _, n0, _ = _setup(5, 256, 4, seed=31)
    monkeypatch.setenv("DG_LAYER2", "1")
    _, n1, _ = _setup(5, 256, 4, seed=31)
    l2 = (n1.h.conv_layer2, n1.h.conv_layer2_multi)
    assert any(f in l2 for f, _ in n1._fwd)
    assert not any(f in l2 for f, _ in n0._fwd)
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    for a0, a1 in zip(n0.act, n1.act):
        assert torch.equal(a0, a1)
    for m0, m1 in zip(n0.relu_mask, n1.relu_mask):
        if m0 is not None:
            assert torch.equal(m0, m1)
    for d0, d1 in zip(n0.dz, n1.dz):
        assert torch.equal(d0, d1)
    assert torch.equal(n0.loss, n1.loss)
    assert torch.allclose(n0.grads, n1.grads, rtol=1e-5, atol=1e-8)


def test_layer2_multi_matches_per_layer_launches(monkeypatch):
    """conv_layer2_multi (a run of d = 256 layers in one launch, one workgroup per board, the
    second output half on a prefetched input chunk) is bit-identical to the per-layer
    conv_layer2 launches at 12 layers: activations, masks, every dZ, loss and gradients."""
    monkeypatch.setenv("DG_LAYER2_MULTI", "0")
    _, n0, _ = _setup(12, 256, 6, seed=41)
    monkeypatch.setenv("DG_LAYER2_MULTI", "1")
    _, n1, _ = _setup(12, 256, 6, seed=41)
    h = n1.h
    assert sum(f is h.conv_layer2_multi for f, _ in n1._fwd) == 1
    assert sum(f is h.conv_layer2_multi for f, _ in n1._bwd_pre) == 1
    assert not any(f is h.conv_layer2 for f, _ in n1._fwd + n1._bwd_pre)
    for _ in range(2):
        n0.forward_backward()
        n1.forward_backward()
    torch.cuda.synchronize()
    for a0, a1 in zip(n0.act, n1.act):
        assert torch.equal(a0, a1)
    for m0, m1 in zip(n0.relu_mask, n1.relu_mask):
        if m0 is not None:
            assert torch.equal(m0, m1)
    for d0, d1 in zip(n0.dz, n1.dz):
        assert torch.equal(d0, d1)
    assert torch.equal(n0.loss, n1.loss)
    assert torch.allclose(n0.grads, n1.grads, rtol=1e-5, atol=1e-8)

@pytest.mark.parametrize("ch", [128, 256])
def test_layer0_side_chain_eager_matches_graph(ch):
    """Layer 0's gradient chain on the side stream (after the last group's bias partials)
    gives the same gradients eagerly and through the one-graph step."""
    from deep_go_amd.models.hip_model import SegmentedStep
    _, net, _ = _setup(12, ch, 6, seed=43)
    assert net._l0_side_at is not None
    p0 = net.params.clone()
    net.forward_backward()
    torch.cuda.synchronize()
    g = net.grads.clone()
    net.load_params(p0)
    step = SegmentedStep(net, None, use_graphs=True)
    net.load_params(p0)
    step.forward_backward()
    torch.cuda.synchronize()
    assert torch.allclose(g, net.grads, rtol=1e-6, atol=1e-9)


def test_first_layer_fused_into_forward_stack(monkeypatch):
    """conv_stack2 l1 mode: the 5x5 first layer runs inside the forward stack's launch
    (default) — its fragment-ordered weights are fwd_weight permuted by stack_frag_linear,
    and activations, ReLU masks, loss and gradients are bit-identical to the standalone
    first-layer launches: conv_l1_frag (DG_STACK_L1=0) and conv_l1 (DG_L1_FRAG=0 too); all
    add the same bf16 bias table."""
    from deep_go_amd.ops import layouts as LY
    monkeypatch.setenv("DG_STACK_L1", "0")
    monkeypatch.setenv("DG_L1_FRAG", "0")
    _, n2, _ = _setup(5, 128, 5, seed=21)
    monkeypatch.setenv("DG_L1_FRAG", "1")
    _, n0, _ = _setup(5, 128, 5, seed=21)
    monkeypatch.setenv("DG_STACK_L1", "1")
    _, n1, _ = _setup(5, 128, 5, seed=21)
    assert n1.stack_l1 and not n0.stack_l1 and not n2.stack_l1
    assert not any(f in (n1.h.conv_l1, n1.h.conv_l1_frag) for f, _ in n1._fwd_train)
    assert any(f is n0.h.conv_l1_frag for f, _ in n0._fwd_train)
    assert any(f is n2.h.conv_l1 for f, _ in n2._fwd_train)
    assert torch.equal(n1.wfrag[0], LY.stack_frag_linear(n1.wf[0]))
    for n in (n0, n1, n2):
        n.forward_backward()
    torch.cuda.synchronize()
    for other in (n0, n2):
        for a0, a1 in zip(other.act, n1.act):
            assert torch.equal(a0, a1)
        for m0, m1 in zip(other.relu_mask, n1.relu_mask):
            if m0 is not None:
                assert torch.equal(m0, m1)
        assert torch.equal(other.loss, n1.loss)
        assert torch.allclose(other.grads, n1.grads, rtol=1e-5, atol=1e-8)


def test_first_layer_frag_kernel_d256(monkeypatch):
    """At d = 256 the first layer runs on conv_l1_frag (two 128-channel passes over one staged
    input frame); its activations and ReLU bits equal the generic conv_l1 kernel's bit for
    bit (same K order, same bf16 bias table), and the model's weight refresh writes the
    two-pass fragment order stack_frag_linear(wf[0], 256)."""
    from deep_go_amd.ops import layouts as LY
    monkeypatch.setenv("DG_L1_FRAG", "0")
    _, n0, _ = _setup(4, 256, 4, seed=5)
    monkeypatch.setenv("DG_L1_FRAG", "1")
    _, n1, _ = _setup(4, 256, 4, seed=5)
    assert any(f is n1.h.conv_l1_frag for f, _ in n1._fwd_train)
    assert any(f is n0.h.conv_l1 for f, _ in n0._fwd_train)
    assert torch.equal(n1.wfrag[0], LY.stack_frag_linear(n1.wf[0], 256))
    # (conv_l1_frag also runs the feature expansion in its prologue: no expansion launch)
    assert not any(f is n1.h.expand_features for f, _ in n1._pre)
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(n0.x0, n1.x0)
    assert torch.equal(n0.act[0], n1.act[0])
    assert torch.equal(n0.relu_mask[0], n1.relu_mask[0])
    assert torch.equal(n0.loss, n1.loss)
    assert torch.allclose(n0.grads, n1.grads, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("layers", [4, 7])
def test_head_fused_into_forward_stack(layers, monkeypatch):
    """The policy head run inside the forward stack's launch (on the resident board image)
    gives the standalone MFMA head's loss, predictions, dZ and gradients bit for bit.  With
    the first layer in the stack, the feature expansion runs in the same launch's prologue
    (conv_stack2_fwd_head_x): no expansion launch in the training step, the same expanded
    frame x0 (which the first layer's weight gradient reads)."""
    monkeypatch.setenv("DG_FUSE_HEAD", "0")
    _, n0, _ = _setup(layers, 128, 5, seed=12)
    monkeypatch.setenv("DG_FUSE_HEAD", "1")
    _, n1, _ = _setup(layers, 128, 5, seed=12)
    assert n0._fwd_train is n0._fwd
    assert any(f is n1.h.conv_stack2_fwd_head_x for f, _ in n1._fwd_train)
    assert not any(f is n1.h.expand_features for f, _ in n1._pre_train)
    assert any(f is n1.h.expand_features for f, _ in n1._pre)   # (evaluation keeps it)
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(n0.x0, n1.x0)
    assert torch.equal(n0.loss, n1.loss) and torch.equal(n0.pred, n1.pred)
    assert torch.equal(n0.dz[-1], n1.dz[-1])
    assert torch.equal(n0.grads, n1.grads)
    # evaluation still runs the standalone head
    n1.evaluate()
    torch.cuda.synchronize()
    assert torch.equal(n1.eval_loss, n1.loss)


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_head_fused_into_d256_forward(dtype, monkeypatch):
    """d = 256: the policy head runs at the end of the forward launch (conv_layer2_multi HEAD
    for bf16, conv_stack_f8 for fp8) on the last layer's frame its workgroup just wrote —
    the standalone MFMA head's loss, predictions, dZ and gradients bit for bit, and no head
    launch in the training step."""
    monkeypatch.setenv("DG_FUSE_HEAD", "0")
    _, n0, _ = _setup(5, 256, 4, seed=13, dtype=dtype)
    monkeypatch.setenv("DG_FUSE_HEAD", "1")
    _, n1, _ = _setup(5, 256, 4, seed=13, dtype=dtype)
    if dtype == "fp8":
        n0.fp8_scales.copy_(n1.fp8_scales)
        n0.fp8_gscales.copy_(n1.fp8_gscales)
    want = n1.h.conv_stack_f8_fwd_head_y8 if dtype == "fp8" else n1.h.conv_layer2_multi_head
    assert any(f is want for f, _ in n1._fwd_train)
    assert n1._head_train[0] is n1._noop and n0._head_train[0] is not n0._noop
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(n0.loss, n1.loss) and torch.equal(n0.pred, n1.pred)
    assert torch.equal(n0.dz[-1], n1.dz[-1])
    assert torch.equal(n0.grads, n1.grads)
    n1.evaluate()
    torch.cuda.synchronize()
    assert torch.equal(n1.eval_loss, n1.loss)


@pytest.mark.parametrize("l0_mask", ["0", "1"])
@pytest.mark.parametrize("layers", [5, 7])
def test_fused_dgrad_stack_matches_per_layer(layers, l0_mask, monkeypatch):
    """conv_stack in EPI_DGRAD mode (the backward-data chain of the hidden layers in one
    board-resident launch) runs the per-layer board dgrad's exact MFMA sequence and ReLU-mask
    gating: every dZ frame is bit-identical."""
    monkeypatch.setenv("DG_DSTACK", "0")
    _, n0, _ = _setup(layers, 128, 5, seed=9)
    monkeypatch.setenv("DG_DSTACK", "1")
    monkeypatch.setenv("DG_L0_MASK", l0_mask)  # "1": layer 0 writes a bitmask -> down to 1
    _, n1, _ = _setup(layers, 128, 5, seed=9)
    assert not n0.dstack and n1.dstack == list(range(layers - 2, 0 if l0_mask == "1" else 1, -1))
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    for d0, d1 in zip(n0.dz, n1.dz):
        assert torch.equal(d0, d1)
    # (same dZ in, same wgrad kernels; the gradients agree up to reduction-order bits)
    assert torch.allclose(n0.grads, n1.grads, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("layers,group,ch,dstack,win", [
    (7, 5, 128, "1", "1"), (9, 3, 128, "1", "1"), (6, 2, 128, "1", "1"), (6, 3, 128, "0", "1"),
    (5, 3, 256, "1", "1"), (7, 5, 128, "1", "0"), (5, 3, 256, "1", "0")])
def test_grouped_wgrads_match_per_layer(layers, group, ch, dstack, win, monkeypatch):
    """Grouped weight gradients (several layers in one launch: the sliding-window kernel
    conv_wgrad_win, or conv_wgrad_multi with DG_WGRAD_WIN=0) give the per-layer launches'
    gradients up to fp32 summation order — after the dgrad stack (128 channels) or after
    the per-layer dgrads run first (256 channels, or DG_DSTACK=0)."""
    monkeypatch.setenv("DG_DSTACK", dstack)
    monkeypatch.setenv("DG_WGRAD_WIN", win)
    monkeypatch.setenv("DG_WGRAD_GROUP", "1")
    monkeypatch.setenv("DG_DGRAD_FIRST", "0")
    _, n0, _ = _setup(layers, ch, 6, seed=11)
    monkeypatch.setenv("DG_WGRAD_GROUP", str(group))
    monkeypatch.setenv("DG_DGRAD_FIRST", "1")
    _, n1, _ = _setup(layers, ch, 6, seed=11)
    assert not n0.wgroups and n1.wgroups and max(len(g) for g in n1.wgroups) <= group
    assert bool(n1.win_groups) == (win == "1")
    n0.forward_backward()
    n1.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(n0.loss, n1.loss)
    assert torch.allclose(n0.grads, n1.grads, rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("layers,ch,dtype,opt", [
    (12, 128, "bf16", "sgd"), (12, 256, "bf16", "sgd"), (6, 128, "fp8", "sgd"),
    (5, 256, "fp8", "sgd"), (5, 128, "bf16", "rmsprop"), (4, 64, "bf16", "sgd")])
def test_fused_update_matches_separate_launches(layers, ch, dtype, opt, monkeypatch):
    """grad_update (elementwise.hip): the gradient pass 2 read straight from the split-K slabs
    and bias partials + SGD / RMSProp + operand refresh + LR decay in ONE launch, against the
    separate slab-reduce / SGD / refresh launches (DG_FUSED_UPDATE=0).  Same fixed summation
    order and update expressions: parameters, gradients, every operand copy and the LR are
    bit-identical after 3 steps (eager, then graph-replayed)."""
    from deep_go_amd.models.hip_model import SegmentedStep
    kw = dict(dtype=dtype, rateDecay=1e-3)
    if opt == "rmsprop":
        kw.update(optimizer="rmsprop", rate=1e-3)
    nets = []
    for fused in ("0", "1"):
        monkeypatch.setenv("DG_FUSED_UPDATE", fused)
        nets.append(_setup(layers, ch, 4, seed=2, **kw)[1])
    net0, net1 = nets
    net1.keep_grads = True       # (the deferred update writes the gradient only on request)
    # (d = 64: no grouped weight-gradient launch, so the step reduces first and the fused
    # launch reads the flat gradient — still one update launch)
    assert net1.can_defer() == (ch >= 128)
    monkeypatch.setenv("DG_FUSED_UPDATE", "0")
    assert not net0.can_defer()

    def copies(n):
        return [t for t in (*n.wfrag, *n.wdfrag, *n.wf8frag, *n.wd8frag, *n.pbias_frag,
                            *n.pbias) if t is not None]

    def eq(a, b):
        # (d = 64 runs the VALU head, whose weight-gradient partials sum through LDS atomics:
        # its gradients are reproducible to rounding only — compare to that)
        return torch.equal(a, b) if ch >= 128 else torch.allclose(a, b, rtol=1e-5, atol=1e-7)

    def check():
        torch.cuda.synchronize()
        assert eq(net0.params, net1.params)
        assert eq(net0.grads, net1.grads)
        assert net0.lr.item() == net1.lr.item()
        assert int(net0.step_count.item()) == int(net1.step_count.item())
        for a, b in zip(copies(net0), copies(net1)):
            assert torch.equal(a, b) if ch >= 128 else torch.allclose(
                a.float(), b.float(), rtol=1e-2, atol=1e-6)
        if dtype == "fp8":
            assert torch.equal(net0.fp8_scales, net1.fp8_scales)
        assert int(net1.gu_tickets.abs().sum().item()) == 0    # tickets left zeroed
    for _ in range(3):
        monkeypatch.setenv("DG_FUSED_UPDATE", "0")
        net0.train_step()
        monkeypatch.setenv("DG_FUSED_UPDATE", "1")
        net1.train_step()
    check()
    steps = []
    for fused, net in (("0", net0), ("1", net1)):
        monkeypatch.setenv("DG_FUSED_UPDATE", fused)
        steps.append(SegmentedStep(net, None, use_graphs=True))
    for _ in range(2):
        monkeypatch.setenv("DG_FUSED_UPDATE", "0")
        steps[0]()
        monkeypatch.setenv("DG_FUSED_UPDATE", "1")
        steps[1]()
    check()


@pytest.mark.parametrize("early,where,C", [(True, "hidden", 128), (False, "hidden", 128),
                                           (True, "layer0", 128), (False, "head", 128),
                                           (True, "layer0", 256)])
def test_fused_update_all_or_nothing_on_producer_tag(early, where, C):
    """nan_policy guard / skip with the gradient pass 2 deferred into the fused update
    (ADVICE r4): the gradient does not exist before the update, so its PRODUCERS check what
    they write — the window weight-gradient slabs, the bias partials (every dZ value they read,
    |dZ| < 2^100, which also bounds the first layer's 5x5 gradient), the head and first-layer
    reduces — and tag the step (HipGoNet._stepflag[1] = step + 1).  The update then skips the
    WHOLE step: no parameter, operand copy or bias table changes, the step counts once in
    bad_steps, the LR still decays.  hidden: a NaN in a hidden layer's dZ frame (window slabs
    + bias partials tag); layer0: a huge finite dZ_0 (the bias bound tags before the early
    update launch, so the hidden layers it updates do not move either); head: a NaN in the
    head's dZ partials.  early: the grouped layers' update runs before the first layer's
    chain ends.  C = 256: the first layer's bias partial is a launch of its own on the side
    stream (not a row of the grouped launch), issued before the event the early update waits
    on."""
    cfg, net, _ = _setup(4, C, 4, seed=1)
    net._early_ok, net._early_env = early, ("1" if early else "0")
    net.forward_backward()
    torch.cuda.synchronize()
    p0 = net.params.clone()
    copies0 = [t.clone() for t in (*net.wfrag, *net.wdfrag, *net.pbias_frag) if t is not None]
    lr0, st0 = net.lr.item(), int(net.step_count.item())
    net.set_defer(True)
    try:
        s = torch.cuda.current_stream().cuda_stream
        net._run(net._pre_train, s)
        net._run(net._fwd_train, s)
        net._run([net._head_train], s)
        if where == "head":
            net.head_dzb.view(-1)[5] = float("nan")
        net.head_reduce()
        net._run(net._bwd_pre, s)
        if where == "hidden":
            net.dz[net.wgroups[0][0]].view(-1)[3000] = float("nan")
        elif where == "layer0":
            net.dz[0].view(-1)[23 * C + 5] = 1e35     # board 0, frame row 1, column 2
        for i in range(net.L - 2, -1, -1):
            net.backward_layer(i)
        net.join_side()
        assert net._early_issued == early
        net.optimizer_step()
    finally:
        net._defer = False
    torch.cuda.synchronize()
    assert int(net._stepflag[1].item()) == st0 + 1          # tagged this step
    assert torch.equal(net.params, p0)
    assert all(torch.equal(a, b) for a, b in zip(
        [t for t in (*net.wfrag, *net.wdfrag, *net.pbias_frag) if t is not None], copies0))
    assert net.bad_steps.item() == 1
    assert net.lr.item() < lr0 and int(net.step_count.item()) == st0 + 1
    net.train_step()                         # the next, healthy step updates again
    torch.cuda.synchronize()
    assert not torch.equal(net.params, p0) and torch.isfinite(net.params).all()
    assert net.bad_steps.item() == 1


@pytest.mark.parametrize("early", [True, False])
def test_fused_update_skips_non_finite_gradient_entries(early):
    """Defence in depth behind the producers' step tag: a non-finite value that reaches the
    deferred pass 2 WITHOUT a producer having seen it (here poked into a slab after the
    window kernel wrote it) is left unapplied entry by entry (that parameter keeps its value)
    and the step is counted in bad_steps.  early: the grouped layers' update runs right after
    their weight-gradient launch (its flag parked for the final launch); else one launch at
    the end."""
    cfg, net, _ = _setup(4, 128, 4, seed=1)
    net.keep_grads = True
    net._early_ok, net._early_env = early, ("1" if early else "0")
    net.forward_backward()
    torch.cuda.synchronize()
    g_ref = net.grads.clone()
    p0 = net.params.clone()
    # poison one slab entry of a hidden layer's pass 2 (the group's slab region) on the
    # stream, just before the update that reads it
    i = net.wgroups[0][0]
    slab, _, S, Mpad, KP, _ = net._red_src[i]
    spec = net.layout.layers[i]
    view = torch.as_strided(net.gslab, (1,), (1,), (slab - net.gslab.data_ptr()) // 4)
    orig = net._issue_early_update

    def poisoned(stream):
        view.fill_(float("nan"))        # co 0, tap 0, ci 0 of the first split
        orig(stream)
    net._issue_early_update = poisoned
    net.set_defer(True)
    try:
        net.forward_backward()
        if not early:
            view.fill_(float("nan"))
        assert net._early_issued == early
        net.optimizer_step()
    finally:
        net._defer = False
    torch.cuda.synchronize()
    w0 = spec.w_off
    assert torch.isnan(net.grads[w0])
    assert net.params[w0].item() == p0[w0].item()
    assert torch.isfinite(net.params).all()
    assert net.bad_steps.item() == 1
    moved = (net.params - p0).abs() > 0
    assert moved.sum().item() > 0.9 * (g_ref != 0).sum().item()


def test_lr_decay_fused_into_weight_refresh():
    """lr_t = lr0 * (1 - decay)^t (optimizer.lua:25-26), applied by the refresh launch."""
    cfg, net, data = _setup(3, 64, 4, rateDecay=1e-3)
    for _ in range(3):
        net.train_step()
    torch.cuda.synchronize()
    assert abs(net.lr.item() - cfg.rate * (1 - 1e-3) ** 3) < 1e-15
    assert int(net.step_count.item()) == 3
    # refresh_weights() alone (init / load) must not decay
    net.refresh_weights()
    torch.cuda.synchronize()
    assert abs(net.lr.item() - cfg.rate * (1 - 1e-3) ** 3) < 1e-15


@pytest.mark.parametrize("layers,stack,ch", [(4, "1", 128), (4, "0", 128), (12, "1", 128),
                                            (5, "1", 256), (5, "0", 256)])
def test_fp8_forward_model_tracks_bf16(layers, stack, ch, monkeypatch):
    """dtype='fp8': hidden-layer forwards on e4m3 MX-MFMA with delayed scaling — the fused
    fp8 layer stack (conv_stack_f8, default) or the per-layer fp8 kernels (DG_STACK=0); loss
    and gradients stay close to the bf16 model with the same weights and batch."""
    _, net_b, _ = _setup(layers, ch, 6, seed=3)
    monkeypatch.setenv("DG_STACK", stack)
    _, net_8, _ = _setup(layers, ch, 6, seed=3, dtype="fp8")
    assert any(p.fp8 for p in net_8.plans) and net_8._fp8_calibrated
    assert net_8.stack_fp8 == (stack == "1")
    if stack == "1":
        from deep_go_amd.ops import layouts as LY
        i = net_8.stack[0]
        assert torch.equal(net_8.wf8frag[i], LY.stack_frag_f8(
            net_8.wf8[i][:ch, :9 * ch].reshape(ch, 9, ch)))
    net_b.forward_backward()
    net_8.forward_backward()
    torch.cuda.synchronize()
    lb, l8 = net_b.mean_loss().item(), net_8.mean_loss().item()
    assert abs(lb - l8) < 0.03 * abs(lb), (lb, l8)
    gb, g8 = net_b.grads, net_8.grads
    # fp8 forward + (stack) e5m2 backward-data: ~1% cosine gap on a random-init net
    assert ((g8 - gb).norm() / gb.norm()).item() < (0.2 if net_8.dstack_fp8 else 0.15)
    assert torch.isfinite(net_8.fp8_scales).all() and (net_8.fp8_scales > 0).all()


@pytest.mark.parametrize("layers,ch", [(6, 128), (5, 256)])
def test_fp8_dgrad_stack_vs_bf16_dgrad(layers, ch, monkeypatch):
    """The e5m2 backward-data stack (DG_FP8_DGRAD=1, default with dtype='fp8') against the
    same fp8-forward model with the bf16 dgrad stack: identical loss (same forward), weight
    gradients within the e5m2 rounding noise, gradient scales finite powers of two."""
    monkeypatch.setenv("DG_FP8_DGRAD", "0")
    _, net_0, _ = _setup(layers, ch, 6, seed=5, dtype="fp8")
    monkeypatch.setenv("DG_FP8_DGRAD", "1")
    _, net_1, _ = _setup(layers, ch, 6, seed=5, dtype="fp8")
    assert net_1.dstack_fp8 and not net_0.dstack_fp8 and net_1.stack_fp8
    net_0.fp8_scales.copy_(net_1.fp8_scales)
    net_0.forward_backward()
    net_1.forward_backward()
    torch.cuda.synchronize()
    assert torch.equal(net_0.loss, net_1.loss)
    g0, g1 = net_0.grads, net_1.grads
    rel = ((g1 - g0).norm() / g0.norm()).item()
    assert rel < 0.12, rel
    gs = net_1.fp8_gscales
    assert torch.isfinite(gs).all() and (gs > 0).all()
    assert torch.equal(torch.exp2(torch.log2(gs).round()), gs)
    assert int(net_1.fp8_sat.sum().item()) == 0


def test_fp8_training_reduces_loss():
    """Same memorisation run as test_loss_decreases, fp8 forward vs bf16: both converge and
    the fp8 trajectory stays close to the bf16 one."""
    from deep_go_amd.models.hip_model import SegmentedStep
    finals = {}
    for dt in ("bf16", "fp8"):
        cfg, net, data = _setup(4, 128, 16, seed=4, dtype=dt, head_relu=False, rate=0.1)
        step = SegmentedStep(net, None, use_graphs=True)
        losses = []
        for _ in range(40):
            step()
            losses.append(net.mean_loss().item())
        torch.cuda.synchronize()
        assert all(np.isfinite(losses)), (dt, losses)
        assert losses[-1] < 0.8 * losses[0], (dt, losses[0], losses[-1])
        finals[dt] = losses[-1]
    assert abs(finals["fp8"] - finals["bf16"]) < 0.1, finals  # both memorise the batch


def test_loss_decreases():
    # head_relu=False: with the reference's head ReLU a large LR kills every logit (the
    # loss then pins at ln(361) exactly, see test_head_relu_dead_logits_quirk)
    cfg, net, data = _setup(4, 64, 16, rate=0.1, head_relu=False)
    losses = []
    for _ in range(40):
        net.train_step()
        losses.append(net.mean_loss().item())
    assert np.isfinite(losses).all()
    assert losses[-1] < 0.8 * losses[0], (losses[0], losses[-1])


def test_rmsprop_step_runs():
    cfg, net, data = _setup(3, 64, 4, optimizer="rmsprop", rate=1e-3)
    p0 = net.params.clone()
    net.train_step()
    torch.cuda.synchronize()
    assert torch.isfinite(net.params).all()
    assert (net.params - p0).abs().max() > 0


def test_eval_matches_train_forward():
    cfg, net, data = _setup(3, 64, 7)
    net.evaluate()
    torch.cuda.synchronize()
    l1 = net.eval_loss.clone()
    p1 = net.eval_pred.clone()
    net.forward_backward()
    torch.cuda.synchronize()
    assert torch.allclose(l1, net.loss)
    assert torch.equal(p1, net.pred)


def test_head_relu_dead_logits_quirk():
    """Reference parity quirk: ReLU before LogSoftMax; if every head
    pre-activation is <= 0 the softmax is uniform and no gradient flows: loss = ln 361."""
    cfg, net, data = _setup(3, 64, 4)
    hd = net.layout.layers[-1]
    net.params[hd.b_off].fill_(-100.0)
    net.forward_backward()
    torch.cuda.synchronize()
    assert abs(net.mean_loss().item() - np.log(361)) < 1e-5
    assert net.grads.abs().max().item() == 0.0


@pytest.mark.parametrize("layers,group", [(8, "5"), (9, "3")])
def test_side_stream_with_ungrouped_layers_matches(layers, group, monkeypatch):
    """8 layers with 5- or 3-layer weight-gradient groups leave hidden layer(s) ungrouped
    below the lowest group; layer 0's side-stream chain must not then share the scratch
    slab with their main-stream wgrads (data race).  Gradients must equal the
    single-stream order."""
    monkeypatch.setenv("DG_WGRAD_GROUP", group)
    monkeypatch.setenv("DG_SIDE_STREAM", "0")
    _, net0, _ = _setup(layers, 128, 4, seed=3)
    net0.forward_backward()
    torch.cuda.synchronize()
    monkeypatch.setenv("DG_SIDE_STREAM", "bias")
    _, net1, _ = _setup(layers, 128, 4, seed=3)
    grouped = set(i for g in net1.wgroups for i in g)
    assert any(i not in grouped for i in range(1, layers - 1))
    for _ in range(3):
        net1.forward_backward()
        torch.cuda.synchronize()
        assert torch.allclose(net1.grads, net0.grads, rtol=1e-5, atol=1e-7)


def test_nan_skip_policy_leaves_parameters_unchanged():
    """nan_policy='skip': a non-finite gradient or loss ON THE DEVICE skips the SGD update
    (0 * NaN must not reach the weights), counts the step, and still decays the rate."""
    cfg, net, _ = _setup(4, 128, 4, seed=1, nan_policy="skip")
    net.forward_backward()
    torch.cuda.synchronize()
    p0 = net.params.clone()
    wf0 = [w.clone() for w in net.wf]
    lr0 = net.lr.item()
    net.grads[17] = float("nan")            # poisoned gradient, finite loss
    net.optimizer_step()
    torch.cuda.synchronize()
    assert torch.equal(net.params, p0)
    assert all(torch.equal(a, b) for a, b in zip(net.wf, wf0))
    assert net.bad_steps.item() == 1 and net.gate.item() == 0.0
    assert net.lr.item() < lr0
    net.forward_backward()
    net.loss[0] = float("inf")              # poisoned loss, finite gradients
    net.optimizer_step()
    torch.cuda.synchronize()
    assert torch.equal(net.params, p0) and net.bad_steps.item() == 2
    net.forward_backward()                  # healthy step: updates again
    net.optimizer_step()
    torch.cuda.synchronize()
    assert net.gate.item() == 1.0 and not torch.equal(net.params, p0)
    assert torch.isfinite(net.params).all()


@pytest.mark.parametrize("layers,ch,B,graphs", [(12, 128, 8, True), (4, 64, 5, False)])
def test_input_prefetch_matches_single_buffer(layers, ch, B, graphs):
    """enable_prefetch (two input buffers, copies on the load stream, one step graph per
    buffer) trains on exactly the same batch sequence as the single-buffer step: per-step
    losses and the final parameters are bit-identical."""
    from deep_go_amd.config import ExperimentConfig
    from deep_go_amd.data.batch import pack_batch
    from deep_go_amd.data.synthetic import random_planes
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    cfg = ExperimentConfig(numLayers=layers, channelSize=ch, batchSize=B, seed=3)
    pool = []
    for j in range(3):
        pool.append(pack_batch(*random_planes(B, seed=50 + j)).cuda())
    runs = []
    for prefetch in (False, True):
        net = HipGoNet(cfg, B, device="cuda")
        if prefetch:
            assert net.enable_prefetch()
        net.set_batch_packed(pool[0])
        step = SegmentedStep(net, None, use_graphs=graphs)
        if graphs and prefetch:
            assert len(step._gsets) == 2
        losses = []
        for i in range(7):
            net.set_batch_packed(pool[i % 3])
            step()
            losses.append(net.mean_loss().item())
        torch.cuda.synchronize()
        runs.append((losses, net.params.clone(), net.correct().item()))
    assert runs[0][0] == runs[1][0]          # the same batch in every step
    if graphs:
        assert torch.equal(runs[0][1], runs[1][1])
        assert runs[0][2] == runs[1][2]
    else:   # the 64-channel per-layer kernels reduce some gradients with atomics
        assert (runs[0][1] - runs[1][1]).abs().max().item() < 1e-5


@pytest.mark.parametrize("ch,layers", [(256, 5), (128, 6)])
def test_fp8_weight_gradient_teacher_forced(ch, layers):
    """MX-fp8 window weight gradients (conv_wgrad_win8.hip) on the fp8 stacks' e4m3 / e5m2
    copies: (1) the fp8 copy-out frames dequantize EXACTLY to the bf16 frames the stacks
    write (same bytes x power-of-two scale); (2) each hidden layer's weight gradient equals
    a float64 CPU oracle — torch's conv2d weight gradient over those dequantized frames —
    to fp32 summation order (the quantization itself is the oracle's input, so the test is
    teacher-forced: it checks the kernel, not the fp8 rounding)."""
    from deep_go_amd.models.hip_model import FP8_PITCH, HipGoNet
    _, net0, data = _setup(layers, ch, 8, seed=47, dtype="fp8")
    # production skips the bf16 frames of the non-last stack layers (nothing reads them);
    # keep_act_frames writes them for the comparison below
    # (and the backward-data stack's bf16 dZ frames below its top: the weight gradients and
    # the bias partials read the e5m2 copies)
    assert net0.act_frames_dropped == list(range(1, layers - 2))
    assert sorted(net0.dz_frames_dropped) == list(range(1, layers - 2))
    net = HipGoNet(net0.cfg, 8, device="cuda", keep_act_frames=True)
    assert net.act_frames_dropped == [] and net.dz_frames_dropped == []
    planes, player, rank, labels = data
    net.set_batch(torch.from_numpy(planes).cuda(), torch.from_numpy(player).cuda(),
                  torch.from_numpy(rank).cuda(), torch.from_numpy(labels).cuda())
    assert net.win8_groups, "fp8 model must use the MX-fp8 window weight gradient"
    net.forward_backward()
    net0.forward_backward()
    torch.cuda.synchronize()
    # dropping the frames changes no result: loss and every gradient (the bias partials
    # from e5m2 x scale == from the bf16 frame) bit for bit
    assert torch.equal(net0.loss, net.loss)
    assert torch.equal(net0.grads, net.grads)
    B = net.B
    hidden = [i for g in net.win8_groups for i in g]
    assert sorted(hidden) == list(range(1, layers - 1))
    for i in hidden:
        s_x = net.fp8_scales[2 * (i - 1) + 1].item()
        s_g = net.fp8_gscales[i].item()
        # fp8 frames [B][448][C]: rows 0..440 are the 21x21 frame
        x8 = net.x8q[i].view(B, FP8_PITCH, ch)[:, :441].view(torch.float8_e4m3fn).float() * s_x
        g8 = net.dz8q[i].view(B, FP8_PITCH, ch)[:, :441].view(torch.float8_e5m2).float() * s_g
        xb = net.act[i - 1].view(B, 441, ch).float()
        gb = net.dz[i].view(B, 441, ch).float()
        # a stack's own input (act[0] from conv_l1, dz[top] from the head) stays unquantized
        # bf16: its fp8 copy is its rounding (e4m3 to nearest: half an ulp, 2^-4 relative;
        # e5m2 rounded stochastically: under one ulp, 2^-2 relative); every other bf16 frame
        # IS the dequantized fp8 image, bit for bit (plus the subnormal step: e4m3 2^-9,
        # e5m2 2^-16)
        if i == 1:
            bad = int(((x8 - xb).abs() > xb.abs() * 2 ** -4 + 2 ** -9 * s_x).sum())
            assert bad == 0, f"layer 1: {bad} fp8 activations off their rounding"
        else:
            assert torch.equal(x8, xb), f"layer {i}: fp8 activation copy != bf16 frame"
        if i == layers - 2:
            bad = int(((g8 - gb).abs() > gb.abs() * 2 ** -2 + 2 ** -16 * s_g).sum())
            assert bad == 0, f"layer {i}: {bad} fp8 gradients off their rounding"
        else:
            assert torch.equal(g8, gb), f"layer {i}: fp8 gradient copy != bf16 frame"
        x = x8.view(B, 21, 21, ch)[:, 1:20, 1:20].permute(0, 3, 1, 2).double().cpu()
        dz = g8.view(B, 21, 21, ch)[:, 1:20, 1:20].permute(0, 3, 1, 2).double().cpu()
        ref = torch.nn.grad.conv2d_weight(x, (ch, ch, 3, 3), dz, padding=1)   # [co][ci][kh][kw]
        spec = net.layout.layers[i]
        got = net.grads[spec.w_off:spec.w_off + spec.w_numel].view(ch, 3, 3, ch)
        got = got.permute(0, 3, 1, 2).double().cpu()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"fp8 wgrad layer {i}: max |err| / max |ref| = {err:.2e}")
        # the fp8 MFMA sums each 128-product block before its fp32 accumulate (not exactly
        # the fp64 order): ~1e-4 of the largest entry, against ~0.06-0.125 per-element
        # quantization steps the oracle already contains
        assert err < 5e-4, (i, err)


@pytest.mark.parametrize("dtype,ch", [("fp8", 128), ("fp8", 256), ("bf16", 128)])
def test_dropped_frames_and_operand_copies_over_many_steps(dtype, ch):
    """frames and operand copies that HipGoNet decides nothing reads
    (_drop_unread_act_frames: the fp8 stacks' non-last bf16 frames; _step_refresh_table: the
    plain / untaken-path weight copies the per-step refresh skips) must stay unread across
    optimizer steps too.  A model with every frame written and the full refresh table
    (keep_act_frames, the init-time refresh table) follows the default one bit for bit over
    several whole steps (graph-replayed, the deferred fused update)."""
    from deep_go_amd.models.hip_model import HipGoNet, SegmentedStep
    _, net0, data = _setup(6, ch, 8, seed=51, dtype=dtype)
    net1 = HipGoNet(net0.cfg, 8, device="cuda", keep_act_frames=True)
    planes, player, rank, labels = data
    net1.set_batch(torch.from_numpy(planes).cuda(), torch.from_numpy(player).cuda(),
                   torch.from_numpy(rank).cuda(), torch.from_numpy(labels).cuda())
    net1._step_refresh = net1._refresh_table.copy()   # refresh every operand copy each step
    if dtype == "fp8":
        assert net0.act_frames_dropped and not net1.act_frames_dropped
        net1.fp8_scales.copy_(net0.fp8_scales)
        net1.fp8_gscales.copy_(net0.fp8_gscales)
        net1.fp8_amax_w.copy_(net0.fp8_amax_w)
    s0 = SegmentedStep(net0, None, use_graphs=True)
    s1 = SegmentedStep(net1, None, use_graphs=True)
    for k in range(6):
        s0()
        s1()
        torch.cuda.synchronize()
        assert torch.equal(net0.loss, net1.loss), k
        assert torch.equal(net0.params, net1.params), k


@pytest.mark.parametrize("args", [["--channels", "128", "--dtype", "bf16"],
                                  ["--channels", "128", "--dtype", "fp8"],
                                  ["--channels", "128", "--dtype", "bf16", "--dp"]])
def test_stream_handoffs_checked_and_serialized_run_bit_identical(args, tmp_path):
    """SURVEY §5.2's stream/event discipline.  Three eager runs of the
    fused training step in fresh processes (tools/stream_check_run.py): (1) with
    DG_CHECK_STREAMS=1 — every cross-stream hand-off (dZ -> side stream, bias partials ->
    slab reduce / early update, the first layer's chain -> main, side join, DP bucket fork to
    the comm stream and its join) bracketed by timing events and verified after each step;
    (2) under AMD_SERIALIZE_KERNEL=3 (the HIP runtime serializes every kernel: no two streams
    overlap); (3) plainly.  The parameters after 3 steps and the last losses must be bit for
    bit identical: nothing in the step depends on how its streams interleave.  The fp8 case
    takes the early update (hidden layers updated beside the first layer's chain); --dp the
    native RCCL communicator's in-graph buckets at world 1."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = {}
    for name, env in (("check", {"DG_CHECK_STREAMS": "1"}),
                      ("serial", {"AMD_SERIALIZE_KERNEL": "3"}), ("plain", {})):
        out = str(tmp_path / f"{name}.pt")
        e = dict(os.environ)
        e.pop("DG_CHECK_STREAMS", None)
        e.pop("AMD_SERIALIZE_KERNEL", None)
        e.update(env)
        r = subprocess.run([sys.executable, os.path.join(root, "tools", "stream_check_run.py"),
                            out, *args], env=e, capture_output=True, text=True, timeout=100)
        assert r.returncode == 0, (name, r.stderr[-3000:])
        outs[name] = torch.load(out, weights_only=True)
    assert outs["check"]["checked"] >= 3 * (4 if "--dp" not in args else 6), outs["check"]
    assert outs["plain"]["checked"] == 0
    for name in ("check", "serial"):
        assert torch.equal(outs[name]["params"], outs["plain"]["params"]), name
        assert torch.equal(outs[name]["loss"], outs["plain"]["loss"]), name

