"""GoCNN on MI355X: a native training-step executor over the hand-written HIP kernels.

This replaces the reference's nn.Sequential + cunn execution (``experiments.lua:97-107``,
``train.lua:4-12``) with an explicit, pre-planned launch sequence:

  zero grads -> expand features (uint8 planes -> bf16 frame) -> conv fwd x (L-1)
  -> fused head (conv + biases + ReLU + log-softmax + NLL + argmax + its backward)
  -> for each layer, last to first: bias grads, wgrad (split-K slabs + reduce), dgrad
     with the ReLU mask fused
  -> [DP: bucketed gradient all-reduce hooks] -> SGD/RMSProp -> LR decay -> bf16 refresh

Every launch's arguments are resolved once at construction (``self._fwd``, ``self._bwd``
lists) so a step is a flat loop of native calls; the whole step, or the segments between
collectives, is then captured into a hipGraph (``torch.cuda.CUDAGraph``) and replayed.

Buffers are static (allocated once, sized for the per-GPU batch): the 12x256 config at
batch 256 needs < 1 GB of HBM, so nothing is ever re-allocated in the step.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..config import NUM_POINTS, ExperimentConfig
from ..data.batch import pack_batch, packed_batch_bytes, unpack_views  # noqa: F401
from ..ops import layouts as LY
from ..ops.native import hip, stream_handle
from ..utils import streamcheck, trace
from .gocnn import ParamLayout, init_params

INPUT_CP = 40  # 37 planes padded to 5 x 8-channel groups


def _ptr(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.data_ptr()


FP8_PITCH = 448   # rows per board of the fp8 copy-out frames (441 + 7 zero rows)
# weight scale margin over the last refresh's |w| max (s_w = margin amax / 448): SGD moves
# the weights between two refreshes; 1.05 saturated up to 3% of layer-steps in the
# memorisation stress run (tests/test_train_gpu.py), 1.25 covers a 25% step-to-step growth
FP8_W_MARGIN = 1.25
# headroom of the delayed power-of-two e5m2 gradient scales over the max of the last
# FP8_GHIST observed amaxes
# (conv_fp8.hip fp8_update_scales; tests/test_train_gpu.py test_fp8_stress_vs_bf16_memorisation)
FP8_G_HEADROOM = 4.0
FP8_GHIST = 16        # gradient amax history length (conv_fp8.hip FP8_GHIST)
REFRESH_PARTS = 512   # weight_refresh workgroups per layer (elementwise.hip)


@dataclass
class ConvPlan:
    index: int
    k: int
    pad: int
    cin: int
    cinp: int        # channels of the input frame
    cout: int
    bm: int
    bn: int
    KP: int          # fwd K (multiple of 64)
    Mpad: int        # fwd M padding
    KPw: int         # wgrad K (multiple of 128)
    Mpad_w: int
    splits: int
    KPd: int = 0     # dgrad K
    Mpad_d: int = 0
    bm_d: int = 128
    bn_d: int = 128
    board: bool = False    # fwd uses the board-tiled kernel
    board_d: bool = False  # dgrad uses the board-tiled kernel
    fp8: bool = False      # forward on the e4m3 MX-MFMA kernel (conv_fp8.hip)


class HipGoNet:
    """Static-buffer GoCNN executor for one GPU (one rank)."""

    def __init__(self, cfg: ExperimentConfig, batch: int, device="cuda",
                 flat_params: Optional[torch.Tensor] = None, num_cus: Optional[int] = None,
                 global_batch: Optional[int] = None, wgrad_group: Optional[int] = None,
                 grad_wire: str = "fp32", keep_act_frames: bool = False):
        if cfg.numLayers < 2:
            raise ValueError("HIP executor needs >= 2 layers (conv stack + head)")
        self.cfg = cfg
        self.B = batch
        self.global_batch = global_batch or batch
        # layers per grouped weight-gradient launch (None: DG_WGRAD_GROUP, default all);
        # data parallelism splits the hidden layers into groups so the top group's
        # all-reduce runs beside the next group's launch (bench.py --wgrad-group)
        self._wgrad_group = wgrad_group
        # keep_act_frames: always write every layer's bf16 activation frame (tests / tools
        # that inspect them); by default an fp8 stack skips frames no launch reads
        self.keep_act_frames = keep_act_frames
        self.device = torch.device(device)
        self.h = hip()
        self.layout = ParamLayout(cfg)
        if num_cus is None:
            num_cus = torch.cuda.get_device_properties(self.device).multi_processor_count
        self.num_cus = num_cus
        L = self.layout.layers
        self.L = len(L)
        npix = batch * NUM_POINTS
        self.npix = npix
        dev = self.device

        # ---- parameters / optimizer state ----
        if flat_params is None:
            flat_params = init_params(self.layout, cfg.seed)
        self.params = flat_params.to(dev, torch.float32).contiguous()
        self.grads = torch.zeros_like(self.params)
        # data-parallel bf16 wire format: every gradient reduce also writes a bf16 twin
        # (grads16, same flat layout), the bucket all-reduces run on it and the optimizer
        # reads it — no conversion kernels around the collectives
        if grad_wire not in ("fp32", "bf16"):
            raise ValueError(f"grad_wire {grad_wire!r}")
        self.grad_wire = grad_wire
        self.grads16 = (torch.zeros(self.params.numel(), dtype=torch.bfloat16, device=dev)
                        if grad_wire == "bf16" else None)
        self.lr = torch.tensor([cfg.rate], dtype=torch.float64, device=dev)
        # [0] the device step counter (the fused update and the weight refresh count it); [1]
        # the step tag: a gradient producer that writes a non-finite / out-of-range value sets
        # it to step + 1 and the fused update then skips the WHOLE step (dg_common.h
        # grad_out_of_range; nan_policy guard / skip stay all-or-nothing with the gradient
        # pass 2 deferred into the update)
        self._stepflag = torch.zeros(2, dtype=torch.int64, device=dev)
        self.step_count = self._stepflag[0:1]
        self._sf = self._stepflag.data_ptr()
        self.ms = None
        if cfg.optimizer == "rmsprop":
            self.ms = torch.ones_like(self.params)
        # non-finite loss guard (cfg.nan_policy == "skip"): device gate read by the optimizer
        self.gate = torch.ones(1, dtype=torch.float32, device=dev)
        self._gate_ticket = torch.zeros(1, dtype=torch.int32, device=dev)   # finite_gate1
        self.bad_steps = torch.zeros(1, dtype=torch.int32, device=dev)
        # fused end of step (grad_update): per-layer + grid tickets, zero between launches
        self.gu_tickets = torch.zeros(self.h.grad_update_tickets(), dtype=torch.int32, device=dev)
        # the fused update with the pass 2 deferred writes the reduced gradient to self.grads
        # only when asked (tests, tools): nothing in the step reads it
        self.keep_grads = False
        # True while a step is issued whose gradient pass 2 is deferred into the fused update
        # (train_step / SegmentedStep's whole-step graph; see can_defer)
        self._defer = False
        self._gate_issued = False   # this step's loss gate already issued (side stream)
        self._early_issued = False  # this step's early update launch issued (main stream)
        self._early_env = os.environ.get("DG_EARLY_UPDATE")   # None: auto (fp8 window)
        self._early_ok = self._early_env != "0"
        self._red_src = {}    # layer -> (slab, bpart, splits, Mpad, KP, bchunks) of its pass 2

        # ---- per-layer plans + bf16 operand weights ----
        self.plans: List[ConvPlan] = []
        self.fp8 = cfg.dtype == "fp8"
        if cfg.dtype not in ("bf16", "fp8"):
            raise ValueError(f"unsupported GPU dtype {cfg.dtype!r} (bf16 | fp8)")
        self.wf8: List[Optional[torch.Tensor]] = []
        self.wf: List[torch.Tensor] = []
        self.wd: List[Optional[torch.Tensor]] = []
        for spec in L[:-1]:
            cinp = INPUT_CP if spec.index == 0 else spec.cin
            board = LY.board_ok(spec.k, cinp)
            bm, bn = LY.pick_tiles(npix, spec.cout, num_cus)
            if board:
                bm = LY.board_bm(spec.cout)
            KP, KPw, Mpad = LY.conv_dims(spec.k, cinp, spec.cout, bm)
            Mpad_w = LY.round_up(spec.cout, 128)
            splits = LY.pick_wgrad_splits(npix, KPw, Mpad_w, num_cus,
                                           self.h.conv_wgrad_wgs_per_cu_for(KPw),
                                           self.h.conv_wgrad_ktile(KPw))
            p = ConvPlan(spec.index, spec.k, spec.pad, spec.cin, cinp, spec.cout, bm, bn, KP,
                         Mpad, KPw, Mpad_w, splits, board=board)
            self.wf.append(torch.zeros((Mpad, KP), dtype=torch.bfloat16, device=dev))
            if spec.index > 0:
                bm_d, bn_d = LY.pick_tiles(npix, spec.cin, num_cus)
                p.board_d = LY.board_ok(spec.k, spec.cout)
                if p.board_d:
                    bm_d = LY.board_bm(spec.cin)
                KPd, _, Mpad_d = LY.conv_dims(spec.k, spec.cout, spec.cin, bm_d)
                p.KPd, p.Mpad_d, p.bm_d, p.bn_d = KPd, Mpad_d, bm_d, bn_d
                self.wd.append(torch.zeros((Mpad_d, KPd), dtype=torch.bfloat16, device=dev))
            else:
                self.wd.append(None)
            p.fp8 = self.fp8 and board and cinp % 128 == 0
            self.wf8.append(torch.zeros((Mpad, KP), dtype=torch.uint8, device=dev)
                            if p.fp8 else None)
            self.plans.append(p)
        self.head = L[-1]
        # conv_stack2 (csrc/kernels/conv_stack2.hip): fragment-ordered forward / dgrad operands
        # of every hidden 3x3 128 -> 128 layer, written by weight_refresh beside wf / wd
        # (+ conv_stack_f8.hip's e4m3 forward operands of the fp8 layers)
        self.wfrag: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        self.wdfrag: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        self.wf8frag: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        self.wd8frag: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        for p in self.plans:
            if p.index == 0 and (self._stack_l1_ok(p) or self._l1_frag_ok(p)):
                # the first layer fused in front of the forward stack (conv_stack2.hip l1
                # mode) or on conv_l1_frag (conv_l1.hip): [cout][1024] weights in fragment
                # order (k linear), no dgrad operand
                self.wfrag[0] = torch.zeros(p.cout * 1024, dtype=torch.bfloat16, device=dev)
            if (p.index > 0 and p.k == 3 and p.cin == p.cout == p.cinp
                    and (p.cout == 128 or (p.cout == 256 and self._layer2_ok(p)))):
                # 128: the layer stacks; 256: the per-layer conv_layer2 kernel
                self.wfrag[p.index] = torch.zeros(p.cout * 9 * p.cin, dtype=torch.bfloat16,
                                                  device=dev)
                self.wdfrag[p.index] = torch.zeros_like(self.wfrag[p.index])
            if (p.fp8 and p.index > 0 and p.k == 3 and p.cin == p.cout == p.cinp
                    and p.cout in (128, 256)):
                self.wf8frag[p.index] = torch.zeros(p.cout * 9 * p.cin, dtype=torch.uint8,
                                                    device=dev)
                # the fp8 backward-data stack's operand (DG_FP8_DGRAD=0: bf16 backward-data)
                if os.environ.get("DG_FP8_DGRAD", "1") != "0":
                    self.wd8frag[p.index] = torch.zeros_like(self.wf8frag[p.index])

        # ---- activation / gradient frames ----
        B = batch
        pads = [s.pad for s in L]
        self.x0 = LY.alloc_frame(B, INPUT_CP, pads[0], dev)
        # act[i]: output of layer i, framed with the pad of layer i+1
        self.act = [LY.alloc_frame(B, L[i].cout, pads[i + 1], dev) for i in range(self.L - 1)]
        # dz[i]: d loss / d pre-activation of layer i, framed with layer i's pad (>=1)
        # (layer i's dgrad reads dz[i] with its own taps: halo = pad_i; layer 0 has no dgrad,
        # so dz[0] keeps pad 1 whatever the first layer's kernel size — the 21x21 geometry
        # of the board-resident dgrad stack)
        self.dzp = [max(1, pads[i]) if i > 0 else 1 for i in range(self.L - 1)]
        self.dz = [LY.alloc_frame(B, L[i].cout, self.dzp[i], dev) for i in range(self.L - 1)]
        # fp8 shadow of the input frame of every fp8 layer (same geometry, 1 byte/elem);
        # per conv layer l: scales[2l] = s_w, scales[2l+1] = s_y (scale of act[l]'s fp8
        # shadow), amax[l] = observed max of act[l] (float bits), delayed scaling
        self.x8: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        for p in self.plans:
            if p.fp8:
                src = self.x0 if p.index == 0 else self.act[p.index - 1]
                self.x8[p.index] = torch.zeros(src.numel(), dtype=torch.uint8, device=dev)
        # forward epilogue bias table (bf16 bias + pos_bias, rebuilt by every weight refresh)
        # and ReLU bitmasks of the board-kernel outputs consumed by a board dgrad
        self.pbias = [torch.zeros((NUM_POINTS, p.cout), dtype=torch.bfloat16, device=dev)
                      if (p.board and not p.fp8) or self._l1_res_ok(p) else None
                      for p in self.plans]
        # the same table in the forward stacks' accumulator-fragment order (coalesced
        # epilogue loads), for every 128-channel board layer (bf16 or fp8)
        self.pbias_frag = [torch.zeros((p.cout // 128) * 24 * 2 * 4 * 64 * 4, dtype=torch.bfloat16,
                                       device=dev)
                           if ((pb is not None and p.cout == 128) or self.wfrag[p.index] is not None
                               or self.wf8frag[p.index] is not None)
                           else None for p, pb in zip(self.plans, self.pbias)]
        self.relu_mask = [None] * len(self.plans)
        for p in self.plans[:-1]:
            nxt = self.plans[p.index + 1]
            # board forwards write the bitmask; so does the board-resident first layer
            # (conv_l1), which lets the dgrad stack reach layer 1 (DG_L0_MASK=0: off).  The
            # pixel-tiled first layer can too (conv_nt_ex), but its byte stores cost +13 us vs
            # the ~5 us saved (measured): there DG_L0_MASK=1 opts in
            l0 = p.index == 0 and (os.environ.get("DG_L0_MASK", "") == "1" or (
                os.environ.get("DG_L0_MASK", "") != "0" and self._l1_res_ok(p)))
            if ((p.board or l0) and nxt.board_d
                    and os.environ.get("DG_RELU_MASK", "1") == "1"):
                self.relu_mask[p.index] = torch.zeros((B, NUM_POINTS, p.cout // 8),
                                                      dtype=torch.uint8, device=dev)
        # MX-fp8 weight gradients of the hidden layers (conv_wgrad_win8.hip, fp8 models;
        # DG_FP8_WGRAD=0: bf16 window kernel): x8q[l] / dz8q[l] = the fp8 copies of layer l's
        # input activation (e4m3) and gradient (e5m2) that the fp8 stacks write beside the
        # bf16 frames (448 rows per board); allocated by _fuse_forward_stack /
        # _fuse_dgrad_stack for the layers they cover
        self.fp8_wgrad = self.fp8 and os.environ.get("DG_FP8_WGRAD", "1") != "0"
        # stochastic rounding of the fp8 backward-data stack's e5m2 gradients, seeded by the
        # device step counter (conv_stack_f8.hip pack_bf8x4_sr; DG_FP8_SR=0: nearest even)
        self.fp8_sr = self.fp8 and os.environ.get("DG_FP8_SR", "1") != "0"
        self.x8q: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        self.dz8q: List[Optional[torch.Tensor]] = [None] * len(self.plans)
        self.fp8_scales = torch.ones(2 * len(self.plans), dtype=torch.float32, device=dev)
        self.fp8_amax = torch.zeros(len(self.plans), dtype=torch.int32, device=dev)
        # |w| max per layer: one slot per weight_refresh workgroup (REFRESH_PARTS), reduced by
        # fp8_update_scales
        self.fp8_amax_w = torch.zeros((len(self.plans), REFRESH_PARTS), dtype=torch.int32,
                                      device=dev)
        # saturation events per layer ([2l] weights, [2l + 1] activations): a step whose
        # observed amax exceeded 448 x the scale in use (values were clamped)
        # ([2L + l] gradients: the e5m2 dz[l] of the fp8 backward-data stack)
        self.fp8_sat = torch.zeros(3 * len(self.plans), dtype=torch.int32, device=dev)
        # e5m2 scales of the gradient frames dz[l] the fp8 backward-data stack quantizes, and
        # their observed |dz| max (delayed scaling, powers of two)
        self.fp8_gscales = torch.ones(len(self.plans), dtype=torch.float32, device=dev)
        self.fp8_gamax = torch.zeros(len(self.plans), dtype=torch.int32, device=dev)
        # the last FP8_GHIST gradient amaxes per layer (conv_fp8.hip: the gradient scale
        # comes from their max)
        self.fp8_ghist = torch.zeros((len(self.plans), FP8_GHIST), dtype=torch.float32,
                                     device=dev)
        self._fp8_calibrated = not self.fp8
        # backward side stream ("bias", the default): the HBM-bound bias-grad partials run on
        # it beside the MFMA-bound weight-gradient launch of the same layers, and the first
        # layer's whole weight-gradient chain beside the last wgrad group (262k -> 264k
        # boards/s at 12x128 when introduced, neutral at 12x256).  DG_SIDE_STREAM=0: one
        # stream.  (Two other modes — the whole wgrad chain, or partials + slab reduces,
        # on the side stream — measured slower and were removed in round 2.)
        side_mode = os.environ.get("DG_SIDE_STREAM", "bias")
        self.side_mode = {"0": "none"}.get(side_mode, side_mode)
        if self.side_mode not in ("none", "bias"):
            raise ValueError(f"DG_SIDE_STREAM={side_mode!r}: expected 0 or bias")
        self.bchunks = self.h.bias_chunks(batch)            # per-layer bias partials
        self.bchunks_g = self.h.bias_chunks_multi(batch)    # grouped (multi-layer) ones
        slab = torch.empty(max(p.splits * p.Mpad_w * p.KPw for p in self.plans),
                           dtype=torch.float32, device=dev)
        cmax = max(p.cout for p in self.plans)
        bpart = torch.empty(self.bchunks * (NUM_POINTS + 19) * cmax, dtype=torch.float32,
                            device=dev)
        self.slabs = [slab] * len(self.plans)
        self.bparts = [bpart] * len(self.plans)
        self.slab = slab

        # ---- step I/O ----
        # one packed uint8 input buffer (planes | player | rank | labels as int32), so a step's
        # batch lands with ONE copy (set_batch_packed / pack_batch); the named views are what
        # the kernels read
        self.inbuf = torch.zeros(packed_batch_bytes(B), dtype=torch.uint8, device=dev)
        self.planes, self.player, self.rank, self.labels = unpack_views(self.inbuf, B)
        self.player.fill_(1)
        self.rank.fill_(1)
        # input prefetch (enable_prefetch): a second input buffer filled on a load stream
        # while the previous step still runs; cur_in = the buffer the next step reads
        self._inbufs = [self.inbuf]
        self.cur_in = 0
        self.load_stream = None
        self._in_ops = None
        self.loss = torch.zeros(B, dtype=torch.float32, device=dev)
        self.pred = torch.zeros(B, dtype=torch.int32, device=dev)
        # evaluation writes its own outputs so it never clobbers the training step's loss
        # (read by the optimizer's finite gate)
        self.eval_loss = torch.zeros(B, dtype=torch.float32, device=dev)
        self.eval_pred = torch.zeros(B, dtype=torch.int32, device=dev)
        hdl = L[-1]
        self.head_gw_part = torch.zeros((B, hdl.k * hdl.k * hdl.cin), dtype=torch.float32,
                                        device=dev)
        self.head_dzb = torch.zeros((B, NUM_POINTS), dtype=torch.float32, device=dev)

        self.side = torch.cuda.Stream(device=dev) if self.side_mode != "none" else None
        # DG_CHECK_STREAMS=1: every cross-stream hand-off bracketed by timing events, verified
        # after each eager step (utils/streamcheck.py; check_streams())
        self.sc = streamcheck.StreamCheck() if streamcheck.enabled() else None
        self._head_red_defer = False
        self._head_red_pending = False
        self._refresh_table = self._build_refresh_table()
        self._step_refresh = None   # the per-step table (plain copies no launch reads dropped)
        self.launches = 0     # native launches issued through _run (SegmentedStep counts them)
        self._build_plans()
        self._head_red_defer = self.side_mode == "bias" and bool(self.wgroups)
        self.refresh_weights()
        self.grad_hooks: List[Tuple[int, Callable[[], None]]] = []  # (after bwd layer i, fn)

    def _g16(self, off: int) -> int:
        """Address of flat gradient element off in the bf16 twin (grad_wire='bf16')."""
        return self.grads16.data_ptr() + 2 * off

    # ------------------------------------------------------------------ planning
    def _build_refresh_table(self) -> np.ndarray:
        rows = []
        for p, wf, wd in zip(self.plans, self.wf, self.wd):
            spec = self.layout.layers[p.index]
            w = self.params[spec.w_off:spec.w_off + spec.w_numel]
            w8 = self.wf8[p.index]
            rows.append([w.data_ptr(), wf.data_ptr(), wd.data_ptr() if wd is not None else 0,
                         p.cout, p.cin, p.k * p.k, p.cinp, p.KP, p.KPd,
                         self.pbias_frag[p.index].data_ptr()
                         if self.pbias_frag[p.index] is not None else 0,
                         w8.data_ptr() if w8 is not None else 0,
                         self.fp8_scales.data_ptr() + 8 * p.index if w8 is not None else 0,
                         self.fp8_amax_w[p.index].data_ptr() if w8 is not None else 0,
                         self.params.data_ptr() + 4 * spec.b_off,
                         self.params.data_ptr() + 4 * spec.pos_off,
                         self.pbias[p.index].data_ptr() if self.pbias[p.index] is not None else 0,
                         _ptr(self.wfrag[p.index]), _ptr(self.wdfrag[p.index]),
                         _ptr(self.wf8frag[p.index]), _ptr(self.wd8frag[p.index])])
        return np.ascontiguousarray(np.array(rows, dtype=np.int64))

    def _build_plans(self):
        h, lay = self.h, self.layout
        P = self.params.data_ptr()
        G = self.grads.data_ptr()
        f4 = 4
        self._pre: List[Tuple[Callable, tuple]] = []
        self._fwd: List[Tuple[Callable, tuple]] = []
        self._fwd_owner: List[int] = []   # layer each forward launch belongs to
        self._bwd: List[List[Tuple[Callable, tuple]]] = []  # per layer (index order)
        self._pre.append((h.expand_features, (
            self.planes.data_ptr(), self.player.data_ptr(), self.rank.data_ptr(),
            self.x0.data_ptr(), self.B, self.plans[0].pad, INPUT_CP)))
        # the training step's input ops (the expansion moves into the forward stack's launch
        # when that runs the first layer, below)
        self._pre_train = self._pre
        for p in self.plans:
            spec = lay.layers[p.index]
            xin = self.x0 if p.index == 0 else self.act[p.index - 1]
            x_pad = spec.pad
            y_pad = lay.layers[p.index + 1].pad
            nxt = self.plans[p.index + 1] if p.index + 1 < len(self.plans) else None
            self._fwd_owner.append(p.index)
            if p.fp8:
                i = p.index
                S = self.fp8_scales.data_ptr()
                y8 = self.x8[i + 1].data_ptr() if nxt is not None and nxt.fp8 else 0
                self._fwd.append((h.conv_board_fp8, (
                    p.k, p.bm, self.wf8[i].data_ptr(), p.KP, p.cout, p.Mpad,
                    self.x8[i].data_ptr(), x_pad, p.cinp, self.B, self.act[i].data_ptr(), y8,
                    y_pad, P + spec.b_off * f4, P + spec.pos_off * f4, S + (2 * i - 1) * f4,
                    S + 2 * i * f4, S + (2 * i + 1) * f4,
                    self.fp8_amax.data_ptr() + i * 4 if y8 else 0,
                    self.relu_mask[i].data_ptr() if self.relu_mask[i] is not None else 0)))
            elif p.board and p.cout == 256 and self.wfrag[p.index] is not None:
                msk = self.relu_mask[p.index]
                self._fwd.append((h.conv_layer2, (
                    h.EPI_FWD, self.wfrag[p.index].data_ptr(),
                    self.pbias_frag[p.index].data_ptr(), xin.data_ptr(),
                    self.act[p.index].data_ptr(), msk.data_ptr() if msk is not None else 0,
                    p.cout, self.B)))
            elif p.board:
                msk = self.relu_mask[p.index]
                self._fwd.append((h.conv_board_ex, (
                    h.EPI_FWD, p.k, p.bm, self.wf[p.index].data_ptr(), p.KP, p.cout, p.Mpad,
                    xin.data_ptr(), x_pad, p.cinp, self.B,
                    self.act[p.index].data_ptr(), y_pad,
                    0, 0, self.pbias[p.index].data_ptr(), 0, 0,
                    msk.data_ptr() if msk is not None else 0)))
            elif self._l1_res_ok(p) and self.wfrag[0] is not None:
                # first layer on conv_l1_frag (conv_l1.hip): one board per workgroup, the
                # input frame gathered once into a conflict-free plane layout, fragment-ordered
                # weights streamed into VGPRs (when the forward stack does not absorb it)
                # (the feature expansion fused into its prologue: it writes x0 itself, so the
                # separate expansion launch leaves _pre)
                msk = self.relu_mask[0]
                self._fwd.append((h.conv_l1_frag, (
                    self.wfrag[0].data_ptr(), self.pbias_frag[0].data_ptr(), xin.data_ptr(),
                    self.B, p.cout, self.act[0].data_ptr(),
                    msk.data_ptr() if msk is not None else 0, self.planes.data_ptr(),
                    self.player.data_ptr(), self.rank.data_ptr())))
            elif self._l1_res_ok(p):
                # first layer board-resident (conv_l1.hip): the 23x23x40 input frame staged
                # once per board instead of a 5x5x40 im2col patch per pixel and tile
                msk = self.relu_mask[p.index]
                self._fwd.append((h.conv_l1, (p.k, self.wf[p.index].data_ptr(), p.KP, p.cout,
                                              p.Mpad, xin.data_ptr(), x_pad, p.cinp, self.B,
                                              self.act[p.index].data_ptr(), y_pad,
                                              P + spec.b_off * f4, P + spec.pos_off * f4,
                                              msk.data_ptr() if msk is not None else 0,
                                              self.pbias[p.index].data_ptr())))
            else:
                msk = self.relu_mask[p.index]
                self._fwd.append((h.conv_nt_ex, (h.EPI_FWD, p.k, p.bm, p.bn,
                                                 self.wf[p.index].data_ptr(), p.KP, p.cout,
                                                 p.Mpad, xin.data_ptr(), x_pad, p.cinp,
                                                 self.npix, self.act[p.index].data_ptr(), y_pad,
                                                 P + spec.b_off * f4, P + spec.pos_off * f4, 0,
                                                 0, msk.data_ptr() if msk is not None else 0)))
            if nxt is not None and nxt.fp8 and not p.fp8:
                # bf16 producer feeding an fp8 layer: quantize its output frame (owned by the
                # consumer: a fused fp8 stack quantizes its own input)
                i = p.index
                self._fwd_owner.append(i + 1)
                self._fwd.append((h.frame_to_fp8, (
                    self.act[i].data_ptr(), self.x8[i + 1].data_ptr(), self.act[i].numel(),
                    self.fp8_scales.data_ptr() + (2 * i + 1) * 4,
                    self.fp8_amax.data_ptr() + i * 4)))
        self._fuse_forward_stack()
        self._l2_tables = []
        self._fwd, self._fwd_owner = self._merge_layer2_runs(self._fwd, self._fwd_owner)
        if any(f is h.conv_l1_frag for f, _ in self._fwd):
            # conv_l1_frag (still in the list: the forward stack did not absorb the first
            # layer) expands the features itself and writes x0: no expansion launch
            self._pre = [op for op in self._pre if op[0] is not h.expand_features]
            self._pre_train = self._pre
        hd = self.head
        hx = self.act[-1]
        self._head_train = (h.head, (hd.k, hx.data_ptr(), hd.pad, hd.cin, self.B,
                                     P + hd.w_off * f4, P + hd.b_off * f4, P + hd.pos_off * f4,
                                     self.labels.data_ptr(), self.loss.data_ptr(),
                                     self.pred.data_ptr(), 0, self.dz[-1].data_ptr(),
                                     self.dzp[-1], self.head_gw_part.data_ptr(),
                                     0, self.head_dzb.data_ptr(),
                                     int(self.cfg.head_relu), 1.0 / self.global_batch))
        self._head_red = (h.head_reduce, (self.head_dzb.data_ptr(), self.head_gw_part.data_ptr(),
                                          self.B, hd.k * hd.k * hd.cin, G + hd.w_off * f4,
                                          G + hd.b_off * f4, G + hd.pos_off * f4, self._sf))
        if self.grads16 is not None:
            self._head_red = (h.head_reduce_w, self._head_red[1][:-1] + (
                self._g16(hd.w_off), self._g16(hd.b_off), self._g16(hd.pos_off), self._sf))
        self._head_eval = (h.head, (hd.k, hx.data_ptr(), hd.pad, hd.cin, self.B,
                                    P + hd.w_off * f4, P + hd.b_off * f4, P + hd.pos_off * f4,
                                    self.labels.data_ptr(), self.eval_loss.data_ptr(),
                                    self.eval_pred.data_ptr(), 0, 0, 0, 0, 0, 0,
                                    int(self.cfg.head_relu), 1.0 / self.global_batch))
        # training: the head runs inside the forward stack's launch when the stack ends at the
        # last hidden layer (its image is already in LDS; conv_stack2.hip + head_body.h);
        # evaluation keeps the standalone head.  DG_FUSE_HEAD=0 keeps the separate launch.
        self._fwd_train = self._fwd
        head_ok = (hd.k == 3 and hd.pad == 1 and self.dzp[-1] == 1
                   and os.environ.get("DG_FUSE_HEAD", "1") != "0")
        head_tail = (P + hd.w_off * f4, P + hd.b_off * f4, P + hd.pos_off * f4,
                     self.labels.data_ptr(), self.loss.data_ptr(), self.pred.data_ptr(),
                     self.dz[-1].data_ptr(), self.head_gw_part.data_ptr(),
                     self.head_dzb.data_ptr(), int(self.cfg.head_relu), 1.0 / self.global_batch)
        last = len(self.plans) - 1
        if (head_ok and self.stack and self.stack[-1] == last
                and (hd.cin == 128 or (hd.cin == 256 and self.stack_fp8))):
            first = self.stack[0]
            fused = (h.conv_stack2_fwd_head, (
                self._stack_table.ctypes.data, len(self._stack_table),
                self._stack_x0.data_ptr(), int(self.stack_l1), self.B) + head_tail)
            if self.stack_fp8:
                # C = 128: the head on the last layer's LDS image; C = 256: on its bf16 frame,
                # read back at the end of the same launch (conv_stack_f8.hip)
                S, AM = self.fp8_scales.data_ptr(), self.fp8_amax.data_ptr()
                fused = (h.conv_stack_f8_fwd_head, (
                    hd.cin, self._stack_table.ctypes.data, len(self.stack),
                    self.act[first - 1].data_ptr(), S + 4 * (2 * (first - 1) + 1),
                    AM + 4 * (first - 1), self.B) + head_tail)
                if self.fp8_wgrad:
                    fused = (h.conv_stack_f8_fwd_head_y8, fused[1] + (self._fwd_y8.ctypes.data,))
            elif self.stack_l1 and self._stack_x0 is self.x0:
                # the feature expansion fused into the stack's first-layer prologue: the
                # launch builds its staged input planes from the packed batch and writes the
                # expanded frame x0 for the first layer's weight gradient (no expansion launch
                # and no x0 gather before the stack; evaluation keeps both)
                fused = (h.conv_stack2_fwd_head_x, (
                    self._stack_table.ctypes.data, len(self._stack_table), self.x0.data_ptr(),
                    self.B, self.planes.data_ptr(), self.player.data_ptr(),
                    self.rank.data_ptr()) + head_tail)
                self._pre_train = [op for op in self._pre if op[0] is not h.expand_features]
            self._fwd_train = [fused if f in (h.conv_stack2_fwd, h.conv_stack_f8,
                                              h.conv_stack_f8_y8) else (f, a)
                               for f, a in self._fwd]
        elif (head_ok and hd.cin == 256 and self._fwd
              and self._fwd[-1][0] is h.conv_layer2_multi
              and self._fwd[-1][1][0] == h.EPI_FWD
              and any(t.ctypes.data == self._fwd[-1][1][1]
                      and int(t[-1, 3]) == self.act[-1].data_ptr() for t in self._l2_tables)):
            # d = 256 bf16: the policy head at the end of the forward run's launch
            # (conv_layer2_multi HEAD: each board's head on the frame its workgroup just wrote)
            _, a = self._fwd[-1]
            self._fwd_train = self._fwd[:-1] + [(h.conv_layer2_multi_head,
                                                 (a[1], a[2], self.B) + head_tail)]
        if any(f in (h.conv_stack2_fwd_head, h.conv_stack2_fwd_head_x,
                     h.conv_stack_f8_fwd_head, h.conv_stack_f8_fwd_head_y8,
                     h.conv_layer2_multi_head)
               for f, _ in self._fwd_train):
            self._head_train = (self._noop, ())
        for p in self.plans:
            spec = lay.layers[p.index]
            i = p.index
            ops = []
            dzp = self.dzp[i]
            xin = self.x0 if i == 0 else self.act[i - 1]
            # bias grads: pass 1 (per board-chunk partials); pass 2 runs inside the slab
            # reduce launch, which also finalises the weight grad
            slab, bpart = self.slabs[i].data_ptr(), self.bparts[i].data_ptr()
            bch = self.bchunks
            if i == 0 and os.environ.get("DG_L0_BIAS_SMALL", "1") != "0":
                # the first layer's partials on the multi-layer kernel's 256-thread,
                # 48-VGPR workgroups (64-board chunks): they fit beside the window kernel's
                # workgroups, where the single-layer launch's 600-thread ones wait for free
                # CUs (12x256 bf16: 552 us on the side stream's critical chain)
                self._l0_btab = np.ascontiguousarray(
                    np.array([[self.dz[i].data_ptr(), bpart, 0]], dtype=np.int64))
                bch = self.bchunks_g
                ops.append((h.bias_grad_partial_multi, (self._l0_btab.ctypes.data, 1, self.B,
                                                        p.cout, dzp, self._sf)))
            else:
                ops.append((h.bias_grad_partial, (self.dz[i].data_ptr(), self.B, p.cout, dzp,
                                                  bpart)))
            # (the first layer's 5x5 as a sliding window over its 23 x 23 input frames was
            # measured slower: profiles/r4_s1_wgrad_l0_window_ab.txt)
            ops.append((h.conv_wgrad, (p.k, self.dz[i].data_ptr(), dzp, p.cout, p.Mpad_w,
                                       xin.data_ptr(), spec.pad, p.cinp, self.B, p.KPw,
                                       p.splits, slab)))
            red = (slab, G + spec.w_off * f4, p.splits, p.cout, p.Mpad_w, p.KPw, p.k * p.k,
                   p.cin, p.cinp, bpart, bch, G + spec.pos_off * f4,
                   G + spec.b_off * f4)
            self._red_src[i] = (slab, bpart, p.splits, p.Mpad_w, p.KPw, bch)
            if self.grads16 is not None:
                ops.append((h.wgrad_reduce_w, red + (self._g16(spec.w_off),
                                                     self._g16(spec.pos_off),
                                                     self._g16(spec.b_off), self._sf)))
            else:
                ops.append((h.wgrad_reduce, red + (self._sf,)))
            if i > 0:
                prev = lay.layers[i - 1]
                if (p.board_d and self.wdfrag[i] is not None and p.cout == 256
                        and self.relu_mask[i - 1] is not None and self.dzp[i] == 1
                        and self.dzp[i - 1] == 1):
                    ops.append((h.conv_layer2, (
                        h.EPI_DGRAD, self.wdfrag[i].data_ptr(), 0, self.dz[i].data_ptr(),
                        self.dz[i - 1].data_ptr(), self.relu_mask[i - 1].data_ptr(), p.cout,
                        self.B)))
                elif p.board_d:
                    msk = self.relu_mask[i - 1]
                    ops.append((h.conv_board_ex, (
                        h.EPI_DGRAD, p.k, p.bm_d, self.wd[i].data_ptr(), p.KPd, p.cin, p.Mpad_d,
                        self.dz[i].data_ptr(), dzp, p.cout, self.B, self.dz[i - 1].data_ptr(),
                        self.dzp[i - 1], 0, 0, 0,
                        0 if msk is not None else self.act[i - 1].data_ptr(), spec.pad,
                        msk.data_ptr() if msk is not None else 0)))
                else:
                    ops.append((h.conv_nt, (h.EPI_DGRAD, p.k, p.bm_d, p.bn_d,
                                            self.wd[i].data_ptr(), p.KPd, p.cin, p.Mpad_d,
                                            self.dz[i].data_ptr(), dzp, p.cout, self.npix,
                                            self.dz[i - 1].data_ptr(), self.dzp[i - 1], 0, 0,
                                            self.act[i - 1].data_ptr(), spec.pad)))
            self._bwd.append(ops)
        self._fuse_dgrad_stack()
        self._bwd_pre, _ = self._merge_layer2_runs(self._bwd_pre)
        self._drop_unread_act_frames()

    def _drop_unread_act_frames(self):
        """fp8 forward stack with the MX-fp8 weight gradients: when no launch of the model
        reads the bf16 activation frame of any non-last stack layer (the weight gradients read
        the e4m3 copies, the backward-data chain the ReLU bits), null those rows' Y so the
        stack skips their dequantized bf16 copy-out (conv_stack_f8.hip MODE 16).
        ``self.act_frames_dropped`` lists the layers whose act frame is then not written."""
        self.act_frames_dropped = []
        self.dz_frames_dropped = []
        t = getattr(self, "_stack_table", None)
        if (not self.keep_act_frames and self.stack_fp8 and getattr(self, "_fwd_y8", None)
                is not None and isinstance(t, np.ndarray) and len(t) > 1):
            used = self._op_pointers(exclude=(t,))   # pointers read by every OTHER launch
            ys = [int(v) for v in t[:-1, 2]]
            if not any(y in used for y in ys):
                t[:-1, 2] = 0
                self.act_frames_dropped = list(self.stack[:-1])
        # the same for the fp8 backward-data stack's bf16 dZ frames (rows i -> dz[i - 1]):
        # the MX-fp8 weight gradients and the bias partials read the e5m2 copies instead
        t = getattr(self, "_dstack_table", None)
        if (not self.keep_act_frames and self.dstack_fp8 and getattr(self, "_dstack_y8", None)
                is not None and isinstance(t, np.ndarray) and len(t) > 1):
            used = self._op_pointers(exclude=(t,))
            ys = [int(v) for v in t[:-1, 2]]
            if not any(y in used for y in ys):
                t[:-1, 2] = 0
                self.dz_frames_dropped = [i - 1 for i in self.dstack[:-1]]

    def _merge_layer2_runs(self, ops, owners=None):
        """Consecutive conv_layer2 launches of one kind whose layers chain (X of the next =
        Y of the previous) become ONE conv_layer2_multi launch: one workgroup per board runs
        the whole run, the second output half of a layer starts on a prefetched input chunk
        and the epilogue stores drain under the next half's MFMAs (csrc/kernels/
        conv_layer2.hip; bit-identical outputs).  DG_LAYER2_MULTI=0: per-layer launches."""
        h = self.h
        owners = list(owners) if owners is not None else [None] * len(ops)
        if os.environ.get("DG_LAYER2_MULTI", "1") == "0":
            return ops, owners
        out, out_own, run = [], [], []

        def flush():
            if len(run) >= 2:
                a0 = run[0][0][1]
                rows = [[a[1], a[2], a[3], a[4], a[5]] for (_, a), _ in run]
                tab = np.ascontiguousarray(np.array(rows, dtype=np.int64))
                self._l2_tables.append(tab)
                out.append((h.conv_layer2_multi, (a0[0], tab.ctypes.data, len(run), a0[6],
                                                  a0[7])))
                out_own.append(run[0][1])
            else:
                for op, ow in run:
                    out.append(op)
                    out_own.append(ow)
            run.clear()
        for op, ow in zip(ops, owners):
            f, a = op
            if f is h.conv_layer2:
                if run and (a[0] != run[-1][0][1][0] or a[3] != run[-1][0][1][4]
                            or len(run) == 16):
                    flush()
                run.append((op, ow))
            else:
                flush()
                out.append(op)
                out_own.append(ow)
        flush()
        return out, out_own

    def _fuse_forward_stack(self):
        """Replace the per-layer forward launches of the longest run of hidden 128->128 3x3
        bf16 layers by ONE conv_stack2_fwd launch (board-resident activations, overlapped
        stores; csrc/kernels/conv_stack2.hip).  DG_STACK=0 keeps per-layer kernels."""
        self.stack = []
        self.stack_fp8 = False
        self.stack_l1 = False
        if os.environ.get("DG_STACK", "1") == "0":
            return
        L = self.layout.layers
        fp8 = self.fp8

        def ok(p):
            if not (p.index > 0 and p.board and p.fp8 == fp8 and p.k == 3
                    and L[p.index].pad == 1 and L[p.index + 1].pad == 1):
                return False
            if not fp8 and p.cout != 128:
                return False          # (bf16 d = 256: per-layer conv_layer2)
            # bf16: 128 channels (conv_stack2); fp8: 128 or 256 (conv_stack_f8)
            return self.wf8frag[p.index] is not None if fp8 else self.wfrag[p.index] is not None
        best, cur = [], []
        for p in self.plans:
            cur = cur + [p.index] if ok(p) and (not cur or
                                                 self.plans[cur[0]].cout == p.cout) else []
            if len(cur) > len(best):
                best = list(cur)
        if len(best) < 2:
            return
        self.stack = best
        rows = []
        for i in best:
            m = self.relu_mask[i]
            if fp8 and m is None:
                # the fp8 stack always writes ReLU bits (its dgrad consumer may read them)
                m = self.relu_mask[i] = torch.zeros((self.B, NUM_POINTS, self.plans[i].cout // 8),
                                                    dtype=torch.uint8, device=self.device)
            if fp8:
                S, AM = self.fp8_scales.data_ptr(), self.fp8_amax.data_ptr()
                rows.append([self.wf8frag[i].data_ptr(), self.pbias_frag[i].data_ptr(),
                             self.act[i].data_ptr(), m.data_ptr(),
                             S + 4 * (2 * i - 1), S + 4 * 2 * i, S + 4 * (2 * i + 1), AM + 4 * i])
            else:
                rows.append([self.wfrag[i].data_ptr(), self.pbias_frag[i].data_ptr(),
                             self.act[i].data_ptr(), m.data_ptr() if m is not None else 0])
        first = best[0]
        # the first layer in front of the stack (conv_stack2.hip l1 mode): its input frame is
        # the expanded network input, its output act[0] leaves by the stack's copy-out
        self.stack_l1 = (not fp8 and first == 1 and self.wfrag[0] is not None
                         and self.relu_mask[0] is not None and self._stack_l1_ok(self.plans[0]))
        if self.stack_l1:
            rows.insert(0, [self.wfrag[0].data_ptr(), self.pbias_frag[0].data_ptr(),
                            self.act[0].data_ptr(), self.relu_mask[0].data_ptr()])
        self._stack_table = np.ascontiguousarray(np.array(rows, dtype=np.int64))
        self._stack_x0 = self.x0 if self.stack_l1 else self.act[first - 1]
        if self.stack_l1:
            members_l1 = {0}
        else:
            members_l1 = set()
        if fp8:
            # fp8 forward stack (conv_stack_f8.hip): quantizes its bf16 input frame itself
            # (amax -> fp8_amax[first - 1]), dequantized bf16 activations + ReLU bits out;
            # with the fp8 weight gradients also the raw e4m3 input of every stack layer
            # (x8q[l], l in the stack: the quantized input, then each non-last output)
            S, AM = self.fp8_scales.data_ptr(), self.fp8_amax.data_ptr()
            args = (self.plans[first].cout, self.h.EPI_FWD, self._stack_table.ctypes.data,
                    len(best), self.act[first - 1].data_ptr(), S + 4 * (2 * (first - 1) + 1),
                    AM + 4 * (first - 1), self.B)
            op = (self.h.conv_stack_f8, args)
            if self.fp8_wgrad:
                for i in best:
                    self.x8q[i] = torch.zeros(self.B * FP8_PITCH * self.plans[i].cin,
                                              dtype=torch.uint8, device=self.device)
                y8 = [self.x8q[first].data_ptr()] + [
                    self.x8q[i + 1].data_ptr() if i != best[-1] else 0 for i in best]
                self._fwd_y8 = np.ascontiguousarray(np.array(y8, dtype=np.int64))
                op = (self.h.conv_stack_f8_y8, args + (self._fwd_y8.ctypes.data,))
            self.stack_fp8 = True
        else:
            op = (self.h.conv_stack2_fwd, (self._stack_table.ctypes.data, len(rows),
                                          self._stack_x0.data_ptr(), int(self.stack_l1),
                                          self.B))
        # every launch owned by a stack layer goes; the stack launch takes the first's place
        members = set(best) | members_l1
        keep, placed = [], False
        for fop, owner in zip(self._fwd, self._fwd_owner):
            if owner in members:
                if not placed:
                    keep.append(op)
                    placed = True
            else:
                keep.append(fop)
        self._fwd = keep

    def _fuse_dgrad_stack(self):
        """Run the backward-data chain of the longest run of hidden 128->128 3x3 layers as
        ONE conv_stack launch in EPI_DGRAD mode: dZ_{i-1} = relu_mask_{i-1} * (W_i^T * dZ_i)
        for i = top .. bottom, board-resident in LDS (csrc/kernels/conv_stack2.hip).  The
        per-layer dgrad launches of those layers are dropped from ``_bwd``; their weight
        gradients run afterwards (they only read dZ_i).  DG_DSTACK=0 keeps per-layer dgrads."""
        self.dstack: List[int] = []
        self.dstack_fp8 = False
        self.wgroups: List[List[int]] = []
        self._bwd_pre: List[Tuple[Callable, tuple]] = []
        self._dgrad_first = False  # every dZ (down to dZ_0) produced in _bwd_pre
        self._dz8_exact = set()    # layers whose e5m2 gradient copy equals their bf16 dZ
        self._l0_side_at = None    # group top whose backward also runs layer 0's chain
        self._pre_dgrads = {}      # layer -> its dgrad ops moved into _bwd_pre
        self._l0_dgrad = []        # layer 1's dgrad (-> dZ_0) when it runs on the side stream
        if os.environ.get("DG_DSTACK", "1") == "0":
            self._dgrads_first()
            return
        L = self.layout.layers

        # fp8 models: the e5m2 backward-data stack (conv_stack_f8 EPI_DGRAD, 128 | 256 ch)
        fp8 = self.fp8 and any(w is not None for w in self.wd8frag)

        def ok(i):
            p = self.plans[i]
            if not (i > 0 and p.board_d and p.k == 3 and L[i].pad == 1
                    and self.dzp[i - 1] == 1 and p.KPd == p.KP
                    and self.relu_mask[i - 1] is not None):
                return False
            if fp8:
                return (self.wd8frag[i] is not None
                        and p.cout == self.plans[len(self.plans) - 1].cout)
            return p.cin == 128 and p.cout == 128 and self.wdfrag[i] is not None
        run = []
        for i in range(len(self.plans) - 1, 0, -1):   # must start at the top hidden layer
            if not ok(i):
                break
            run.append(i)
        if len(run) < 2:
            self._dgrads_first()
            return
        self.dstack = run
        self.dstack_fp8 = fp8
        if fp8:
            S = self.fp8_scales.data_ptr()
            GS, GA = self.fp8_gscales.data_ptr(), self.fp8_gamax.data_ptr()
            rows = [[self.wd8frag[i].data_ptr(), 0, self.dz[i - 1].data_ptr(),
                     self.relu_mask[i - 1].data_ptr(), GS + 4 * i, S + 4 * 2 * i,
                     GS + 4 * (i - 1), GA + 4 * (i - 1)] for i in run]
            self._dstack_table = np.ascontiguousarray(np.array(rows, dtype=np.int64))
            args = (self.plans[run[0]].cout, self._dstack_table.ctypes.data,
                    len(run), self.dz[run[0]].data_ptr(), GS + 4 * run[0], GA + 4 * run[0],
                    self.B)
            sr = self.step_count.data_ptr() if self.fp8_sr else 0
            if self.fp8_wgrad:
                # the raw e5m2 gradient of every run layer for the fp8 weight gradients:
                # dz8q[top] = the quantized input, dz8q[i - 1] = each non-last output
                for i in run:
                    self.dz8q[i] = torch.zeros(self.B * FP8_PITCH * self.plans[i].cout,
                                               dtype=torch.uint8, device=self.device)
                y8 = [self.dz8q[run[0]].data_ptr()] + [
                    self.dz8q[i - 1].data_ptr() if i != run[-1] else 0 for i in run]
                # dz8q[j] that are exactly the bf16 frame dz[j] (the copy-out bytes)
                self._dz8_exact = {i - 1 for i in run if i != run[-1]}
                self._dstack_y8 = np.ascontiguousarray(np.array(y8, dtype=np.int64))
                self._bwd_pre.append((self.h.conv_stack_f8_dgrad,
                                      args + (self._dstack_y8.ctypes.data, sr)))
            else:
                self._bwd_pre.append((self.h.conv_stack_f8_dgrad, args + (0, sr)))
        else:
            rows = [[self.wdfrag[i].data_ptr(), 0, self.dz[i - 1].data_ptr(),
                     self.relu_mask[i - 1].data_ptr()] for i in run]
            self._dstack_table = np.ascontiguousarray(np.array(rows, dtype=np.int64))
            self._bwd_pre.append((self.h.conv_stack2, (self.h.EPI_DGRAD,
                                                      self._dstack_table.ctypes.data, len(run),
                                                      self.dz[run[0]].data_ptr(), 0, self.B)))
        self._dstack_run = run
        for i in run:  # per-layer dgrad dropped: ops = [bias partial, wgrad, reduce]
            self._bwd[i] = self._bwd[i][:3]
        # the remaining per-layer dgrads below the stack (layer 1 -> dZ_0) right after it, so
        # every dZ exists before the weight gradients (the first layer's chain can then run
        # beside the grouped launch)
        if (os.environ.get("DG_DGRAD_FIRST", "1") != "0" and self.side_mode in ("none", "bias")
                and all(len(self._bwd[i]) <= 3 or i == run[-1] - 1
                        for i in range(1, run[-1]))):
            for i in range(run[-1] - 1, 0, -1):
                if len(self._bwd[i]) > 3:
                    self._pre_dgrads[i] = self._bwd[i][3:]
                    self._bwd_pre.extend(self._bwd[i][3:])
                    self._bwd[i] = self._bwd[i][:3]
            self._dgrad_first = True
        self._group_wgrads(set([run[0]] + [i - 1 for i in run]))

    def _dgrads_first(self):
        """No board-resident dgrad stack for this shape (e.g. 256 channels): still run the
        whole backward-data chain first — the per-layer dgrad launches, top to bottom, right
        after the head — so every dZ exists before the weight gradients and those can run
        as grouped launches (fewer split-K partials).  DG_DGRAD_FIRST=0 keeps the
        interleaved per-layer order."""
        if (os.environ.get("DG_DGRAD_FIRST", "1") == "0"
                or self.side_mode not in ("none", "bias")):
            return
        moved = []
        for i in range(len(self.plans) - 1, 0, -1):
            ops = self._bwd[i]
            if len(ops) > 3:
                self._pre_dgrads[i] = ops[3:]
                self._bwd_pre.extend(ops[3:])
                self._bwd[i] = ops[:3]
                moved.append(i)
        if moved:
            self._dgrad_first = True
            self._group_wgrads(set(range(len(self.plans))))

    def _layer2_ok(self, p: ConvPlan) -> bool:
        """A hidden 3x3 256 -> 256 bf16 layer runs forward and backward-data on conv_layer2.hip
        (weights streamed into VGPRs in fragment order, the board's input frame through two
        64-channel chunk buffers; DG_LAYER2=0: the board kernel conv_board.hip)."""
        lay = self.layout.layers
        return (p.index > 0 and not p.fp8 and p.board and p.k == 3 and p.cin == p.cout == 256
                and lay[p.index].pad == 1 and lay[p.index + 1].pad == 1
                and os.environ.get("DG_LAYER2", "1") != "0")

    def _stack_l1_ok(self, p: ConvPlan) -> bool:
        """The first layer can run inside the bf16 forward stack's launch (conv_stack2.hip l1
        mode: 5x5 over the 23x23x40 input frame, 128 outputs, K = 1024; DG_STACK_L1=0: its
        own conv_l1 launch)."""
        lay = self.layout.layers
        return (p.index == 0 and not self.fp8 and p.k == 5 and p.cinp == 40 and p.cout == 128
                and p.KP == 1024 and lay[0].pad == 2 and len(lay) > 2 and lay[1].pad == 1
                and os.environ.get("DG_STACK_L1", "1") != "0"
                and os.environ.get("DG_STACK", "1") != "0" and self._l1_res_ok(p))

    def _l1_frag_ok(self, p: ConvPlan) -> bool:
        """The 5x5 / 40-channel first layer on conv_l1_frag (conv_l1.hip: board per
        workgroup, fragment-ordered weights, conflict-free input planes) when the forward
        stack does not absorb it (d = 256, fp8 models).  DG_L1_FRAG=0: conv_l1."""
        lay = self.layout.layers
        return (p.index == 0 and p.KP == 1024 and len(lay) > 2 and self._l1_res_ok(p)
                and os.environ.get("DG_L1_FRAG", "1") != "0"
                and bool(self.h.conv_l1_frag_ok(p.k, lay[0].pad, p.cinp, p.cout, lay[1].pad)))

    def _l1_res_ok(self, p: ConvPlan) -> bool:
        """First layer on the board-resident kernel (conv_l1.hip) where its shape checks
        pass; otherwise the pixel-tiled implicit GEMM (conv_nt_ex)."""
        return (p.index == 0 and not p.board and not p.fp8
                and bool(self.h.conv_l1_ok(p.k, self.layout.layers[0].pad, p.cinp, p.Mpad, p.KP)))

    @staticmethod
    def _noop(*_):
        pass

    def _group_wgrads(self, dz_ready):
        """Weight gradients of up to DG_WGRAD_GROUP consecutive same-shape layers whose dZ
        the dgrad stack has already produced run as ONE three-slice launch
        (conv_wgrad_multi).  The machine is filled by the layers instead of by pixel
        splits, so each layer is cut into ~5x fewer splits: ~5x fewer fp32 partial slabs
        to write and reduce (50 -> 10 MB per 128-channel layer).

        Default group size: all hidden layers in one launch (12x128: 245k -> 248k boards/s
        vs groups of 4/5/7/10), under data parallelism too.  Round 1 used groups of 5 under
        DP so the first bucket's all-reduce could overlap the second group; round 2 measured
        that a comm-stream kernel does NOT co-schedule with these full-machine launches
        (every CU's VGPR file is full: bench.py --force-dp --comm proxy, 0% overlap,
        profiles/r2_comm_overlap_proxy.txt), so the split only costs."""
        self.wgroups: List[List[int]] = []
        self.win_groups = set()
        self.win8_groups = set()
        self._l0_side_at = None
        G = self._wgrad_group or int(os.environ.get("DG_WGRAD_GROUP", "16"))
        G = min(G, 16)                # MAXWL / RD_MAXL / BG_MAXL of the multi-layer kernels
        if G < 2 or self.side_mode not in ("none", "bias"):
            return
        lay = self.layout.layers
        h = self.h

        def key(i):
            p = self.plans[i]
            if (i not in dz_ready or p.k not in (3, 5)
                    or h.conv_wgrad_ktile(p.KPw) != 384):
                return None
            return (p.k, p.cout, p.Mpad_w, p.KPw, p.cinp, lay[i].pad)
        groups, cur = [], []
        for i in range(len(self.plans) - 1, -1, -1):
            k = key(i)
            if cur and (k is None or k != key(cur[0]) or len(cur) == G):
                groups.append(cur)
                cur = []
            if k is not None:
                cur.append(i)
        if cur:
            groups.append(cur)
        groups = [g for g in groups if len(g) >= 2]
        if not groups:
            return
        self.wgroups = groups
        # with dZ_0 produced up front (dgrad-first), the first layer's bias partial + wgrad +
        # reduce run on the side stream beside the last group's weight-gradient launch
        # Only when every layer from 1 up to the lowest group is itself grouped: an ungrouped
        # layer j below the group would run its per-layer wgrad on the main stream into the
        # shared slab / bias-partial buffers while layer 0's chain still uses them on the
        # side stream (e.g. 8 layers under DP: groups [6..2] and [1] -> [1] is dropped).
        grouped = set(i for g in groups for i in g)
        l0_ok = (self.side_mode == "bias" and self._dgrad_first and 0 not in grouped
                 and all(i in grouped for i in range(1, groups[-1][0] + 1)))
        # layer 0's gradient chain runs on the side stream after the last group's bias
        # partials (on the main stream before that group's launch measured -2.1% at 12x128,
        # -0.4% at 12x256: profiles/r2_l0_first_ab.txt; removed in round 3)
        self._l0_side_at = groups[-1][0] if l0_ok else None
        # layer 1's dgrad (-> dZ_0; d = 256 bf16, where the backward-data run stops at layer
        # 2) stays on the main stream before the grouped launch: on the side stream after the
        # bias partials it could not co-reside with the window workgroups (112 KB of LDS) and
        # stretched past the window kernel's end (12x256: +0.5% on the main stream once the
        # bias partials fit beside the window kernel; profiles/r3_bias_partial_small_wg.txt)
        wgs = h.conv_wgrad_wgs_per_cu_for(self.plans[groups[0][0]].KPw)
        gslab_elems = 0
        plan_splits = {}
        win_ok = os.environ.get("DG_WGRAD_WIN", "1") != "0"
        for g in groups:
            p = self.plans[g[0]]
            if (win_ok and p.k == 3 and lay[g[0]].pad == 1 and self.dzp[g[0]] == 1
                    and p.cout % 64 == 0 and p.cinp % 64 == 0 and p.KPw >= 9 * p.cinp):
                # sliding-window kernel (conv_wgrad_win.hip): one X window per K-step for
                # all 9 taps, 43 instead of 171 B of LDS-DMA per MFMA; fp8 models whose
                # stacks write the fp8 copies of every layer of the group: its MX-fp8 form
                # (conv_wgrad_win8.hip, one 4-wave workgroup per CU)
                self.win_groups.add(tuple(g))
                if (self.fp8_wgrad and self.B % 4 == 0
                        and all(self.x8q[i] is not None and self.dz8q[i] is not None
                                for i in g)):
                    self.win8_groups.add(tuple(g))
                    S = h.conv_wgrad_win8_splits(len(g), p.cout, p.cinp, self.B, self.num_cus)
                else:
                    S = h.conv_wgrad_win_splits(len(g), p.cout, p.cinp, self.B, self.num_cus)
                plan_splits[tuple(g)] = S
                gslab_elems = max(gslab_elems, len(g) * S * p.Mpad_w * p.KPw)
                continue
            tiles = (p.KPw // 384) * (p.Mpad_w // 128) * len(g)
            S = max(1, min((self.num_cus * wgs) // tiles, self.npix // 256))
            plan_splits[tuple(g)] = S
            gslab_elems = max(gslab_elems, len(g) * S * p.Mpad_w * p.KPw)
        self.gslab = torch.empty(gslab_elems, dtype=torch.float32, device=self.device)
        bpart_per = self.bchunks_g * (NUM_POINTS + 19) * max(self.plans[g[0]].cout for g in groups)
        self.gbpart = torch.empty(G * bpart_per, dtype=torch.float32, device=self.device)
        G_ = self.grads.data_ptr()
        f4 = 4
        self._wgroup_tables = []
        for g in groups:
            S = plan_splits[tuple(g)]
            p0 = self.plans[g[0]]
            spec0 = lay[g[0]]
            per = S * p0.Mpad_w * p0.KPw
            wrows, brows, rrows = [], [], []
            w8 = tuple(g) in self.win8_groups
            for j, i in enumerate(g):
                xin = self.x0 if i == 0 else self.act[i - 1]
                slab = self.gslab.data_ptr() + 4 * j * per
                bpart = self.gbpart.data_ptr() + 4 * j * bpart_per
                spec = lay[i]
                if w8:   # fp8 copies + their scales: gradient s_g[i], input s_y[i - 1]
                    wrows.append([self.dz8q[i].data_ptr(), self.x8q[i].data_ptr(), slab,
                                  self.fp8_gscales.data_ptr() + 4 * i,
                                  self.fp8_scales.data_ptr() + 4 * (2 * (i - 1) + 1)])
                else:
                    wrows.append([self.dz[i].data_ptr(), xin.data_ptr(), slab])
                # bias partials: from the e5m2 copy where it is exactly the bf16 frame (the
                # fp8 backward-data stack's copy-out; not its top input, which it rounds)
                if w8 and i in self._dz8_exact:
                    brows.append([self.dz8q[i].data_ptr(), bpart,
                                  self.fp8_gscales.data_ptr() + 4 * i])
                else:
                    brows.append([self.dz[i].data_ptr(), bpart, 0])
                rrows.append([slab, G_ + spec.w_off * f4, bpart, G_ + spec.pos_off * f4,
                              G_ + spec.b_off * f4, S, p0.cout, p0.Mpad_w, p0.KPw,
                              p0.k * p0.k, p0.cin, p0.cinp, self.bchunks_g]
                             + ([self._g16(spec.w_off), self._g16(spec.pos_off),
                                 self._g16(spec.b_off)] if self.grads16 is not None else []))
                self.plans[i].splits = S
                self._red_src[i] = (slab, bpart, S, p0.Mpad_w, p0.KPw, self.bchunks_g)
                # ops = [bias partial, wgrad, reduce, (dgrad)]: the group's first layer
                # launches all three passes for the whole group
                self._bwd[i][0:3] = [(self._noop, ())] * 3
            # layer 0's bias partials as one more row of the last group's launch (its chain
            # runs on the side stream right after it) at d = 128: 12x128 fp8 +1.1%, bf16
            # equal; at d = 256 the 5x5 weight gradient then starts earlier beside the window
            # kernel and stretches it (12x256 fp8 -6.6%, bf16 equal;
            # profiles/r4_s2_l0_bias_merge_ab.txt)
            p_l0 = self.plans[0]
            if (g is groups[-1] and self._l0_side_at is not None and len(brows) < 16
                    and p_l0.cout == p0.cout and p0.cout <= 128
                    and self.dzp[0] == self.dzp[g[0]]
                    and self._bwd[0][0][0] is h.bias_grad_partial_multi):
                brows.append([self.dz[0].data_ptr(), self.bparts[0].data_ptr(), 0])
                self._bwd[0][0] = (self._noop, ())
            tabs = [np.ascontiguousarray(np.array(r, dtype=np.int64))
                    for r in (wrows, brows, rrows)]
            self._wgroup_tables.extend(tabs)
            wt, bt, rt = tabs
            self._bwd[g[0]][0:3] = [
                (h.bias_grad_partial_multi, (bt.ctypes.data, len(bt), self.B, p0.cout,
                                             self.dzp[g[0]], self._sf)),
                (h.conv_wgrad_win8 if w8 else h.conv_wgrad_win,
                 (wt.ctypes.data, len(g), p0.cout, p0.Mpad_w, p0.cinp, self.B, p0.KPw, S,
                  self._sf))
                if tuple(g) in self.win_groups else
                (h.conv_wgrad_multi, (p0.k, wt.ctypes.data, len(g), self.dzp[g[0]],
                                      p0.cout, p0.Mpad_w, spec0.pad, p0.cinp, self.B, p0.KPw,
                                      S)),
                (h.wgrad_reduce_multi_w if self.grads16 is not None else h.wgrad_reduce_multi,
                 (rt.ctypes.data, len(rt))),
            ]

    # ------------------------------------------------------------------ execution
    def _run(self, ops, s):
        for f, a in ops:
            f(*a, s)
            if f is not HipGoNet._noop:
                self.launches += 1

    # ------------------------------------------------------------------ input prefetch
    def enable_prefetch(self) -> bool:
        """Double-buffered step inputs.  Every ``set_batch*`` copies into the buffer the
        previous step does NOT read, on a load stream that waits only for the step before
        that, so the copy (pinned H2D in the trainer, a D2D copy in the bench) runs beside the
        previous step instead of in front of the next one.  The launches that read the inputs
        (feature expansion, the heads: labels) exist once per buffer — the second set is the
        first with the input pointers substituted — and SegmentedStep captures one step graph
        per buffer.  Reference: the loader threads filling the next minibatch while the
        current one trains (/root/reference/data.lua:11-27).  Call before SegmentedStep.
        (A form with the copy as a memcpy node inside the step graph was measured and dropped
        in round 6: HIP runs a graph's H2D memcpy node as a blit kernel, which ran after the
        step's last kernel — +40 us per step; profiles/r6_host_pool_prefetch.txt.)"""
        if self.load_stream is not None:
            return True
        buf1 = torch.zeros_like(self.inbuf)
        v0 = unpack_views(self.inbuf, self.B)
        v1 = unpack_views(buf1, self.B)
        v1[1].fill_(1)
        v1[2].fill_(1)
        m = {a.data_ptr(): b.data_ptr() for a, b in zip(v0, v1)}

        def sub(op):
            f, a = op
            return (f, tuple(m.get(x, x) if type(x) is int else x for x in a))
        names = ("_pre", "_pre_train", "_fwd", "_fwd_train")
        ops0 = {n: list(getattr(self, n)) for n in names}
        ops0["_head_train"] = self._head_train
        ops0["_head_eval"] = self._head_eval
        ops1 = {n: [sub(op) for op in ops0[n]] for n in names}
        ops1["_head_train"] = sub(self._head_train)
        ops1["_head_eval"] = sub(self._head_eval)
        self._in_ops = [ops0, ops1]
        self._in_views = [v0, v1]
        self._inbufs = [self.inbuf, buf1]
        self.load_stream = torch.cuda.Stream(device=self.device)
        self._rel_ev = [torch.cuda.Event(), torch.cuda.Event()]
        return True

    def select_inputs(self, k: int):
        """Make input buffer k the one the (eager) launch lists read."""
        self.cur_in = k
        if self._in_ops is None:
            return
        for n, v in self._in_ops[k].items():
            setattr(self, n, v)
        self.inbuf = self._inbufs[k]
        self.planes, self.player, self.rank, self.labels = self._in_views[k]

    def _load(self, fill, device_src: bool):
        """Run ``fill(buffer, views)`` for the next batch: in place without prefetch; with it,
        into the other buffer on the load stream (after the step that last read it), and the
        compute stream waits for the copy before the next step's launches.  A device source
        may still be being written by work issued on the compute stream, so then the load
        stream waits for all of it (the overlap is for host sources: the loader's pinned
        slots, copied by the SDMA engines)."""
        if self.load_stream is None:
            fill(self.inbuf, (self.planes, self.player, self.rank, self.labels))
        else:
            main = torch.cuda.current_stream(self.device)
            self._rel_ev[self.cur_in].record(main)       # all issued reads of the current one
            t = 1 - self.cur_in
            self.load_stream.wait_event(self._rel_ev[1 - t if device_src else t])
            with torch.cuda.stream(self.load_stream):
                fill(self._inbufs[t], self._in_views[t])
                ready = torch.cuda.Event()
                ready.record(self.load_stream)
            if self.sc:
                self.sc.produce("load->compute", self.load_stream)
            main.wait_event(ready)
            if self.sc:
                self.sc.consume("load->compute", main)
            self.select_inputs(t)
        if not self._fp8_calibrated:
            self.calibrate_fp8()

    def set_batch(self, planes: torch.Tensor, player: torch.Tensor, rank: torch.Tensor,
                  labels: torch.Tensor, non_blocking: bool = True):
        """Copy one batch into the static input buffers (device or pinned host tensors)."""
        def fill(_, v):
            v[0].copy_(planes.reshape(self.B, 9, NUM_POINTS), non_blocking=non_blocking)
            v[1].copy_(player, non_blocking=non_blocking)
            v[2].copy_(rank, non_blocking=non_blocking)
            v[3].copy_(labels, non_blocking=non_blocking)
            if self.load_stream is not None:
                for x in (planes, player, rank, labels):
                    if x.is_cuda:
                        x.record_stream(self.load_stream)
        self._load(fill, any(x.is_cuda for x in (planes, player, rank, labels)))

    def set_batch_packed(self, packed: torch.Tensor, non_blocking: bool = True):
        """One copy of a ``pack_batch`` buffer (device or pinned host) into the inputs."""
        def fill(buf, _):
            buf.copy_(packed, non_blocking=non_blocking)
            if packed.is_cuda and self.load_stream is not None:
                packed.record_stream(self.load_stream)
        self._load(fill, packed.is_cuda)

    def set_batch_packed_from(self, loader):
        """Next batch of a BatchLoader with pinned packed slots: one async copy (the loader
        releases the slot on an event recorded on the stream that copied it)."""
        self._load(lambda buf, _: loader.next_packed_to(buf), False)

    def forward(self):
        s = stream_handle()
        self._run(self._pre, s)
        self._run(self._fwd, s)

    def forward_backward(self):
        """Loss/pred into self.loss/self.pred; gradients (mean over global batch) in
        self.grads.  Registered grad hooks fire right after their layer's wgrad."""
        s = stream_handle()
        # (no gradient zeroing: every gradient entry is written — not accumulated — by the
        # slab reduces and the deterministic head reduce)
        self._run(self._pre_train, s)
        self._run(self._fwd_train, s)
        self._run([self._head_train], s)
        self.head_reduce()
        self._run(self._bwd_pre, s)
        hooks = dict()
        for li, fn in self.grad_hooks:
            hooks.setdefault(li, []).append(fn)
        if hooks.get(self.L - 1):
            self.join_side()            # the head's gradients final (deferred reduce)
        for fn in hooks.get(self.L - 1, []):
            fn()
        for i in range(self.L - 2, -1, -1):
            self.backward_layer(i, hooks.get(i, ()))
        self.join_side()

    def head_reduce(self):
        """The head's weight / bias gradient reduce over the fused head's per-board partials.
        Nothing before the optimizer reads it.  With the side stream and grouped weight
        gradients it is deferred: the first group's side-stream work
        runs it beside the grouped wgrad launch, whose 2-per-CU grid leaves CUs free (it does
        not co-schedule beside the backward-data stack: run there the step was 1% slower)."""
        if self._head_red_defer:
            self._head_red_pending = True
            return
        self._run([self._head_red], stream_handle())

    def _flush_head_reduce(self, stream):
        if self._head_red_pending:
            self._head_red_pending = False
            self._run([self._head_red], stream)

    def backward_layer(self, i: int, hooks=()):
        """Layer i's backward: bias grads + wgrad + slab reduce (final grads of layer i, then
        ``hooks``) and the dgrad into layer i-1.  The two halves only share dZ_i (read-only),
        so with a side stream the weight-gradient chain runs beside the dgrad chain — the
        critical path is the dgrad sequence, and each kernel's ramp/tail is filled by the
        other stream's work.  Callers end the backward with ``join_side()``."""
        ops = self._layer_ops(i)
        main = torch.cuda.current_stream()
        if self.side_mode == "none":
            self._run(ops[:3], main.cuda_stream)
            for fn in hooks:
                fn()
        elif self.side_mode == "bias":
            side = self.side
            l0_side = self._l0_side_at == i
            sc = self.sc
            if i == 0 and self._l0_side_at is not None:
                if sc:
                    sc.produce("l0-chain->main", side)
                main.wait_stream(side)           # layer 0's chain ran on the side stream
                if sc:
                    sc.consume("l0-chain->main", main)
            else:
                if sc:
                    sc.produce("dz->side", main)
                side.wait_stream(main)           # dZ of the layer (group) final
                if sc:
                    sc.consume("dz->side", side)
                self._flush_head_reduce(side.cuda_stream)
                self._issue_loss_gate(side.cuda_stream)
                self._run(ops[:1], side.cuda_stream)
                l0 = self._l0_dgrad + self._layer_ops(0)[:3] if l0_side else None
                if l0_side and self._defer:
                    # layer 0's bias partial (where it is a launch of its own: d = 256) and
                    # what produces its dZ_0 BEFORE the event the early update waits on: the
                    # partial's |dZ_0| check is a step-tag producer, and the early update must
                    # read the tag only after every producer (all-or-nothing).  The
                    # 5x5 slab reduce after it cannot trip on its own: |dZ_0| < 2^100 and
                    # x0 in {0, 1} bound the 5x5 gradient below the reduce's 2^120
                    k = len(self._l0_dgrad) + 1
                    self._run(l0[:k], side.cuda_stream)
                    l0 = l0[k:]
                ev = side.record_event()         # partials ready for the reduce
                if sc:
                    sc.produce("partials->reduce", side)
                # then dZ_0 and the first layer's whole chain, joined at layer 0.  Measured
                # (profiles/r3_l0_chain_stream_ab.txt): the chain before the partials, or on a
                # third stream beside the grouped launch, is 5-6% slower at 12x128 and
                # 0.3-1.6% at 12x256 — compute beside the window kernel slows it; and its
                # bias partial on the main stream after the window kernel (its 5x5 weight
                # gradient then starts ~50 us earlier beside it) stretched the fp8 window
                # kernel by 100 us: -6% at 12x256 fp8, 0 elsewhere
                # (profiles/r4_s1_l0_bias_main_ab.txt)
                if l0_side:
                    self._run(l0, side.cuda_stream)
                self._run(ops[1:2], main.cuda_stream)
                main.wait_event(ev)
                if sc:
                    sc.consume("partials->reduce", main)
                self._run(ops[2:3], main.cuda_stream)
                if l0_side:
                    self._issue_early_update(main.cuda_stream)
            for fn in hooks:
                fn()
        self._run(ops[3:], main.cuda_stream)

    def _issue_loss_gate(self, stream):
        """With the gradient pass 2 deferred the update's gate is the loss alone: issue it on
        the side stream as soon as the loss exists (beside the weight-gradient launch), not
        in front of the fused update."""
        if (self._defer and not self._gate_issued and self.cfg.nan_policy != "raise"
                and self.grads16 is None):
            self._run([(self.h.finite_gate, (self.loss.data_ptr(), self.B, 0, 0,
                                             self.gate.data_ptr(), self.bad_steps.data_ptr()))],
                      stream)
            self._gate_issued = True

    def _layer_ops(self, i: int):
        """Layer i's backward ops [bias partial, wgrad, pass 2, (dgrad)]; with the step's
        gradient pass 2 deferred into the fused update, the pass-2 launch (the slab reduce
        that also finishes the bias gradients) is left out."""
        ops = self._bwd[i]
        if self._defer and len(ops) >= 3 and i in self._defer_layers():
            ops = ops[:2] + [(self._noop, ())] + ops[3:]
        return ops

    def _defer_layers(self) -> set:
        """Layers whose pass 2 the fused update takes over when deferred: the grouped
        weight-gradient launch's layers (their slabs / partials are regions of their own, ~12
        splits each).  A layer outside it (the first layer's side-stream chain: 64 splits of
        a 5x5 x 40 K) keeps its own slab reduce — its wide split-K sum is a poor fit for the
        update's per-tile blocks (measured: 128 us for the fused kernel with it, the reduce
        alone 10 us)."""
        return set(self.wgroups[0]) if len(self.wgroups) == 1 else set()

    def can_defer(self) -> bool:
        """Whether a training step may leave its gradients as split-K slabs and bias partials
        for the fused update (grad_update: pass 2 + SGD / RMSProp + operand refresh + LR decay
        in one launch) instead of reducing them first.  Needs a single-GPU step (a collective
        needs the reduced gradient; the bf16 wire twin is a DP format), no gradient hooks, and
        every layer's slabs / partials in buffers of their own: one grouped weight-gradient
        launch, plus at most the first layer's own chain.  DG_FUSED_UPDATE=0: never (and the
        optimizer keeps the separate SGD + refresh launches)."""
        if os.environ.get("DG_FUSED_UPDATE", "1") == "0":
            return False
        if self.global_batch != self.B or self.grads16 is not None or self.grad_hooks:
            return False
        if len(self.wgroups) != 1:
            return False
        return all(i in self._red_src for i in self.wgroups[0])

    def set_defer(self, on: bool):
        """Issue the following backward + optimizer_step with the gradient pass 2 deferred
        into the fused update (see can_defer; ignored when it does not hold)."""
        self._defer = bool(on) and self.can_defer()

    def join_side(self):
        self._flush_head_reduce(stream_handle())
        if self.side is not None:
            cur = torch.cuda.current_stream()
            if self.sc:
                self.sc.produce("side->join", self.side)
            cur.wait_stream(self.side)
            if self.sc:
                self.sc.consume("side->join", cur)

    def check_streams(self) -> int:
        """DG_CHECK_STREAMS=1: synchronize and verify every cross-stream hand-off recorded
        since the last check (raises on a violation); returns how many were checked (0 when
        the mode is off or the step ran inside a graph capture)."""
        return self.sc.check() if self.sc else 0

    def evaluate(self):
        s = stream_handle()
        self._run(self._pre, s)
        self._run(self._fwd, s)
        f, a = self._head_eval
        f(*a, s)

    def optimizer_step(self, grad_scale: float = 1.0):
        """The update: [finite gate] -> [fp8 scale update] -> ONE fused launch (grad_update:
        the gradient's pass 2 when the step deferred it, SGD / RMSProp on every parameter,
        the operand copies the next step reads, LR decay).  DG_FUSED_UPDATE=0: the separate
        SGD / RMSProp and weight-refresh launches."""
        s = stream_handle()
        n = self.layout.numel
        gate = 0
        slabs = self._defer
        # (bf16 wire: the optimizer reads the all-reduced bf16 twin)
        w16 = self.grads16 is not None
        g = self.grads16.data_ptr() if w16 else self.grads.data_ptr()
        if self.cfg.nan_policy != "raise" and not (slabs and self._gate_issued):
            # gate = finite(loss) [and finite(gradients)]: under DP every rank sees the same
            # all-reduced gradient, so all ranks skip together.  With the pass 2 deferred the
            # gradient does not exist yet: the gate is the loss, and the fused update leaves
            # any non-finite gradient entry unapplied (and counts the step in bad_steps)
            dp = self.global_batch != self.B
            # (one launch: the loss check and the gradient scan together)
            self.h.finite_gate1(0 if dp else self.loss.data_ptr(), self.B,
                                0 if (slabs or w16) else g, g if (w16 and not slabs) else 0,
                                0 if slabs else n, self.gate.data_ptr(),
                                self.bad_steps.data_ptr(), self._gate_ticket.data_ptr(), s)
            gate = self.gate.data_ptr()
        if self.cfg.nan_policy != "raise":
            gate = self.gate.data_ptr()
        self._gate_issued = False
        if not (slabs and self._early_issued):
            self._fp8_update(s)
        if os.environ.get("DG_FUSED_UPDATE", "1") == "0":
            if self.ms is not None:
                (self.h.rmsprop_bf16 if w16 else self.h.rmsprop)(
                    self.params.data_ptr(), g, self.ms.data_ptr(), n, self.lr.data_ptr(),
                    float(self.cfg.rmsprop_decay), grad_scale, gate, s)
            else:
                (self.h.sgd_bf16 if w16 else self.h.sgd)(self.params.data_ptr(), g, n,
                                                         self.lr.data_ptr(), grad_scale, gate, s)
            # bf16 (+ e4m3) operand copies of the updated weights + lr *= (1 - rateDecay)
            t = self._step_refresh_table()
            self.h.weight_refresh_decay(t.ctypes.data, len(t), self.lr.data_ptr(),
                                        float(self.cfg.rateDecay), self.step_count.data_ptr(), s)
            return
        t = self._gu_table(slabs)
        hd = self.head
        plain = (hd.w_off, n - hd.w_off)
        if slabs and self._early_issued:
            # the hidden layers and the head were updated by the early launch (beside the
            # first layer's gradient chain): the rest, then the LR decay
            t = self._gu_split(t)[1]
            plain = (0, 0)
        self._early_issued = False
        self._gu_launch(t, plain, grad_scale, gate, 1, s)

    def _gu_launch(self, t, plain, grad_scale, gate, final, s):
        w16 = self.grads16 is not None
        self.h.grad_update(t.ctypes.data, len(t), plain[0], plain[1],
                           self.params.data_ptr(), self.grads.data_ptr(),
                           self.grads16.data_ptr() if w16 else 0,
                           self.ms.data_ptr() if self.ms is not None else 0,
                           float(self.cfg.rmsprop_decay), grad_scale, gate, self.lr.data_ptr(),
                           float(self.cfg.rateDecay), self.step_count.data_ptr(),
                           self.gu_tickets.data_ptr(), self.bad_steps.data_ptr(),
                           int(self.keep_grads), final,
                           # the step tag is rank-local: under DP the all-reduced gradient's
                           # full finite gate decides (the same on every rank)
                           self._sf + 8 if self.global_batch == self.B else 0, s)

    def _gu_split(self, t):
        """(early rows, late rows) of a deferred step's grad_update table: the grouped
        launch's layers (their slabs and bias partials exist once it ends) | the rest (the
        first layer: its side-stream chain ends later)."""
        sp = getattr(self, "_gu_split_tabs", None)
        if sp is None:
            early = self._defer_layers()
            idx_e = [k for k, p in enumerate(self.plans) if p.index in early]
            idx_l = [k for k, p in enumerate(self.plans) if p.index not in early]
            sp = (np.ascontiguousarray(t[idx_e]), np.ascontiguousarray(t[idx_l]))
            self._gu_split_tabs = sp
        return sp

    def _issue_early_update(self, stream):
        """Deferred single-GPU step: update the grouped launch's layers and the head as soon
        as their gradients exist (right after the grouped weight-gradient launch, on the main
        stream beside the first layer's side-stream chain) instead of after it; the fused
        update's final launch then covers only the first layer and decays the LR.  Taken with
        the MX-fp8 weight gradients (the early launch fills the CUs the fp8 window kernel
        leaves while the first layer's 5x5 gradient finishes: +1.1% at 12x256 fp8) and at
        d >= 256 in bf16 (+0.4% at 12x256 once its window kernel runs at wave priority 1); the
        bf16 step at 12x128 measured 0.6% slower / equal with it
        (profiles/r4_s1_early_update_park_ab.txt, profiles/r4_s2_early_update_ab.txt).
        DG_EARLY_UPDATE=0 / 1: never / always."""
        if not (self._defer and self._early_ok and self.cfg.nan_policy != "raise"
                and len(self._gu_split(self._gu_table(True))[1]) > 0):
            return
        if (self._early_env is None and not self.win8_groups
                and max(self.plans[i].cout for g in self.wgroups for i in g) < 256):
            return
        self._fp8_update(stream)
        hd = self.head
        t = self._gu_split(self._gu_table(True))[0]
        self._gu_launch(t, (hd.w_off, self.layout.numel - hd.w_off), 1.0,
                        self.gate.data_ptr(), 0, stream)
        self._early_issued = True

    def _gu_table(self, slabs: bool) -> np.ndarray:
        """grad_update's table: the per-step refresh row of every conv layer + where its
        gradient comes from (slabs: the split-K slabs / bias partials of its pass 2; else the
        flat gradient) and its parameter offsets."""
        key = "_gu_tab_slabs" if slabs else "_gu_tab_grads"
        t = getattr(self, key, None)
        if t is None:
            ref = self._step_refresh_table()
            rows = []
            for r, p in zip(ref, self.plans):
                spec = self.layout.layers[p.index]
                src = (self._red_src[p.index] if slabs and p.index in self._defer_layers()
                       else (0, 0, 0, 0, 0, 0))
                rows.append([int(x) for x in r] + [int(x) for x in src]
                            + [spec.w_off, spec.b_off, spec.pos_off])
            t = np.ascontiguousarray(np.array(rows, dtype=np.int64))
            assert t.shape[1] == self.h.grad_update_cols()
            setattr(self, key, t)
        return t

    def _op_pointers(self, exclude=()) -> set:
        """Every integer argument (and int64 table entry) of the launches the model issues:
        the input / forward / head / backward op lists that forward(), forward_backward(),
        evaluate() and backward_layer() run."""
        vals = set()

        def add(op):
            f, a = op
            for v in a:
                if isinstance(v, int):
                    vals.add(v)
        for lst in (self._pre, self._fwd, self._fwd_train, self._bwd_pre,
                    getattr(self, "_l0_dgrad", []), *self._bwd):
            for op in lst:
                add(op)
        for op in (self._head_train, self._head_red, self._head_eval):
            add(op)
        # every int64 launch table the model holds (stack / dgrad-stack / layer-run / grouped
        # weight-gradient / fp8 copy-out tables), except the refresh tables (operand copies
        # are what _step_refresh_table decides about) and any passed in `exclude`
        skip = {id(getattr(self, "_refresh_table", None)), id(getattr(self, "_step_refresh", None)),
                id(getattr(self, "_gu_tab_slabs", None)), id(getattr(self, "_gu_tab_grads", None))}
        skip.update(id(t) for t in exclude)
        for name, v in vars(self).items():
            for t in (v if isinstance(v, (list, tuple)) else [v]):
                if (isinstance(t, np.ndarray) and t.dtype == np.int64 and id(t) not in skip):
                    vals.update(int(x) for x in t.ravel())
        return vals

    def _step_refresh_table(self) -> np.ndarray:
        """The optimizer's refresh table: the full one minus the operand copies no launch of
        the model reads — the plain bf16 / e4m3 layouts where the board-resident stacks read
        fragment-ordered ones, and fragment orders of paths not taken (an fp8 model's bf16
        fragments, ...) — so the per-step refresh does not rewrite them.  Built on the first
        optimizer step, when every launch table exists."""
        if self._step_refresh is None:
            used = self._op_pointers()
            t = self._refresh_table.copy()
            # wf, wd, wf8 (plain) and wf_frag, wd_frag, wf8_frag, wd8_frag (stack orders)
            for col in (1, 2, 10, 16, 17, 18, 19):
                for r in range(len(t)):
                    if t[r, col] and int(t[r, col]) not in used:
                        t[r, col] = 0
            self._step_refresh = np.ascontiguousarray(t)
        return self._step_refresh

    def refresh_weights(self):
        """bf16 (and fp8) operand copies of the fp32 master weights (init / load)."""
        s = stream_handle()
        n = len(self._refresh_table)
        self.h.weight_refresh(self._refresh_table.ctypes.data, n, s)
        if self.fp8:  # first pass observed |w| max: derive s_w, requantize with it
            self._fp8_update(s)
            self.h.weight_refresh(self._refresh_table.ctypes.data, n, s)

    def _fp8_update(self, s):
        """Delayed scaling: s_w from the last refresh's weight amax (+5%), s_y from the last
        forward's activation amax; runs BEFORE the refresh that quantizes with s_w."""
        if self.fp8:
            self.h.fp8_update_scales(len(self.plans), self.fp8_scales.data_ptr(),
                                     self.fp8_amax_w.data_ptr(), REFRESH_PARTS,
                                     self.fp8_amax.data_ptr(), FP8_W_MARGIN, FP8_G_HEADROOM,
                                     self.fp8_sat.data_ptr(), self.fp8_gscales.data_ptr(),
                                     self.fp8_gamax.data_ptr(), self.fp8_ghist.data_ptr(), s)

    def calibrate_fp8(self):
        """Forward(+backward) passes on the current inputs to observe activation (and, with
        the fp8 backward-data stack, gradient) ranges, then derive the fp8 scales (called
        automatically on the first batch of an fp8 model).  Three passes: each layer's range
        is observed through inputs quantized with the scales of the pass before."""
        s = stream_handle()
        for _ in range(3):
            if self.dstack_fp8:
                self.forward_backward()
            else:
                self.evaluate()
            self._fp8_update(s)
            self.h.weight_refresh(self._refresh_table.ctypes.data, len(self._refresh_table), s)
        self.fp8_sat.zero_()   # the calibration passes start from unit scales
        self._fp8_calibrated = True

    def train_step(self):
        """forward + backward + update; the gradient pass 2 deferred into the fused update
        when can_defer() holds (self.grads is then written by that launch)."""
        self.set_defer(True)
        try:
            self.forward_backward()
            self.optimizer_step()
        finally:
            self._defer = False

    # ------------------------------------------------------------------ helpers
    def mean_loss(self) -> torch.Tensor:
        return self.loss.sum() / self.B

    def correct(self) -> torch.Tensor:
        return (self.pred == self.labels).sum()

    def load_params(self, flat: torch.Tensor):
        self.params.copy_(flat.to(self.params.device, torch.float32))
        self.refresh_weights()

    def state_tensors(self):
        return {"params": self.params, "lr": self.lr, "step": self.step_count}

    def memory_bytes(self) -> int:
        uniq = {t.data_ptr(): t for t in (*self.slabs, *self.bparts)}
        ts = [self.params, self.grads, *uniq.values(), self.x0, *self.act, *self.dz, *self.wf,
              *[w for w in self.wd if w is not None]]
        return sum(t.numel() * t.element_size() for t in ts)


class SegmentedStep:
    """The training step (forward, backward, [gradient all-reduce], optimizer) as hipGraphs.

    Modes (``self.mode``):
      graph      no collectives: the whole step is ONE graph (a graph-to-graph boundary costs
                 ~10 us of idle GPU per step);
      dp-graph   native RCCL communicator (parallel/dp.py NativeComm): still ONE graph.  After
                 the backward of the lowest layer of each gradient bucket, the comm stream is
                 forked from the compute stream by an event and the bucket's ncclAllReduce is
                 captured there, so it overlaps the remaining backward; the compute stream
                 joins the comm stream before the optimizer.  No host work per bucket;
      dp-segments torch.distributed communicator: graph segments between buckets, the
                 all-reduces issued from the host between segment replays (the fallback);
      eager      no graphs (debugging, ``--no-graph``).
    Segment boundaries sit right after the wgrad of the lowest layer of each DP bucket
    (``parallel.dp.make_buckets``)."""

    def __init__(self, net: HipGoNet, bucketer=None, use_graphs: bool = True, warmup: int = 1):
        self.net = net
        self.bucketer = bucketer
        if bucketer is not None and hasattr(bucketer, "sc"):
            bucketer.sc = net.sc         # DG_CHECK_STREAMS: comm fork / join checked too
        fire_after = {}
        if bucketer is not None:
            for bi, (_, _, first_layer) in enumerate(bucketer.buckets):
                fire_after.setdefault(first_layer, []).append(bi)
        segs: List[Tuple[List[Callable[[], None]], List[int]]] = []
        cur: List[Callable[[], None]] = []
        in_graph = (bucketer is not None and getattr(bucketer, "in_graph", False)
                    and use_graphs)

        def emit(fn):
            cur.append(fn)

        emit(lambda: net._run(net._pre_train, stream_handle()))
        emit(lambda: net._run(net._fwd_train, stream_handle()))
        emit(lambda: net._run([net._head_train], stream_handle()))
        emit(net.head_reduce)
        emit(lambda: net._run(net._bwd_pre, stream_handle()))
        if net.L - 1 in fire_after:
            emit(net.join_side)               # the head's gradients final (deferred reduce)
            segs.append((cur, fire_after[net.L - 1]))
            cur = []
        for i in range(net.L - 2, -1, -1):
            emit(lambda i=i: net.backward_layer(i))
            if i in fire_after:
                # bucket grads final on the main stream: backward_layer already makes the
                # main stream wait for a layer's (group's) side-stream bias partials (and the
                # deferred head reduce before them); only layer 0's chain may still run on the
                # side stream, so only layer 0's bucket joins it — the others' all-reduces
                # overlap that chain (in-graph collectives only: a separately captured
                # segment must join every stream it forked)
                if i == 0 or net._l0_side_at is None or not in_graph:
                    emit(net.join_side)
                segs.append((cur, fire_after[i]))
                cur = []
        if cur:
            emit(net.join_side)
            segs.append((cur, []))
        self.segments = segs
        self.use_graphs = use_graphs
        self.in_graph_comm = bucketer is not None and getattr(bucketer, "in_graph", False)
        if not use_graphs:
            self.mode = "eager"
        elif bucketer is None:
            self.mode = "graph"
        else:
            self.mode = "dp-graph" if self.in_graph_comm else "dp-segments"
        self.graphs = []
        self.opt_graph = None
        self.full_graph = None
        self.fb_graph = None
        # one graph set per input buffer (HipGoNet.enable_prefetch): the replay picks the
        # set of the buffer the last set_batch filled
        self._gsets = {}
        if use_graphs:
            cur = net.cur_in
            for k in range(len(net._inbufs)):
                net.select_inputs(k)
                self._capture(warmup)
                self._gsets[k] = (self.graphs, self.fb_graph, self.full_graph)
                self.graphs = []
            net.select_inputs(cur)
            self.graphs, self.fb_graph, self.full_graph = self._gsets[cur]

    def _pick(self):
        if len(self._gsets) > 1:
            self.graphs, self.fb_graph, self.full_graph = self._gsets[self.net.cur_in]

    @staticmethod
    def _call_all(fns):
        for f in fns:
            f()

    def _fb_in_stream(self):
        """forward + backward with the in-graph (stream-ordered) collectives."""
        for fns, fire in self.segments:
            self._call_all(fns)
            for b in fire:
                self.bucketer.enqueue(b)
        self.bucketer.join()

    def _capture(self, warmup: int):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        net = self.net
        self.seg_launches = [0] * len(self.segments)
        with torch.cuda.stream(s):
            for _ in range(max(1, warmup)):
                if self.in_graph_comm:
                    self._fb_in_stream()       # also connects the communicator eagerly
                else:
                    for si, (fns, _) in enumerate(self.segments):
                        n0 = net.launches
                        self._call_all(fns)
                        self.seg_launches[si] = net.launches - n0
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        if self.mode == "dp-graph":
            # thread-local capture: RCCL's own threads may call HIP while we capture
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._fb_in_stream()
            self.fb_graph = g
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._fb_in_stream()
                self.net.optimizer_step()
            self.full_graph = g
        else:
            for si, (fns, _) in enumerate(self.segments):
                # a segment whose launches were all grouped away (e.g. the layers of a
                # grouped weight-gradient launch issued by the group's top layer) is not
                # captured: an empty capture is what a wrong-stream capture looks like, so
                # none may be produced on purpose (tests treat that warning as an error)
                if self.seg_launches[si] == 0:
                    self.graphs.append(None)
                    continue
                g = torch.cuda.CUDAGraph()
                n0 = net.launches
                with torch.cuda.graph(g):
                    self._call_all(fns)
                assert net.launches > n0, "segment capture recorded no launch"
                self.graphs.append(g)
            if self.mode == "graph":
                # the whole step: its gradient pass 2 deferred into the fused update
                g = torch.cuda.CUDAGraph()
                net.set_defer(True)
                try:
                    with torch.cuda.graph(g):
                        for fns, _ in self.segments:
                            self._call_all(fns)
                        self.net.optimizer_step()
                finally:
                    net.set_defer(False)
                self.full_graph = g
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.net.optimizer_step()
        self.opt_graph = g
        torch.cuda.synchronize()

    def forward_backward(self):
        """Gradients (all-reduced across ranks when DP) of the batch in the input buffers."""
        self._pick()
        if self.fb_graph is not None:
            with trace.range("fwd_bwd_graph"):
                self.fb_graph.replay()
            return
        if self.in_graph_comm:          # eager with the native communicator
            self._fb_in_stream()
            if not self.use_graphs:
                self.net.check_streams()
            return
        for si, (fns, fire) in enumerate(self.segments):
            with trace.range(f"segment{si}"):
                if self.use_graphs:
                    if self.graphs[si] is not None:
                        self.graphs[si].replay()
                else:
                    self._call_all(fns)
            if self.bucketer is not None:
                with trace.range("allreduce_issue"):
                    for b in fire:
                        self.bucketer.fire(b)
        if self.bucketer is not None:
            with trace.range("allreduce_wait"):
                self.bucketer.wait()

    def optimizer(self):
        with trace.range("optimizer"):
            if self.use_graphs:
                self.opt_graph.replay()
            else:
                self.net.optimizer_step()

    def __call__(self):
        self._pick()
        if self.full_graph is not None:
            with trace.range("step_graph"):
                self.full_graph.replay()
            return
        if not self.use_graphs and self.bucketer is None:
            # eager whole step: the same launches as the whole-step graph
            self.net.set_defer(True)
            try:
                for fns, _ in self.segments:
                    self._call_all(fns)
                self.net.optimizer_step()
            finally:
                self.net.set_defer(False)
            self.net.check_streams()
            return
        self.forward_backward()
        self.optimizer()
        if not self.use_graphs:
            self.net.check_streams()
