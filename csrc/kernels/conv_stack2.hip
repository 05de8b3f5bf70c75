// Fused run of hidden 3x3 layers (C -> C, C = 128, pad 1), board-resident in LDS, with the
// weights streamed straight into VGPRs: no LDS weight ring, no barrier inside a layer.
//
// One workgroup (8 waves) owns one board for ALL layers of the run (forward stack, or the
// backward-data chain in EPI_DGRAD mode):
//   * the board's zero-bordered 21x21x128 frame lives in LDS (two 64-channel images of 448
//     XOR-swizzled 128-B rows, 112 KB; the head_body.h layout);
//   * wave (wm, wn) computes output channels wm*64 .. +64 x pixels wn*96 .. +96 as 4 x 6
//     v_mfma_f32_16x16x32_bf16 fragments; a layer is 18 K-steps (2 chunks of 64 input
//     channels x 9 taps) of 2 MFMA k-halves;
//   * the A operand (weights) of a K-step comes from global memory (L2 / L1: every board
//     reads the same 288 KB per layer) in FRAGMENT ORDER (weight_refresh writes it:
//     [step 18][wm 2][kk 2][i 4][lane 64][8 bf16]), so one global_load_dwordx4 per
//     fragment moves one contiguous KB per wave, straight into the registers the MFMA
//     reads.  Each k-half's fragments for the next K-step are loaded as soon as that
//     k-half's MFMAs have issued (half a step ahead, across layer boundaries); the
//     compiler's own vmcnt waits cover them.
//
// Why: the previous design (conv_stack.hip) staged each [128 co][64 k] weight tile through
// an LDS ring by LDS-DMA, which needs one workgroup barrier per K-step (the tile is written
// by all waves and read by all).  With two waves per SIMD both hit that barrier together,
// and the phase timer put the idle barrier + DMA-issue + wait at ~900 of ~2700 cycles per
// K-step (profiles/r1_kbench_stack_final.json).  Here the image is the only shared LDS
// state, and it is read-only for the whole layer, so waves only meet at the layer's
// epilogue (2 barriers per layer instead of 18).  10 layers x 256 boards on one MI355X:
// forward 250 -> 233 us, dgrad 242 -> 224 us, bit-identical outputs
// (profiles/r2_kbench_stack2.json).
//
// The epilogue writes the layer's bf16 output straight back INTO the LDS image (the next
// layer's input):
//   EPI_FWD   : + (bias + pos-bias) table, ReLU          (forward; writes ReLU bitmask)
//   EPI_DGRAD : * ReLU bitmask of the layer below       (dZ_{i-1} = mask * W_i^T dZ_i)
// and the global store of that output (activation / gradient frame for the wgrads, plus
// the forward's bitmask) is spread over the next layer's first 12 K-steps, under its MFMAs.
//
// LDS: 12 KB head scratch + 112 KB image = 124 KB: one 8-wave workgroup per CU.
//
// Reference ops: nn.SpatialZeroPadding + SpatialConvolutionMM + Add + ReLU per layer
// (experiments.lua:137-147) and their backward through the stack (train.lua:10).
#include <stdio.h>
#include <stdlib.h>

#include "dg_common.h"
#include "dg_features.h"
#include "head_body.h"

using namespace dg;

namespace {

constexpr int EPI_FWD = 1;
constexpr int EPI_DGRAD = 2;
constexpr int C = 128;
constexpr int F = 21;                     // 19 + 2 * pad(1)
constexpr int FF = F * F;                 // 441
constexpr int HROWS = 448;                // halo rows padded to whole 8-wave DMA rounds
constexpr int H_BYTES = HROWS * 128;      // one 64-channel image
constexpr int T = 9;
constexpr int NSTEP = 2 * T;              // chunks x taps
constexpr int MAXL = 24;
constexpr int MF = 4;                     // 64 co per wave (4 fragments of 16)
constexpr int NF = 6;                     // 96 px per wave (6 fragments of 16)
constexpr int NW = 8;
constexpr int NT = NW * 64;
constexpr int SCRATCH = 12 * 1024;        // head_body scratch (fused head)
constexpr int STEP_BYTES = 2 * 2 * MF * 64 * 16;   // one K-step of one layer: 16 KB
constexpr int WM_BYTES = STEP_BYTES / 2;           // one co-half: 8 KB
constexpr int CO_STEPS = (NPTS * 8 + NT - 1) / NT;  // copy-out steps per 64-channel image (6)

static_assert(dghead::scratch_bytes(C) <= SCRATCH, "head scratch");

struct StackLayer {
  const char* A;        // fragment-ordered weights (18 x 16 KB; dgrad: flipped, transposed)
  const bf16_t* pbias;  // EPI_FWD: bf16 bias + pos-bias in fragment order ([24][2][4][64] x 4)
  char* Y;              // output frame [B][21][21][128] bf16
  uint8_t* mask;        // [B][361][16] ReLU bits: EPI_FWD writes (optional), EPI_DGRAD reads
};
struct StackArgs {
  const char* X0;       // input frame [B][21][21][128] bf16 of the first layer (l1: the
                        // network input frame [B][23][23][40])
  int nl;
  int fuse_head;        // EPI_FWD: run the policy head on the final image
  int l1;               // EPI_FWD: row 0 is the network's first layer (5x5, 40 -> 128 channels)
  // l1 with the feature expansion fused (in_planes non-null): the prologue builds the staged
  // input planes from the packed uint8 batch itself and writes the expanded frame to X0 (the
  // first layer's weight gradient reads it) instead of gathering X0 written by a launch before
  const uint8_t* in_planes;   // [B][9][361]
  const uint8_t* in_player;   // [B]
  const uint8_t* in_rank;     // [B]
  StackLayer L[MAXL];
  dghead::HeadMArgs head;  // (head_body.h; X unused: the image is resident)
  // STAG: the staggered two-group schedule (see the K loop): the co-half-0 group's MFMA
  // priority (0: none, 1 | 2: s_setprio) and an initial delay of the co-half-1 group
  // (s_sleep 127 rounds)
  int stag_prio;
  int stag_delay;
};

DG_DEV int fsig(int f) { return ((f % F) + 3 * (f / F)) & 7; }

// The network's first layer fused in front of the forward stack (l1 mode): 5x5 over the
// zero-bordered 23x23 frame of the 37 input planes padded to 40 channels (80 B per pixel),
// staged linearly into the (still unused) image area.  K runs over the 125 8-channel
// (tap, chunk) groups padded to 128 (K = 1024 = 16 K-steps; the padding chunks have zero
// weights): a lane's 8 K values are one chunk, so a 32-wide k-half mixes taps — conv_l1.hip's
// scheme, with the weights fragment-ordered like the hidden layers' ([16][2][2][4][64] x 8,
// k linear).  Layer 0's output is written into the image by the usual epilogue (the frame is
// dead by then: every read precedes the epilogue's first barrier).
// Staged layout: 16-B cells (8 channels), chunk-major planes, frame rows padded to 35 cells:
// cell(c8, y, x) = c8 * 816 + 35 y + x.  A ds_read_b128 phase takes 16 lanes = 16
// consecutive board pixels of one chunk (or of two consecutive chunks); with a row pitch of
// 35 = 3 (mod 16) the step from the end of one board row to the start of the next is also
// +1 cell (mod 16) and a plane stride of 816 = 0 (mod 16) keeps the second chunk on the other
// 8 residues, so its 16 cells sit on 16 distinct 4-bank groups (modelled 0.28 extra LDS
// cycles per phase vs 1.47 for the linear 80-B-per-pixel frame: 5.9M -> ~1M conflict cycles
// per launch).  The DMA gathers each cell from the linear [23][23][40] frame.
constexpr int L1F = 23;
constexpr int L1XB = 80;                        // bytes per pixel (40 bf16) in HBM
constexpr int L1_BYTES = L1F * L1F * L1XB;       // 42320
constexpr int L1RP = 35;                         // LDS cells per frame row
constexpr int L1PS = 816;                        // LDS cells per 8-channel plane
constexpr int L1_CELLS = 5 * L1PS;               // 4080 (65,280 B)
constexpr int L1_STEPS = 16;
constexpr int L1_CHUNKS = 125;

// s_waitcnt lgkmcnt(0) (LDS writes of this wave done), vmcnt/expcnt untouched, then barrier:
// unlike __syncthreads() this does not drain the weight loads already in flight
DG_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
// two fp32 -> packed bf16 (RNE, v_cvt_pk_bf16_f32)
DG_DEV uint32_t bf16x2_bits(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}
// ... then ReLU as a packed int16 max with 0 (v_pk_max_i16)
DG_DEV uint32_t relu_bf16x2(f32x2 v) {
  const s16x2 h = __builtin_bit_cast(s16x2, __builtin_convertvector(v, bf16x2v));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, s16x2{0, 0}));
}
// packed bf16 pair -> two fp32
DG_DEV f32x2 bf16x2_f32(uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}
// bits 0 / 1 of nib -> 0xffff / 0xffff0000 halves (v_bfe_i32 x 2 + v_perm_b32)
DG_DEV uint32_t pair_mask(uint32_t nib) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)nib, 0, 1);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)nib, 1, 1);
  return __builtin_amdgcn_perm(hi, lo, 0x07060100u);
}

// (the staggered schedule's LDS counters: grp_signal / grp_wait, dg_common.h)

// MODE: 0 in production; timing ablations for tools/kbench_stack.py (wrong results):
// 2 = no A loads in the K loop, 4 = no copy-out, 8 = no B reads in the K loop, 16 = no
// epilogue (nothing written back into the image)
template <int EPI, int MODE, bool STAG = false>
__global__ void __launch_bounds__(NT) conv_stack2_kernel(StackArgs a) {
  // epilogue schedule (see the K loop)
  constexpr bool TWO_GROUP = EPI == EPI_DGRAD && !STAG;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int b = blockIdx.x;
  char* sH = smem + SCRATCH;  // image c at sH + c * H_BYTES
  // STAG counters R0 R1 (waves past their reads of image 0 / 1 in this layer, 8 per layer)
  // and W0 W1 (waves of co-half 0 / 1 that wrote their image, 4 per layer), in the head
  // scratch (unused until the head, after the final barrier)
  LDS_AS unsigned* cnt = (LDS_AS unsigned*)(smem + SCRATCH - 16);
  if constexpr (STAG) {
    if (tid < 4) cnt[tid] = 0u;
    const int wmu = __builtin_amdgcn_readfirstlane(wm);
    if (wmu == 0 && a.stag_prio == 1) __builtin_amdgcn_s_setprio(1);
    if (wmu == 0 && a.stag_prio == 2) __builtin_amdgcn_s_setprio(2);
    if (wmu == 1)
      for (int d = 0; d < a.stag_delay; ++d) __builtin_amdgcn_s_sleep(127);
  }

  // ---- prologue: the first layer's input frame (both 64-channel images) by LDS-DMA ----
  if (EPI == EPI_FWD && a.l1 && a.in_planes) {
    // fused expansion: every frame pixel's 5 cells (8 channels each) computed here; border
    // pixels are zero; interior pixels also go to the expanded frame X0 (its border is zero
    // from allocation and never written).  The same planes as expand_features (dg_features.h).
    const uint8_t* plb = a.in_planes + (size_t)b * 9 * NPTS;
    const int pi = a.in_player[b], rk = a.in_rank[b];
    char* Xw = (char*)a.X0 + (size_t)b * L1_BYTES;
    for (int f = tid; f < L1F * L1F; f += NT) {
      const int y = f / L1F, x = f - (f / L1F) * L1F;
      uint4 cell[5];
#pragma unroll
      for (int c8 = 0; c8 < 5; ++c8) cell[c8] = uint4{0u, 0u, 0u, 0u};
      if (y >= 2 && y < 21 && x >= 2 && x < 21) {
        float v[40];
        expand_point(plb + (y - 2) * BOARD + (x - 2), pi, rk, v);
#pragma unroll
        for (int c8 = 0; c8 < 5; ++c8) {
          cell[c8] = uint4{pack_bf16x2(v[8 * c8], v[8 * c8 + 1]), pack_bf16x2(v[8 * c8 + 2], v[8 * c8 + 3]),
                           pack_bf16x2(v[8 * c8 + 4], v[8 * c8 + 5]), pack_bf16x2(v[8 * c8 + 6], v[8 * c8 + 7])};
          *(uint4*)(Xw + f * L1XB + c8 * 16) = cell[c8];
        }
      }
#pragma unroll
      for (int c8 = 0; c8 < 5; ++c8)
        *(uint4*)(sH + (c8 * L1PS + y * L1RP + x) * 16) = cell[c8];
    }
  } else if (EPI == EPI_FWD && a.l1) {   // (l1: a linear copy of the 23x23x40 frame, whole 1-KB
                                         // blocks; the last block's tail re-reads the last 16 B)
    const char* Xb = a.X0 + (size_t)b * L1_BYTES;
    for (int blk = wave; blk < (L1_CELLS + 63) / 64; blk += NW) {
      // cell -> (chunk, frame row, column); padding cells re-read pixel 0 (never used)
      const int cell = blk * 64 + lane;
      const int c8 = cell / L1PS, rem = cell - c8 * L1PS;
      const int y = rem / L1RP, x = rem - y * L1RP;
      const int off = (c8 < 5 && y < L1F && x < L1F) ? (y * L1F + x) * L1XB + c8 * 16 : 0;
      glds16(Xb + off, (LDS_AS void*)(sH + blk * 1024));
    }
  } else {
    const char* Xb = a.X0 + (size_t)b * FF * C * 2;
    for (int j = wave; j < 2 * (HROWS / 8); j += NW) {
      const int c = j / (HROWS / 8), jj = j - c * (HROWS / 8);
      int r = jj * 8 + (lane >> 3);
      r = r < FF ? r : FF - 1;
      const int rl = jj * 8 + (lane >> 3);  // LDS row this lane fills (slot lane & 7)
      const int gs_ = (lane & 7) ^ fsig(rl);
      glds16(Xb + ((size_t)r * C + c * 64 + gs_ * 8) * 2,
             (LDS_AS void*)(sH + c * H_BYTES + jj * 1024));
    }
  }

  const int lr = lane & 15;
  const int lq = lane >> 4;
  // this lane's B-fragment rows: pixel p = wn*96 + j*16 + lr (clamped), frame row fp,
  // swizzle signature fs (before & 7)
  // packed per fragment: row byte offset fp*128 (16 bits) | (fs & 7) << 16 (one VGPR each)
  uint32_t pk[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = wn * NF * 16 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    pk[j] = (uint32_t)(((h + 1) * F + (w + 1)) * 128) | ((uint32_t)(((w + 1) + 3 * (h + 1)) & 7) << 16);
  }
  const uint32_t a_lane = (uint32_t)(wm * WM_BYTES + lane * 16);

  // A fragments of one k-half of a K-step (A = the step's 16 KB): 4 x 1 KB pieces, one
  // global_load_dwordx4 each.  Plain loads (the compiler counts them and waits for them);
  // the sched_barriers in the step pin where they issue — left alone the scheduler sinks
  // them next to their consumer, a half step later.
  auto load_A = [&](const char* A, int kk, bf16x8 (&r)[MF]) {
    const char* p = A + a_lane + kk * MF * 1024;
#pragma unroll
    for (int i = 0; i < MF; ++i) r[i] = *(const bf16x8*)(p + i * 1024);
  };
  // B fragments (pixels x 32 channels of k-half kk) of K-step s from the resident image:
  // slot (kk*4 + lq) ^ sig, and kk = 1 is kk = 0 with bit 2 of the slot flipped
  auto read_B = [&](int s, int kk, bf16x8 (&bfr)[NF]) {
    const int c = s / T, t = s % T;
    const LDS_AS char* sHc = (const LDS_AS char*)(sH + c * H_BYTES);
    const int toff = (t / 3 - 1) * F + (t % 3 - 1);
    const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int off = (int)(pk[j] & 0xFFFFu) + toff * 128 +
                      ((lq ^ (((int)(pk[j] >> 16) + tsig) & 7)) * 16);
      bfr[j] = lds_read_b128(sHc + (off ^ (kk * 64)));
    }
  };
  // l1 mode, layer 0: B fragments of k-half kk of K-step s from the staged input frame
  auto read_B1 = [&](int s, int kk, bf16x8 (&bfr)[NF]) {
    int kc = s * 8 + kk * 4 + lq;          // this lane group's chunk (tap, c8)
    if (kc >= L1_CHUNKS) kc = 0;          // padding chunks: zero weights
    const int t = kc / 5, c8 = kc - (kc / 5) * 5;
    const int koff = (c8 * L1PS + (t / 5 - 2) * L1RP + (t % 5 - 2)) * 16;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      int p = wn * NF * 16 + j * 16 + lr;
      if (p >= NPTS) p = 0;
      const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
      bfr[j] = lds_read_b128((const LDS_AS char*)(sH + ((h + 2) * L1RP + (w + 2)) * 16 + koff));
    }
  };
  auto mma = [&](const bf16x8 (&af)[MF], const bf16x8 (&bfr)[NF], f32x4 (&acc)[MF][NF]) {
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  };

  // Copy-out of the previous layer's output (resident in the image) to HBM, one 16-B piece
  // (8 channels of one pixel) per thread and K-step: image 0 (channels 0..63) in K-steps
  // 0..5, image 1 in K-steps 9..14 — each image only while the K loop is reading it, i.e.
  // after the barrier that completes it and before the epilogue that overwrites it.  The
  // piece of a step is read from LDS after the step's first k-half and stored at its end.
  // Step s: half hf = s / 9, j = s % 9; thread tid handles channel piece q = tid & 7 of
  // image hf at pixel p = tid / 8 + 64 j (128 contiguous bytes per pixel and image).
  auto co_read = [&](int s_) -> uint4 {
    const int hf = s_ >= T, j = s_ - hf * T;
    const int p = min((tid >> 3) + 64 * j, NPTS - 1);
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    return *(const uint4*)(sH + hf * H_BYTES + f * 128 + (((tid & 7) ^ fsig(f)) * 16));
  };
  auto co_store = [&](int s_, const uint4& v, const StackLayer& Lo) {
    // lanes past the board re-store pixel 360 (same value): every wave issues the stores
    const int hf = s_ >= T, j = s_ - hf * T;
    const int p = min((tid >> 3) + 64 * j, NPTS - 1);
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    const int co_q = hf * 8 + (tid & 7);
    *(uint4*)(Lo.Y + ((size_t)(b * FF + f) * C) * 2 + co_q * 16) = v;
    if (EPI == EPI_FWD && Lo.mask) {
      // bit per nonzero bf16 half (post-ReLU: every half is in [0, 0x7fff]): h + 0x7fff has
      // bit 15 set iff h != 0, with no carry out of the half; gather bits 15 / 31 of the
      // four words to channel order (bit 2k: word k low half, 2k + 1: its high half)
      const uint32_t m = (((v.x + 0x7fff7fffu) >> 15) & 0x10001u) |
                         (((v.y + 0x7fff7fffu) >> 13) & 0x40004u) |
                         (((v.z + 0x7fff7fffu) >> 11) & 0x100010u) |
                         (((v.w + 0x7fff7fffu) >> 9) & 0x400040u);
      Lo.mask[((size_t)b * NPTS + p) * 16 + co_q] = (uint8_t)(m | (m >> 15));
    }
  };

  __syncthreads();  // image landed (the compiler waits for the LDS-DMA before the barrier)

  bf16x8 Ak[2][MF];
  load_A(a.L[0].A, 0, Ak[0]);
  load_A(a.L[0].A, 1, Ak[1]);  // (first waits: nothing newer in flight)

  for (int l = 0; l < a.nl; ++l) {
    const StackLayer L = a.L[l];
    const char* A_next = l + 1 < a.nl ? a.L[l + 1].A : L.A;
    const StackLayer Lprev = a.L[l > 0 ? l - 1 : 0];
    const bool co_on = l > 0;
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 co_v;

    // One K-step.  A k-half's fragments (the next step's) are re-loaded right after that
    // k-half's MFMAs are issued: one register set, half a step of prefetch distance.  Plain
    // loads the compiler counts; the sched_barriers pin where they issue (left alone, the
    // scheduler sinks them next to their consumer).  The copy-out store goes last, after
    // the loads, so waiting for a load never waits for a store issued after it.
    auto kstep = [&](const int s, const bool co) {
      // (past the last step of the last layer: a harmless re-load of step 0)
      const char* An = s + 1 < NSTEP ? L.A + (s + 1) * STEP_BYTES : A_next;
      bf16x8 bfr[NF];
      if constexpr (!(MODE & 8)) read_B(s, 0, bfr);
      mma(Ak[0], bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(MODE & 2)) load_A(An, 0, Ak[0]);
      if (co) co_v = co_read(s);
      if constexpr (!(MODE & 8)) read_B(s, 1, bfr);
      __builtin_amdgcn_sched_barrier(0);
      mma(Ak[1], bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!(MODE & 2)) load_A(An, 1, Ak[1]);
      if (co) co_store(s, co_v, Lprev);
      __builtin_amdgcn_sched_barrier(0);
    };
    // Rolled loops with a per-step copy-out branch.  The compiler's wait at their head is
    // then vmcnt(0) (the k-half-1 loads of the step before and its copy-out store drain
    // there); measured faster than every variant with exact waits: two branch-free loops
    // (copy-out steps / the rest: fwd 229 -> 234 us, dgrad 216 -> 224 us) and unrolled by 2
    // or 3 (267 / 279 us; profiles/r2_kbench_stack2.json).
    //
    // Two-group schedule of the backward-data chain (TWO_GROUP; the waves of co-half wm write
    // image wm in the epilogue):
    //   steps 0..8 (image 0) | barrier A | steps 9..17 (image 1) | wm 0: write image 0 |
    //   barrier B | wm 1: write image 1 (beside wm 0's next steps 0..8, which read image 0)
    // Barrier A: every wave is past its image-0 reads and image 1 holds the layer input
    // (wm 1 wrote it before arriving); barrier B: image 0 holds the output and every wave is
    // past its image-1 reads.  Same 2 barriers per layer as writing both images between two
    // barriers, but half of the epilogue runs beside the other half's MFMAs (dgrad stack
    // -0.9..-3% in the kernel bench; the forward keeps one write phase between two barriers).
    // dgrad: this wave's ReLU-bit words of the layer below (the epilogue's gates), loaded two
    // K-steps before the end of the loop, so co-half 0's epilogue (first, right after the
    // loop) does not wait for them (dgrad stack -1.7%, step +0.3%)
    uint2 em[NF];
    auto load_em = [&]() {
      int z1 = 0;
      asm volatile("" : "+v"(z1));
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
        em[j] = *(const uint2*)(L.mask + ((size_t)b * NPTS + p) * 16 + wm * 8 + z1);
      }
    };
    int s = 0;
    // STAG: layer index among the staggered layers (the fused first layer keeps barriers)
    const unsigned kx = (unsigned)(l - (EPI == EPI_FWD && a.l1 ? 1 : 0));
    if (EPI == EPI_FWD && l == 0 && a.l1) {
      // the fused first layer: 16 K-steps over the staged input frame (nothing to copy out)
#pragma unroll 1
      for (; s < L1_STEPS; ++s) {
        const char* An = s + 1 < L1_STEPS ? L.A + (s + 1) * STEP_BYTES : A_next;
        bf16x8 bfr[NF];
        read_B1(s, 0, bfr);
        mma(Ak[0], bfr, acc);
        __builtin_amdgcn_sched_barrier(0);
        load_A(An, 0, Ak[0]);
        read_B1(s, 1, bfr);
        __builtin_amdgcn_sched_barrier(0);
        mma(Ak[1], bfr, acc);
        __builtin_amdgcn_sched_barrier(0);
        load_A(An, 1, Ak[1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      auto chunk = [&](const int h2) {
        if (h2 == 1 && TWO_GROUP) lds_barrier();  // A
        // STAG: image h2 holds the previous layer's output once its co-half wrote it
        if constexpr (STAG) grp_wait(cnt + 2 + h2, 4u * kx);
        if (!(MODE & 4) && co_on) {
#pragma unroll 1
          for (; s < h2 * T + CO_STEPS; ++s) {
            int tt = s;
            asm volatile("" : "+s"(tt));
            kstep(tt, true);
          }
        }
#pragma unroll 1
        for (; s < (h2 + 1) * T; ++s) {
          if (EPI == EPI_DGRAD && s == NSTEP - 2) load_em();
          kstep(s, false);
        }
        if constexpr (STAG) grp_signal(cnt + h2);   // past this layer's reads of image h2
      };
      if constexpr (STAG) {
        // (two inlined chunks: a rolled chunk loop around the counter asm costs ~100 spills)
        chunk(0);
        chunk(1);
      } else {
#pragma unroll 1
        for (int h2 = 0; h2 < 2; ++h2) chunk(h2);
      }
    }

    // ---- epilogue: write the layer's output back into the LDS image ----
    // every global load of the epilogue is issued before the first use
    // (an opaque zero in the addresses: otherwise the compiler hoists all per-fragment
    // table addresses out of the layer loop and spills them)
    int z0 = 0;
    asm volatile("" : "+v"(z0));
    uint2 eb[NF][EPI == EPI_FWD ? MF : 1];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
      if constexpr (EPI == EPI_FWD) {
        const uint2* pf = (const uint2*)L.pbias + ((wn * NF + j) * 2 + wm) * 4 * 64 + lane + z0;
#pragma unroll
        for (int i = 0; i < MF; ++i) eb[j][i] = pf[i * 64];
      }
    }
    auto write_out = [&]() {
      if constexpr ((MODE & 16) != 0) {   // (the accumulators stay live: no MFMA is dropped)
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j) asm volatile("" ::"v"(acc[i][j]));
        return;
      }
#pragma unroll
      for (int j = 0; j < NF; ++j) {
        const int p = wn * NF * 16 + j * 16 + lr;
        // the LDS offsets below derive from an opaque copy of pk[j]: left visible, the
        // compiler hoists all 24 (fragment, slot) offsets out of the layer loop, spills them
        // (forward: 256 VGPRs) and reloads each with a full vmcnt(0) wait in every epilogue
        uint32_t pkj = pk[j];
        asm volatile("" : "+v"(pkj));
        const int f = (int)(pkj & 0xFFFFu) >> 7;
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int cl = i * 16 + lq * 4;  // channel within the wave's 64-channel image
          const f32x4 v = acc[i][j];
          uint2 o;
          if constexpr (EPI == EPI_FWD) {
            // packed fp32 bias add, bf16 pack, ReLU on the packed bf16 (max as int16: the
            // same as relu before the rounding, -0 included)
            o.x = relu_bf16x2(f32x2{v[0], v[1]} + bf16x2_f32(eb[j][i].x));
            o.y = relu_bf16x2(f32x2{v[2], v[3]} + bf16x2_f32(eb[j][i].y));
          } else {
            // the 4 ReLU bits of these channels gate the bf16 pairs
            const uint32_t word = (i < 2) ? em[j].x : em[j].y;
            const uint32_t nib = word >> ((cl & 31) >> 3 << 3) >> (cl & 4);
            o.x = bf16x2_bits(f32x2{v[0], v[1]}) & pair_mask(nib);
            o.y = bf16x2_bits(f32x2{v[2], v[3]}) & pair_mask(nib >> 2);
          }
          const int slot = (cl >> 3) ^ (int)(pkj >> 16);
          if (p < NPTS) *(uint2*)(sH + z0 + wm * H_BYTES + f * 128 + slot * 16 + (cl & 4) * 2) = o;
        }
      }
    };
    // Staggered two-group schedule (STAG): no workgroup barrier inside the run.  Co-half g's
    // waves write image g once all 8 waves are past their reads of it in this layer (R_g),
    // then count themselves in W_g; a wave reads image c of a layer once co-half c has
    // written it (W_c).  Both groups run chunk 0 (image 0) first, so co-half 0 may run up to
    // half a layer ahead of co-half 1: its epilogue runs beside co-half 1's last K-steps and
    // co-half 1's beside co-half 0's next image-0 K-steps — every wave's epilogue overlaps
    // the other group's MFMAs (the barrier schedules below idle the MFMA pipes through it).
    if constexpr (STAG) {
      if (!(EPI == EPI_FWD && l == 0 && a.l1)) {
        grp_wait(cnt + wm, 8u * (kx + 1));
        write_out();
        grp_signal(cnt + 2 + wm);
        continue;
      }
    }
    if constexpr (TWO_GROUP) {
      if (wm == 0) write_out();  // image 0: dead since barrier A
      lds_barrier();             // B
      if (wm == 1) write_out();  // image 1 (the next layer's barrier A publishes it)
      continue;
    }
    // forward: both groups write between two barriers (measured +0.9% over the two-group
    // schedule in the step; the l1 layer's input frame fills image 0 for all 16 steps anyway)
    lds_barrier();
    if (EPI == EPI_FWD && l == 0 && a.l1) {
      // the image area held the first layer's input frame: zero the 21x21 frame's border
      // rows / columns (the next layer's taps read them) and the padding rows 441..447
      for (int u = tid; u < 87 * 8 * 2; u += NT) {
        const int img = u / (87 * 8), k = (u >> 3) % 87, q = u & 7;
        const int row = k < 21 ? k : k < 42 ? 420 + (k - 21) : k < 61 ? (k - 41) * 21
                        : k < 80 ? (k - 60) * 21 + 20 : 441 + (k - 80);
        *(uint4*)(sH + img * H_BYTES + row * 128 + q * 16) = uint4{0u, 0u, 0u, 0u};
      }
    }
    write_out();
    lds_barrier();  // the next layer's input is complete
  }
  lds_barrier();  // C: image 1 of the last layer's output (wm 1) is complete
  // last layer's output: exposed copy-out — not with the fused head (training): its only
  // readers are the head (here, on the resident image) and the evaluation forward, which runs
  // the head-less launch; the head's backward gates with the image itself, not the bitmask
  if (EPI != EPI_FWD || !a.fuse_head) {
    const StackLayer Ll = a.L[a.nl - 1];
    for (int s_ = 0; s_ < CO_STEPS; ++s_) co_store(s_, co_read(s_), Ll);
    for (int s_ = T; s_ < T + CO_STEPS; ++s_) co_store(s_, co_read(s_), Ll);
  }
  // the policy head on the board image that is already in LDS (no re-staging, no launch)
  if constexpr (EPI == EPI_FWD) {
    if (a.fuse_head) dghead::head_body<C>(a.head, b, sH, smem, [](int) {});
  }
}

template <int EPI, int MODE, bool STAG = false>
hipError_t launch_stack2(const StackArgs& a, int B, hipStream_t stream) {
  constexpr size_t lds = SCRATCH + 2 * (size_t)H_BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_stack2_kernel<EPI, MODE, STAG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL((conv_stack2_kernel<EPI, MODE, STAG>), dim3(B), dim3(NT), lds, stream,
                     a);
  return hipGetLastError();
}

int g_stack2_mode = 0;  // ablation MODE of the forward (0 = production)
// the staggered schedule: -1 = not yet read from DG_STACK2_STAG ("MODE[,PRIO[,DELAY]]"), else
// 0 off, 1 both stacks, 2 the backward-data stack only (default: 12x128 bf16 step 303.8-304.3k
// vs 302.1-302.6k with neither, 4 interleaved rounds on one box, profiles/r5_stack2_stag.txt;
// the forward measured slower, kbench 244 vs 228 us); its co-half-0 priority and co-half-1
// start delay
int g_stack2_stag = -1, g_stack2_prio = 1, g_stack2_delay = 0;
void stack2_sched_from_env() {
  if (g_stack2_stag >= 0) return;
  const char* e = getenv("DG_STACK2_STAG");
  g_stack2_stag = 2;
  if (e && *e) {
    int v = 0, p = g_stack2_prio, d = g_stack2_delay;
    const int n = sscanf(e, "%d,%d,%d", &v, &p, &d);
    g_stack2_stag = n >= 1 && v >= 0 && v <= 2 ? v : 2;
    if (n >= 2) g_stack2_prio = p;
    if (n >= 3) g_stack2_delay = d;
  }
}

hipError_t stack2_launch(int epi, const long long* table, int nl, const void* X0, int l1, int B,
                         const dghead::HeadMArgs* head, hipStream_t stream,
                         const uint8_t* in_planes = nullptr, const uint8_t* in_player = nullptr,
                         const uint8_t* in_rank = nullptr) {
  if (nl <= 0 || nl > MAXL || B <= 0) return hipErrorInvalidValue;
  if (epi != EPI_FWD && epi != EPI_DGRAD) return hipErrorInvalidValue;
  if (l1 && (epi != EPI_FWD || nl < 2)) return hipErrorInvalidValue;
  static_assert(L1_CELLS * 16 <= 2 * H_BYTES, "l1 frame in the image area");
  StackArgs a;
  a.l1 = l1 ? 1 : 0;
  if (in_planes && (!l1 || !in_player || !in_rank)) return hipErrorInvalidValue;
  a.in_planes = in_planes;
  a.in_player = in_player;
  a.in_rank = in_rank;
  a.fuse_head = 0;
  a.head = dghead::HeadMArgs{};
  stack2_sched_from_env();
  a.stag_prio = g_stack2_prio;
  a.stag_delay = g_stack2_delay;
  const bool stag = g_stack2_stag == 1 || (g_stack2_stag == 2 && epi == EPI_DGRAD);
  a.X0 = (const char*)X0;
  a.nl = nl;
  for (int i = 0; i < nl; ++i) {
    a.L[i].A = (const char*)table[4 * i];
    a.L[i].pbias = (const bf16_t*)table[4 * i + 1];
    a.L[i].Y = (char*)table[4 * i + 2];
    a.L[i].mask = (uint8_t*)table[4 * i + 3];
    if (!a.L[i].A || !a.L[i].Y) return hipErrorInvalidValue;
    if (epi == EPI_FWD && !a.L[i].pbias) return hipErrorInvalidValue;
    if (epi == EPI_DGRAD && !a.L[i].mask) return hipErrorInvalidValue;
  }
  if (head) {
    if (epi != EPI_FWD) return hipErrorInvalidValue;
    a.fuse_head = 1;
    a.head = *head;
  }
  if (epi == EPI_DGRAD) {
    if (stag) {
      if (g_stack2_mode == 16) return launch_stack2<EPI_DGRAD, 16, true>(a, B, stream);
      return launch_stack2<EPI_DGRAD, 0, true>(a, B, stream);
    }
    if (g_stack2_mode == 16) return launch_stack2<EPI_DGRAD, 16>(a, B, stream);
    return launch_stack2<EPI_DGRAD, 0>(a, B, stream);
  }
  if (stag) {
    if (g_stack2_mode == 16) return launch_stack2<EPI_FWD, 16, true>(a, B, stream);
    return launch_stack2<EPI_FWD, 0, true>(a, B, stream);
  }
  switch (g_stack2_mode) {  // forward: the MODE ablations too (kbench_stack.py)
    case 2: return launch_stack2<EPI_FWD, 2>(a, B, stream);
    case 6: return launch_stack2<EPI_FWD, 6>(a, B, stream);
    case 14: return launch_stack2<EPI_FWD, 14>(a, B, stream);
    case 4: return launch_stack2<EPI_FWD, 4>(a, B, stream);
    case 10: return launch_stack2<EPI_FWD, 10>(a, B, stream);
    case 16: return launch_stack2<EPI_FWD, 16>(a, B, stream);
    default: return launch_stack2<EPI_FWD, 0>(a, B, stream);
  }
}

}  // namespace

extern "C" {

void dg_conv_stack2_set_mode(int m) { g_stack2_mode = m; }

// the staggered two-group schedule (overrides DG_STACK2_STAG): on 0 / 1, co-half-0 MFMA
// priority 0..2, co-half-1 start delay (s_sleep 127 rounds)
void dg_conv_stack2_set_sched(int stag, int prio, int delay) {
  g_stack2_stag = stag >= 0 && stag <= 2 ? stag : 0;
  g_stack2_prio = prio;
  g_stack2_delay = delay;
}

// table: nl rows of {A (fragment-ordered weights), pbias_frag, Y, mask} (int64 pointers)
//   epi 1 (forward): pbias required, mask optional (written)
//   epi 2 (dgrad)  : mask required (read; ReLU bits of the layer below), pbias unused
// l1 (EPI_FWD only): row 0 is the network's first layer (5x5 over the [B][23][23][40] input
// frame X0; its A = the [128][1024] weights in fragment order, k linear)
hipError_t dg_conv_stack2(int epi, const long long* table, int nl, const void* X0, int l1, int B,
                          hipStream_t stream) {
  return stack2_launch(epi, table, nl, X0, l1, B, nullptr, stream);
}

// Forward stack + the 3x3 / 128-channel policy head fused after its last layer.
hipError_t dg_conv_stack2_fwd_head(const long long* table, int nl, const void* X0, int l1, int B,
                                   const float* w, const float* bias, const float* posb,
                                   const int* labels, float* loss, int* pred, void* dZ,
                                   float* gw_part, float* dzb, int head_relu, float grad_scale,
                                   hipStream_t stream) {
  const dghead::HeadMArgs h{nullptr, w, bias, posb, labels, loss, pred, nullptr, (char*)dZ,
                            gw_part, dzb, head_relu, grad_scale};
  return stack2_launch(EPI_FWD, table, nl, X0, l1, B, &h, stream);
}

// The same with the feature expansion fused into the first layer's prologue (l1 only): the
// packed batch's planes / player / rank in, the expanded frame X0 written out.
hipError_t dg_conv_stack2_fwd_head_x(const long long* table, int nl, void* X0, int B,
                                     const void* planes, const void* player, const void* rank,
                                     const float* w, const float* bias, const float* posb,
                                     const int* labels, float* loss, int* pred, void* dZ,
                                     float* gw_part, float* dzb, int head_relu, float grad_scale,
                                     hipStream_t stream) {
  const dghead::HeadMArgs h{nullptr, w, bias, posb, labels, loss, pred, nullptr, (char*)dZ,
                            gw_part, dzb, head_relu, grad_scale};
  return stack2_launch(EPI_FWD, table, nl, X0, 1, B, &h, stream, (const uint8_t*)planes,
                       (const uint8_t*)player, (const uint8_t*)rank);
}

}  // extern "C"
