// FP8 forward layer stack (BASELINE config 5, the MX-fp8 MFMA path): the conv_stack2 design
// (one workgroup owns one board for ALL hidden 3x3 C -> C layers, weights streamed
// straight into VGPRs in fragment order, no barrier inside a layer) with the resident board
// image in OCP e4m3 and the K loop on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4
// (2x the bf16 MFMA rate on gfx950):
//   * the fp8 image is 21 x 21 frame rows of 128 B (one byte per channel, 56 KB), 16-B slot
//     (c / 16) ^ ((x + 3y) & 7) — the bf16 stack's swizzle on the same 128-B row geometry;
//   * a layer is 9 K-steps (one tap, K = 128 channels) of one MFMA per 16 x 16 fragment:
//     half the K-steps of the bf16 stack for the same bytes moved per step.  A fragment
//     (16 co x 128 k, 32 B per lane: lane group g holds k = 32g .. 32g + 31,
//     tools/fp8_mfma_probe.hip) = two global_load_dwordx4 of the fragment-ordered e4m3
//     weights [tap 9][wm 2][i 4][half 2][lane 64][16 B] (weight_refresh writes them);
//     B fragment = two ds_read_b128 of the image row;
//   * epilogue: y = relu(s_x s_w acc + bias + pos-bias), its amax folded into amax[l] (one
//     atomic per workgroup: delayed scaling, fp8_update_scales turns it into next step's
//     s_y), and e4m3(y / s_y) written back into the image as the next layer's input;
//   * the bf16 activation frame and ReLU bitmask of every layer (for the bf16 backward) are
//     copied out of the image during the next layer's first 6 K-steps, dequantized
//     (x s_y): the backward sees exactly the activations the fp8 forward consumed;
//   * the LAST layer writes a bf16 image instead (the conv_stack2 two-64-channel-image
//     layout over the same 112 KB), so the fused policy head (head_body.h) runs on it as in
//     the bf16 stack;
//   * prologue: the bf16 input frame (conv_l1's output) is quantized into the image with
//     its scale; its amax is folded in as well.
// fp8 copy-out (optional y8 table, the MX-fp8 weight gradient's operands, conv_wgrad_win8.hip):
// the raw e4m3 / e5m2 image bytes — the quantized input (X8_0) and every non-last layer's
// quantized output (Y8) — are stored beside the bf16 frames, in frames of 448 rows per board
// (441 + 7 zero rows, never written).
// Scales are device scalars named per layer in the launch table (s_in, s_w, s_out, amax_out):
// HipGoNet points them into its fp8_scales / fp8_gscales arrays (delayed scaling).
// EPI_DGRAD runs the backward-data chain the same way: e5m2 gradient image (the wider range),
// e4m3 flipped/transposed weights (MX MFMA A e4m3 x B e5m2), ReLU-mask epilogue, dequantized
// bf16 dZ frames copied out for the weight gradients.
//
// C = 256 (config 5's d = 256): the e4m3 image is 441 rows of 256 B (113 KB, slot swizzle
// ((x + 3y) & 15)) — resident where a bf16 one (226 KB) cannot be.  The 256 output channels
// run as two passes of 128 (96 accumulator registers per lane each); pass 0's e4m3 output
// is parked in the LDS left over (around the image) until pass 1 has read the whole input,
// then both halves go into the image.  A K-step is one (tap, 128-channel chunk) pair: 18 per
// pass.  The last layer's bf16 output goes straight to HBM from the epilogue (no bf16
// image fits): the head runs as its own launch (head_mfma<256>).
//
// LDS: 12 KB head scratch + 112 KB image region = 124 KB (C = 128); 160 KB (C = 256):
// one 8-wave workgroup per CU.
//
// Reference ops: nn.SpatialConvolutionMM + nn.Add + nn.ReLU per hidden layer
// (experiments.lua:137-147).
#include <stdio.h>
#include <stdlib.h>

#include "dg_common.h"
#include "head_body.h"

using namespace dg;

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

namespace {

constexpr int F = 21;
constexpr int FF = F * F;                 // 441
constexpr int HROWS = 448;
constexpr int H_BYTES = HROWS * 128;      // one bf16 64-channel image (C = 128 last layer)
constexpr int T = 9;                      // taps
constexpr int MAXL = 24;
constexpr int MF = 4;                     // 64 co per wave
constexpr int NF = 6;                     // 96 px per wave
constexpr int NW = 8;
constexpr int NT = NW * 64;
constexpr int SCRATCH = 12 * 1024;
constexpr int STEP_BYTES = 2 * MF * 2 * 64 * 16;  // 16 KB per (tap, chunk) K-step
constexpr int WM_BYTES = STEP_BYTES / 2;
constexpr float FP8_MAX = 448.f;      // e4m3
constexpr float BF8_MAX = 57344.f;    // e5m2
constexpr int EPI_FWD = 1;
constexpr int EPI_DGRAD = 2;
constexpr int FP8P = 448;             // fp8 copy-out frames: rows per board
constexpr int IMG2 = 61440;           // C = 128 staggered schedule: second image's offset

static_assert(dghead::scratch_bytes(128) + 64 + 16 + 4 * 24 <= SCRATCH, "head scratch");

// per-channel-count geometry
template <int C>
struct Geo {
  static constexpr int NC = C / 128;              // 128-channel chunks = output passes
  static constexpr int ROWB = C;                  // image row bytes (e4m3)
  static constexpr int SLOTS = C / 16;            // 16-B slots per row
  static constexpr int SIGM = SLOTS - 1;          // swizzle mask
  static constexpr int STEPS = T * NC;            // K-steps per pass
  static constexpr int PIECES = NPTS * SLOTS;     // copy-out pieces
  static constexpr int CO_STEPS = (PIECES + NT - 1) / NT;   // 6 | 12
  static constexpr int IMG = FF * ROWB;           // image bytes
  static constexpr int PARK1 = SCRATCH / 128;     // C = 256: pass-0 pixels parked in [0, 12K)
  // (C = 128: the staggered schedule's second e4m3 image at IMG2, its dump rows and tap
  // over-reads up to row 487 inside the allocation; the last layer's bf16 image 2 x H_BYTES)
  static constexpr int LDS = C == 128 ? SCRATCH + IMG2 + 488 * 128 : 160 * 1024;
  static constexpr int AMAX_OFF = C == 128 ? SCRATCH - 64 : SCRATCH + IMG + (NPTS - PARK1) * 128;
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(C == 128 || AMAX_OFF + 64 <= LDS, "park area");
};

struct F8Layer {
  const char* A8;       // fragment-ordered e4m3 weights (9 x 16 KB x (C/128)^2); dgrad: the
                        // flipped, transposed operand
  const bf16_t* pbias;  // EPI_FWD: bf16 bias + pos-bias in the stack's fragment order
  char* Y;              // bf16 output frame [B][21][21][C] (activation / dZ of the layer below)
  uint8_t* mask;        // [B][361][C/8] ReLU bits: EPI_FWD writes, EPI_DGRAD reads (layer below)
  const float* s_in;    // scale of this layer's quantized input (device scalar)
  const float* s_w;     // scale of its e4m3 weights
  const float* s_out;   // scale its output is quantized with (the next layer's s_in)
  unsigned* amax_out;   // |output| max folded in here (float bits; delayed scaling)
  uint8_t* Y8;          // optional fp8 copy of the quantized output [B][448][C] (non-last)
};
struct F8Args {
  const char* X0;       // bf16 input frame of the first layer
  const float* s_x0;    // its quantization scale
  unsigned* amax_x0;    // its |x| max (folded in by the prologue)
  uint8_t* X8_0;        // optional fp8 copy of the quantized input [B][448][C]
  int nl;
  int fuse_head;        // C = 128, EPI_FWD only
  // EPI_DGRAD: stochastic rounding of the e5m2 gradient quantization (MODE bit 32), random
  // bits from a hash of (step counter, layer, element); null: round to nearest even
  const long long* sr_step;
  int stag_delay;       // STAG: co-half-1 start delay (s_sleep 127 rounds; 0 in production)
  int stag_on;          // (host) this launch runs the staggered schedule
  unsigned long long* dbg;   // MODE bit 256 (diagnostics): s_memtime stamps of boards 0..7,
                             // [board][wave][layer][8]
  F8Layer L[MAXL];
  dghead::HeadMArgs head;
};

// swizzle signature of frame row f (16-B slot s of the row lives at s ^ sig): a table over
// v = (x + 3y) & 7, which steps by 1 along raster order (also across a board-row wrap, and by
// tsig = dx + 3 dy for a tap).  A B-fragment read (ds_read_b128) serves lanes in 4 groups of
// 16 that mix two lane groups lq (slots 8c + 2lq + h): the sig must not disturb bit 1 of the
// slot there.  C = 256: v's bits spread to slot bits {0, 2, 3}; C = 128 (8 slots, two rows
// per 64 banks): a searched table.  Modelled bank conflicts of the 9-tap B reads (all
// fragments): 1728 / 1728 group-reads (C = 128) and 2256 / 3456 (C = 256) extra cycles with
// the round-2 sig (x + 3y) & mask, 72 and 144 with these.
template <int C>
DG_DEV int sig_of(int v) {
  constexpr uint32_t TAB = C == 128 ? 0x60147107u : 0xDC985410u;
  return (int)((TAB >> (4 * (v & 7))) & 15u);
}
DG_DEV int fv(int f) { return ((f % F) + 3 * (f / F)) & 7; }
template <int C>
DG_DEV int fsig(int f) { return sig_of<C>(fv(f)); }
DG_DEV int fsig8(int f) { return ((f % F) + 3 * (f / F)) & 7; }

DG_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0), vmcnt / expcnt untouched
  __builtin_amdgcn_s_barrier();
}

DG_DEV uint32_t pack_fp8x4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}

// workgroup max of non-negative v folded into *amax (one atomic per workgroup); s_tmp: 8
// floats of LDS; every thread calls it (contains a barrier)
DG_DEV void wg_amax(float v, unsigned* amax, float* s_tmp) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) s_tmp[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = s_tmp[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = fmaxf(m, s_tmp[w]);
    atomicMax(amax, __float_as_uint(m));
  }
}

// e4m3 (EPI_FWD: activations) or e5m2 (EPI_DGRAD: gradients, the wider range) packing
template <int EPI>
DG_DEV uint32_t pack8x4(float a, float b, float c, float d) {
  if constexpr (EPI == EPI_FWD) return pack_fp8x4(a, b, c, d);
  int v = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_bf8_f32(c, d, v, true);
  return (uint32_t)v;
}
// e5m2 packing with stochastic rounding: the 4 conversions take 4 rotations of one 32-bit
// hash (each conversion's rounding decision rests on different hash bits).  Unbiased: a
// value between two e5m2 neighbours rounds up with probability equal to its fractional
// position, so the dgrad chain and the weight-gradient sums over ~92k pixels keep the small
// consistent components that round-to-nearest erases (the memorisation stall of
// tools/fp8_memo.py: tests/test_train_gpu.py test_fp8_stress_vs_bf16_memorisation).
// (one multiply-xorshift round: the keys are distinct per element and step, and the SR
// decision needs well-spread bits per element, not a full avalanche mix; the two-round
// finalizer it replaces cost 8 VALU per fragment — test_fp8_dgrad_stochastic_rounding_is_
// unbiased checks the statistics)
DG_DEV uint32_t sr_hash(uint32_t x) {
  x *= 0x9E3779B1u;
  return x ^ (x >> 16);
}
DG_DEV uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
DG_DEV uint32_t pack_bf8x4_sr(float a, float b, float c, float d, uint32_t h) {
  int v = __builtin_amdgcn_cvt_sr_bf8_f32(a, (int)h, 0, 0);
  v = __builtin_amdgcn_cvt_sr_bf8_f32(b, (int)rotl32(h, 8), v, 1);
  v = __builtin_amdgcn_cvt_sr_bf8_f32(c, (int)rotl32(h, 16), v, 2);
  v = __builtin_amdgcn_cvt_sr_bf8_f32(d, (int)rotl32(h, 24), v, 3);
  return (uint32_t)v;
}
template <int EPI, int MODE>
DG_DEV uint32_t pack8x4q(float a, float b, float c, float d, uint32_t key) {
  if constexpr (EPI == EPI_DGRAD && (MODE & 32) != 0) return pack_bf8x4_sr(a, b, c, d, sr_hash(key));
  return pack8x4<EPI>(a, b, c, d);
}

// 2 e4m3 / e5m2 -> 2 bf16 scaled by the power of two s (one v_cvt_scalef32_pk_bf16_*)
template <int EPI, bool HI>
DG_DEV uint32_t deq2(uint32_t w, float s) {
  if constexpr (EPI == EPI_FWD)
    return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)w, s, HI));
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_bf8((int)w, s, HI));
}

// 4 e4m3 bytes -> their 4 ReLU bits
DG_DEV uint32_t nzbits4(uint32_t w) {
  uint32_t t = w | (w >> 4);
  t |= t >> 2;
  t = (t | (t >> 1)) & 0x01010101u;
  return (t * 0x204081u) >> 21 & 0xFu;   // bits 0, 8, 16, 24 gathered into 21..24
}

// EPI_FWD: the forward stack (e4m3 activations, bias + pos-bias + ReLU, ReLU bits out);
// EPI_DGRAD: the backward-data chain dZ_{l-1} = mask_{l-1} * (W_l^T dZ_l) (e5m2 gradients,
// e4m3 weights: MX MFMA with A e4m3 / B e5m2), dequantized bf16 dZ frames out.
// MODE: 0 in production; timing ablations (tools/kbench_stack.py, wrong results):
// 2 = no A loads in the K loop, 4 = no copy-out, 64 = no epilogue (bias / quantize / image
// writes), 128 = no B reads (register operands).  MODE bit 8 (production, fp8 weight
// gradients): also store the raw fp8 copies (X8_0, every non-last layer's Y8) — a compile-time
// switch: a runtime null test around the store splits the K loop's blocks and costs 24-45
// spilled VGPRs.  MODE bit 16 (with 8): no dequantized bf16 copy-out of the non-last layers —
// every consumer reads the fp8 copies instead (forward: the MX-fp8 weight gradient, the
// backward-data chain reads ReLU bits; backward-data: the weight gradient and the bias-gradient
// partials read the e5m2 copies); the table's Y is null there.  MODE bit 32 (EPI_DGRAD):
// stochastic rounding of the e5m2 quantization (pack_bf8x4_sr)
template <int C, int EPI, int MODE, bool STAG = false>
__global__ void __launch_bounds__(NT) conv_stack_f8_kernel(F8Args a) {
  static_assert(!STAG || C == 128, "the staggered schedule needs the half-major K-steps");
  using G = Geo<C>;
  constexpr int NC = G::NC;
  constexpr int ROWB = G::ROWB;
  constexpr float QMAX = EPI == EPI_FWD ? FP8_MAX : BF8_MAX;
  constexpr int BFMT = EPI == EPI_FWD ? 0 : 1;   // MX MFMA B-operand format: e4m3 | e5m2
  constexpr bool BF16_LAST_IMAGE = C == 128 && EPI == EPI_FWD;  // last layer feeds the head
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int b = blockIdx.x;
  char* sI = smem + SCRATCH;                       // e4m3 image (C = 128 last layer: bf16)
  // STAG (C = 128): double-buffered image — layer l reads image l & 1 (at img_rd) and writes
  // its output into the other one, so a group's epilogue never waits for the other group's
  // reads of the layer's input
  int img_rd = 0;
  float* s_amax = (float*)(smem + G::AMAX_OFF);    // 2 x 8 floats (alternating per layer)
  // STAG (C = 128): counters W0 W1 (at cnt + 2, + 3: the waves of co-half 0 / 1 that wrote
  // their half of a layer's output, 4 per layer) and each layer's |y| max (float bits, ds_max
  // per wave; folded into amax_out once at the end) below the wg_amax slots, in the head
  // scratch (the head runs after the last of them is read)
  LDS_AS unsigned* cnt = (LDS_AS unsigned*)(smem + SCRATCH - 64 - 16);
  LDS_AS unsigned* s_lmax = (LDS_AS unsigned*)(smem + SCRATCH - 64 - 16 - 4 * MAXL);
  if constexpr (STAG) {
    if (tid < 4) cnt[tid] = 0u;
    if (tid < MAXL) s_lmax[tid] = 0u;
    const int wmu = __builtin_amdgcn_readfirstlane(wm);
    if (wmu == 1)
      for (int d = 0; d < a.stag_delay; ++d) __builtin_amdgcn_s_sleep(127);
  }

  // (MODE bit 256: per-wave s_memtime stamps of the layer phases, boards 0..7)
  auto stamp = [&](int l, int k) {
    if constexpr ((MODE & 256) != 0) {
      if (b < 8) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        if (lane == 0) a.dbg[((b * NW + wave) * MAXL + l) * 8 + k] = t;
      }
    }
  };
  // stochastic-rounding key base of this step (EPI_DGRAD, MODE bit 32)
  uint32_t sr_seed = 0;
  if constexpr (EPI == EPI_DGRAD && (MODE & 32) != 0)
    sr_seed = (uint32_t)*a.sr_step * 0x9E3779B9u;
  // ---- prologue: quantize the bf16 input frame into the image ----
  {
    const float inv = 1.f / *a.s_x0;
    const char* Xb = a.X0 + (size_t)b * FF * C * 2;
    float m = 0.f;
    for (int u = tid; u < FF * (C / 8); u += NT) {     // 8-channel pieces
      const int f = u / (C / 8), q = u % (C / 8);
      const uint4 v = *(const uint4*)(Xb + (size_t)u * 16);
      float x[8] = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xFFFF0000u),
                    __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xFFFF0000u),
                    __uint_as_float(v.z << 16), __uint_as_float(v.z & 0xFFFF0000u),
                    __uint_as_float(v.w << 16), __uint_as_float(v.w & 0xFFFF0000u)};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        m = fmaxf(m, fabsf(x[e]));
        x[e] = fmaxf(fminf(x[e] * inv, QMAX), -QMAX);
      }
      uint2 o;
      const uint32_t key = sr_seed + (uint32_t)((b * FF + f) * C + q * 8);
      o.x = pack8x4q<EPI, MODE>(x[0], x[1], x[2], x[3], key);
      o.y = pack8x4q<EPI, MODE>(x[4], x[5], x[6], x[7], key + 4);
      *(uint2*)(sI + f * ROWB + (((q >> 1) ^ fsig<C>(f)) * 16) + (q & 1) * 8) = o;
      // the fp8 copy of the quantized input (the fp8 weight gradient's operand)
      if constexpr ((MODE & 8) != 0) *(uint2*)(a.X8_0 + ((size_t)(b * FP8P + f) * C + q * 8)) = o;
    }
    if constexpr (STAG) {
      // the second image's zero border (frame rows 0 / 20, columns 0 / 20: the taps' padding;
      // the epilogues write interior pixels only) and its rows 441..447
      for (int u = tid; u < 87 * 8; u += NT) {
        const int k = u >> 3, q = u & 7;
        const int row = k < 21 ? k : k < 42 ? 420 + (k - 21) : k < 61 ? (k - 41) * 21
                        : k < 80 ? (k - 60) * 21 + 20 : 441 + (k - 80);
        *(uint4*)(sI + IMG2 + row * ROWB + q * 16) = uint4{0, 0, 0, 0};
      }
    }
    wg_amax(m, a.amax_x0, s_amax + 8);  // (contains the barrier: image complete)
  }

  const int lr = lane & 15;
  const int lq = lane >> 4;
  // per fragment: row byte offset f*ROWB (20 bits) | v = (x + 3y) & 7 << 20.  C = 128: the
  // 23 pixel slots past the board (wave 3's last fragment) sit on dump rows 441..463 of the
  // LDS past the e4m3 image (free until the last layer's bf16 image), so the lean epilogue
  // stores them without a branch; C = 256 reads pixel 0 there
  // (recomputed at every layer's start from an opaque lane index: kept live across the
  // epilogue, the 6 words get spilled there and reloaded on its critical path)
  uint32_t pk[NF];
  auto make_pk = [&]() {
    int lro = lr;
    asm volatile("" : "+v"(lro));
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      int p = wn * NF * 16 + j * 16 + lro;
      int f;
      if (p >= NPTS) {
        f = C == 128 ? FF + (p - NPTS) : F + 1;
      } else {
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
        f = (h + 1) * F + (w + 1);
      }
      pk[j] = (uint32_t)(f * ROWB) | ((uint32_t)fv(f) << 20);
    }
  };
  const uint32_t a_lane = (uint32_t)(wm * WM_BYTES + lane * 16);

  // A fragments i0, i0+1 of one K-step (A = the step's 16 KB): 2 KB per fragment
  auto load_A = [&](const char* A, int i0, i32x8 (&r)[MF]) {
    const char* p = A + a_lane;
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i) {
      const i32x4 lo = *(const i32x4*)(p + (2 * i) * 1024);
      const i32x4 hi = *(const i32x4*)(p + (2 * i + 1) * 1024);
      r[i] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
  };
  // B fragments (16 pixels x 128 channels of chunk c) of K-step st = t * NC + c (the weight
  // layout's [tap][chunk] order): lane group lq reads slots 8c + 2lq, 8c + 2lq + 1 (XOR the
  // row signature; the odd slot = even ^ 16 B)
  auto read_B = [&](int st, i32x8 (&bfr)[NF]) {
    int t, slot0;
    if constexpr (C == 128) {
      // half-major K-steps: step st = units 2 st (lane groups 0, 1) and 2 st + 1 (2, 3) of
      // n = 9 * half + tap (64 channels of one tap each): steps 0..3 read only channels 0..63
      // (co-half 0's output), 5..8 only 64..127, step 4 both (the staggered schedule's order)
      const int n = 2 * st + (lq >> 1);
      const int hh = n >= T ? 1 : 0;
      t = n - T * hh;
      slot0 = 4 * hh + 2 * (lq & 1);
    } else {
      t = st / NC;
      slot0 = 8 * (st - (st / NC) * NC) + 2 * lq;
    }
    const int toff = (t / 3 - 1) * F + (t % 3 - 1);
    const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
    const LDS_AS char* base = (const LDS_AS char*)(sI + img_rd);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int off = (int)(pk[j] & 0xFFFFFu) + toff * ROWB +
                      ((slot0 ^ sig_of<C>((int)(pk[j] >> 20) + tsig)) * 16);
      const i32x4 lo = *(const LDS_AS i32x4*)(base + off);
      const i32x4 hi = *(const LDS_AS i32x4*)(base + (off ^ 16));
      bfr[j] = i32x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    }
  };
  auto mma = [&](const i32x8 (&af)[MF], int i0, const i32x8 (&bfr)[NF], f32x4 (&acc)[MF][NF]) {
    // each MFMA cluster at wave priority 1 (12x128 fp8 +0.5%, 12x256 fp8 +0.7%;
    // profiles/r4_s2_wave_priority_ab.txt)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = i0; i < i0 + 2; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bfr[j], acc[i][j], 0,
                                                                      BFMT, 0, 127, 0, 127);
    __builtin_amdgcn_s_setprio(0);
  };

  // Copy-out of the previous layer's output (the e4m3 image) as bf16 (x s_prev) + ReLU bits:
  // thread tid handles 16-B piece u = tid + 512 s (pixel u / SLOTS, channels 16 (u % SLOTS)),
  // read from LDS in the step before it is stored.  Pieces past the board repeat the last
  // one (same bytes): every wave issues the same stores.
  // (C = 128: the waves of co-half wm copy out channels 64 wm .. 64 wm + 63 — the half they
  // wrote themselves — 256 threads x 6 steps, as the staggered schedule requires)
  auto co_pq = [&](int s_, int tq, int& p, int& q) {
    if constexpr (C == 128) {
      const int u = min((tq & 255) + 256 * s_, NPTS * 4 - 1);
      p = u >> 2;
      q = 4 * (tq >> 8) + (u & 3);
    } else {
      const int u = min(tq + NT * s_, G::PIECES - 1);
      p = u / G::SLOTS;
      q = u % G::SLOTS;
    }
  };
  auto co_read = [&](int s_) -> uint4 {
    int p, q;
    co_pq(s_, tid, p, q);
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    return *(const uint4*)(sI + img_rd + f * ROWB + ((q ^ fsig<C>(f)) * 16));
  };
  // (y8: the fp8 copy of the previous layer's output, or null)
  // (yb / y8b: the bf16 / fp8 output frames advanced to this board, per layer)
  auto co_store = [&](int s_, const uint4& v, char* yb, uint8_t* y8b, uint8_t* mask,
                      float s_prev) {
    // (opaque piece index: visible, the compiler hoists the per-step 64-bit store offsets
    // out of the layer loop and spills them — reloaded with vmcnt(0) in every layer)
    int tq = tid;
    asm volatile("" : "+v"(tq));
    int p, q;
    co_pq(s_, tq, p, q);
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    const int inner = f * C + q * 16;                  // element offset within the board
    if constexpr ((MODE & 8) != 0) *(uint4*)(y8b + inner) = v;
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[8];
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // (s_prev is a power of two: fp8_update_scales rounds every such scale up to one)
      o[2 * k] = deq2<EPI, false>(wd[k], s_prev);
      o[2 * k + 1] = deq2<EPI, true>(wd[k], s_prev);
      if constexpr (EPI == EPI_FWD)
        bits |= nzbits4(wd[k]) << (4 * k);   // ReLU bit = byte nonzero (values are >= 0)
    }
    if constexpr ((MODE & 16) == 0) {
      char* yp = yb + inner * 2;
      *(uint4*)yp = uint4{o[0], o[1], o[2], o[3]};
      *(uint4*)(yp + 16) = uint4{o[4], o[5], o[6], o[7]};
    }
    if constexpr (EPI == EPI_FWD)
      *(uint16_t*)(mask + ((size_t)b * NPTS + p) * (C / 8) + q * 2) = (uint16_t)bits;
  };

  i32x8 Ak[MF];
  load_A(a.L[0].A8, 0, Ak);
  load_A(a.L[0].A8, 2, Ak);

  if constexpr (C != 128) make_pk();
  // The layer loop.  The body is conv_stack_f8_layer.inc.h (why it is a textual include:
  // there).  Every variant but C = 256 backward-data splits it; that one keeps one rolled loop
  // (split, it went 248 -> 256 VGPRs + 1 spill and its kernel time up to +4%).  The C = 256
  // forward keeps the general epilogue in both copies (its lean form measured no faster).
  if constexpr (!(C == 256 && EPI == EPI_DGRAD)) {
    for (int l = 0; l + 1 < a.nl; ++l) {
      constexpr bool last = false;
#include "conv_stack_f8_layer.inc.h"
    }
    {
      const int l = a.nl - 1;
      constexpr bool last = true;
#include "conv_stack_f8_layer.inc.h"
    }
  } else {
    for (int l = 0; l < a.nl; ++l) {
      const bool last = l + 1 == a.nl;
#include "conv_stack_f8_layer.inc.h"
    }
  }
  if constexpr (STAG) {
    // every layer's |y| max (the last layer's barrier ordered every wave's ds_max before it)
    if (tid < a.nl - 1) atomicMax(a.L[tid].amax_out, s_lmax[tid]);
    __syncthreads();   // (the slots sit in the head scratch)
  }
  if constexpr (BF16_LAST_IMAGE) {
    // last layer's output (bf16 image): exposed copy-out + mask, as conv_stack2 (skipped with
    // the fused head: training reads neither; evaluation runs the head-less launch)
    const F8Layer Ll = a.L[a.nl - 1];
    const int co_q = tid & 15;
    for (int s_ = 0; s_ < (a.fuse_head ? 0 : (NPTS * 16 + NT - 1) / NT); ++s_) {
      const int p = min((tid >> 4) + 32 * s_, NPTS - 1);
      const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
      const int f = (h + 1) * F + (w + 1);
      const uint4 v =
          *(const uint4*)(sI + (co_q >> 3) * H_BYTES + f * 128 + (((co_q & 7) ^ fsig8(f)) * 16));
      *(uint4*)(Ll.Y + ((size_t)(b * FF + f) * C) * 2 + co_q * 16) = v;
      typedef unsigned short us2 __attribute__((ext_vector_type(2)));
      auto nz2 = [](uint32_t x) {
        const us2 m = __builtin_elementwise_min(__builtin_bit_cast(us2, x), us2{1, 1});
        const uint32_t t = __builtin_bit_cast(uint32_t, m);
        return (t | (t >> 15)) & 3u;
      };
      Ll.mask[((size_t)b * NPTS + p) * 16 + co_q] =
          (uint8_t)(nz2(v.x) | (nz2(v.y) << 2) | (nz2(v.z) << 4) | (nz2(v.w) << 6));
    }
    if (a.fuse_head) dghead::head_body<C>(a.head, b, sI, smem, [](int) {});
  }
  if constexpr (C == 256 && EPI == EPI_FWD) {
    // the 256-channel image does not stay in LDS as bf16: the fused head reads the last
    // layer's bf16 frame back (this workgroup's stores, retired here) — no head launch
    if (a.fuse_head) {
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      dghead::HeadMArgs h = a.head;
      h.X = a.L[a.nl - 1].Y;
      dghead::head_from_frame<256>(h, b, smem);
    }
  }
}

int g_f8_mode = 0;

// The staggered schedule (C = 128): -1 = not yet read from DG_STACK_F8_STAG ("MODE[,DELAY]"),
// else 0 off, 1 both stacks (default: with every C = 128 variant's layer body split in two,
// conv_stack_f8_layer.inc.h, the staggered forward is the faster one again — 144.2 vs 147.3 us
// per 10 layers; 12x128 fp8 step 416.9-419.6k vs 410.0-414.4k with the backward-data stack
// only, same box, profiles/r5_stack_f8_stag.txt §10), 2 the backward-data stack only;
// co-half-1 start delay
int g_f8_stag = -1, g_f8_delay = 0;
void f8_sched_from_env() {
  if (g_f8_stag >= 0) return;
  const char* e = getenv("DG_STACK_F8_STAG");
  g_f8_stag = 1;
  if (e && *e) {
    int v = 0, d = g_f8_delay;
    const int n = sscanf(e, "%d,%d", &v, &d);
    g_f8_stag = n >= 1 && v >= 0 && v <= 2 ? v : 1;
    if (n >= 2) g_f8_delay = d;
  }
}

template <int C, int EPI, int MODE, bool STAG>
hipError_t launch_f8_s(const F8Args& a, int B, hipStream_t stream) {
  constexpr size_t lds = Geo<C>::LDS;
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_stack_f8_kernel<C, EPI, MODE, STAG>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL((conv_stack_f8_kernel<C, EPI, MODE, STAG>), dim3(B), dim3(NT), lds, stream,
                     a);
  return hipGetLastError();
}

// (the timing ablations run the barrier schedule only)
unsigned long long* g_f8_dbg = nullptr;   // MODE bit 256 stamps (diagnostics)

template <int C, int EPI, int MODE>
hipError_t launch_f8(const F8Args& a, int B, hipStream_t stream) {
  if constexpr (C == 128 && (MODE & (2 | 4 | 64 | 128)) == 0) {
    if constexpr (MODE == 24 || MODE == 56) {
      if (g_f8_dbg) {
        if (g_f8_mode == 4)   // (stamps of the no-copy-out ablation, barrier schedule)
          return launch_f8_s<C, EPI, MODE | 256 | 4, false>(a, B, stream);
        return a.stag_on ? launch_f8_s<C, EPI, MODE | 256, true>(a, B, stream)
                         : launch_f8_s<C, EPI, MODE | 256, false>(a, B, stream);
      }
    }
    if (a.stag_on) return launch_f8_s<C, EPI, MODE, true>(a, B, stream);
  }
  return launch_f8_s<C, EPI, MODE, false>(a, B, stream);
}

template <int C>
hipError_t launch_mode(int epi, const F8Args& a, int B, hipStream_t stream) {
  const bool y8 = a.X8_0 != nullptr;
  // no bf16 frame wanted for any non-last layer (with the fp8 copies): skip their bf16 copy-out
  bool any_y = false;
  for (int i = 0; i + 1 < a.nl; ++i) any_y |= a.L[i].Y != nullptr;
  if (epi == EPI_DGRAD) {
    if (a.sr_step) {
      if (!y8) return launch_f8<C, EPI_DGRAD, 32>(a, B, stream);
      if (any_y) return launch_f8<C, EPI_DGRAD, 40>(a, B, stream);
      // the production backward-data chain and its timing ablations
      switch (g_f8_mode) {
        case 2: return launch_f8<C, EPI_DGRAD, 56 | 2>(a, B, stream);
        case 4:
          if (g_f8_dbg) return launch_f8<C, EPI_DGRAD, 56>(a, B, stream);   // (stamped variant)
          return launch_f8<C, EPI_DGRAD, 56 | 4>(a, B, stream);
        case 64: return launch_f8<C, EPI_DGRAD, 56 | 64>(a, B, stream);
        case 68: return launch_f8<C, EPI_DGRAD, 56 | 68>(a, B, stream);
        case 198: return launch_f8<C, EPI_DGRAD, 56 | 198>(a, B, stream);
        default: return launch_f8<C, EPI_DGRAD, 56>(a, B, stream);
      }
    }
    if (!y8) return launch_f8<C, EPI_DGRAD, 0>(a, B, stream);
    return any_y ? launch_f8<C, EPI_DGRAD, 8>(a, B, stream)
                 : launch_f8<C, EPI_DGRAD, 24>(a, B, stream);
  }
  if (y8 && any_y) return launch_f8<C, EPI_FWD, 8>(a, B, stream);
  if (y8) {
    // the production forward (fp8 copies only) and its timing ablations
    switch (g_f8_mode) {
      case 2: return launch_f8<C, EPI_FWD, 24 | 2>(a, B, stream);
      case 4:
        if (g_f8_dbg) return launch_f8<C, EPI_FWD, 24>(a, B, stream);   // (stamped variant)
        return launch_f8<C, EPI_FWD, 24 | 4>(a, B, stream);
      case 64: return launch_f8<C, EPI_FWD, 24 | 64>(a, B, stream);
      case 68: return launch_f8<C, EPI_FWD, 24 | 68>(a, B, stream);
      case 128: return launch_f8<C, EPI_FWD, 24 | 128>(a, B, stream);
      case 196: return launch_f8<C, EPI_FWD, 24 | 196>(a, B, stream);
      case 198: return launch_f8<C, EPI_FWD, 24 | 198>(a, B, stream);
      default: return launch_f8<C, EPI_FWD, 24>(a, B, stream);
    }
  }
  switch (g_f8_mode) {
    case 2: return launch_f8<C, EPI_FWD, 2>(a, B, stream);
    case 4: return launch_f8<C, EPI_FWD, 4>(a, B, stream);
    case 6: return launch_f8<C, EPI_FWD, 6>(a, B, stream);
    default: return launch_f8<C, EPI_FWD, 0>(a, B, stream);
  }
}

// table: nl rows of 8 int64 {A8, pbias, Y, mask, s_in, s_w, s_out, amax_out}

hipError_t f8_launch(int C, int epi, const long long* table, int nl, const void* X0,
                     const float* s_x0, unsigned* amax_x0, int B, const dghead::HeadMArgs* head,
                     const long long* y8, const long long* sr_step, hipStream_t stream) {
  if (nl <= 0 || nl > MAXL || B <= 0 || !s_x0 || !amax_x0) return hipErrorInvalidValue;
  if ((C != 128 && C != 256) || (epi != EPI_FWD && epi != EPI_DGRAD)) return hipErrorInvalidValue;
  if (head && epi != EPI_FWD) return hipErrorInvalidValue;
  if (sr_step && epi != EPI_DGRAD) return hipErrorInvalidValue;
  F8Args a;
  f8_sched_from_env();
  a.stag_delay = g_f8_delay;
  a.stag_on = C == 128 && (g_f8_stag == 1 || (g_f8_stag == 2 && epi == EPI_DGRAD)) ? 1 : 0;
  a.dbg = g_f8_dbg;
  a.sr_step = sr_step;
  a.X0 = (const char*)X0;
  a.s_x0 = s_x0;
  a.amax_x0 = amax_x0;
  a.X8_0 = y8 ? (uint8_t*)y8[0] : nullptr;
  if (y8 && !a.X8_0) return hipErrorInvalidValue;
  a.nl = nl;
  a.fuse_head = head ? 1 : 0;
  a.head = head ? *head : dghead::HeadMArgs{};
  for (int i = 0; i < nl; ++i) {
    const long long* t = table + 8 * i;
    F8Layer& L = a.L[i];
    L.A8 = (const char*)t[0];
    L.pbias = (const bf16_t*)t[1];
    L.Y = (char*)t[2];
    L.mask = (uint8_t*)t[3];
    L.s_in = (const float*)t[4];
    L.s_w = (const float*)t[5];
    L.s_out = (const float*)t[6];
    L.amax_out = (unsigned*)t[7];
    L.Y8 = y8 ? (uint8_t*)y8[1 + i] : nullptr;
    // (a y8 table covers every layer: all non-last copies present, the last absent)
    if (y8 && (i + 1 == nl) != (L.Y8 == nullptr)) return hipErrorInvalidValue;
    // (Y of a non-last forward layer may be null when the fp8 copies are written: then every
    // non-last Y must be null and the bf16 copy-out is skipped)
    const bool y_opt = y8 && i + 1 < nl;
    if (!L.A8 || (!L.Y && !y_opt) || !L.mask || !L.s_in || !L.s_w || !L.s_out || !L.amax_out)
      return hipErrorInvalidValue;
    if (y_opt && i > 0 && (L.Y == nullptr) != (a.L[0].Y == nullptr)) return hipErrorInvalidValue;
    if (epi == EPI_FWD && !L.pbias) return hipErrorInvalidValue;
  }
  return C == 128 ? launch_mode<128>(epi, a, B, stream) : launch_mode<256>(epi, a, B, stream);
}

}  // namespace

extern "C" {

void dg_conv_stack_f8_set_mode(int m) { g_f8_mode = m; }

// the staggered schedule of C = 128 (overrides DG_STACK_F8_STAG): 0 off, 1 both stacks, 2
// backward-data only; co-half-1 start delay (s_sleep 127 rounds)
void dg_conv_stack_f8_set_debug(unsigned long long* dbg) { g_f8_dbg = dbg; }

void dg_conv_stack_f8_set_sched(int stag, int delay) {
  g_f8_stag = stag >= 0 && stag <= 2 ? stag : 1;
  g_f8_delay = delay;
}

// table: nl rows of {A8 (fragment-ordered e4m3 weights), pbias_frag, Y, mask, s_in, s_w,
// s_out, amax_out} (int64); epi 1 forward, 2 backward-data; sr_step (backward-data): the
// device step counter seeding stochastic rounding of the e5m2 gradients (null: nearest even)
hipError_t dg_conv_stack_f8(int C, int epi, const long long* table, int nl, const void* X0,
                            const float* s_x0, unsigned* amax_x0, int B, const long long* y8,
                            const long long* sr_step, hipStream_t stream) {
  return f8_launch(C, epi, table, nl, X0, s_x0, amax_x0, B, nullptr, y8, sr_step, stream);
}

// C = 128: the head on the last layer's LDS image; 256: on its bf16 frame, read back
hipError_t dg_conv_stack_f8_fwd_head(int C, const long long* table, int nl, const void* X0,
                                     const float* s_x0, unsigned* amax_x0, int B, const float* w,
                                     const float* bias, const float* posb, const int* labels,
                                     float* loss, int* pred, void* dZ, float* gw_part,
                                     float* dzb, int head_relu, float grad_scale,
                                     const long long* y8, hipStream_t stream) {
  const dghead::HeadMArgs h{nullptr, w, bias, posb, labels, loss, pred, nullptr, (char*)dZ,
                            gw_part, dzb, head_relu, grad_scale};
  return f8_launch(C, EPI_FWD, table, nl, X0, s_x0, amax_x0, B, &h, y8, nullptr, stream);
}

}  // extern "C"
