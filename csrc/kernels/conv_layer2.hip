// One hidden 3x3 layer (C -> C, C = 256, pad 1) per launch, forward or backward-data, on
// conv_stack2's K loop: fragment-ordered weights streamed from L2 into VGPRs half a K-step
// ahead, B fragments from a board-resident 64-channel image, no barrier inside a chunk.
//
// A 21x21x256 bf16 frame (226 KB) does not fit in LDS, so there is no multi-layer stack at
// d = 256 (the fp8 stack holds its one-byte image; conv_stack_f8.hip).  Here a workgroup
// (8 waves) owns one board x 128 output channels (grid B x 2): the board's input frame
// streams through two 56 KB chunk buffers (64 channels each; chunk c+1's LDS-DMA is spread
// over chunk c's 9 tap steps, one barrier per chunk), 36 K-steps of 64 k.  The epilogue
// stages the bf16 tile pixel-major in the (then free) chunk buffers and stores it as
// coalesced 16-B pieces (+ the forward's ReLU bits); borders of the output frame are never
// written (zero).
//   EPI_FWD  : Y = relu(W * X + bias table)            (writes the ReLU bitmask)
//   EPI_DGRAD: Y = ReLU bits of the layer below * (W_d * X)  (W_d: flipped, transposed)
// The per-layer board kernel it replaces (conv_board.hip) stages the weights through an LDS
// ring with a barrier per K-step.
// Reference ops: SpatialConvolutionMM + Add + ReLU (experiments.lua:137-147) and their
// backward (train.lua:10).
#include "dg_common.h"
#include "head_body.h"

#include <cstdlib>

using namespace dg;

namespace {

constexpr int EPI_FWD = 1;
constexpr int EPI_DGRAD = 2;
constexpr int F = 21;
constexpr int FF = F * F;
constexpr int HROWS = 448;
constexpr int H_BYTES = HROWS * 128;       // one 64-channel chunk image
constexpr int T = 9;
constexpr int MF = 4, NF = 6;              // wave tile 64 co x 96 px
constexpr int NW = 8, NT = NW * 64;
constexpr int STEP_BYTES = 2 * 2 * MF * 64 * 16;   // 16 KB: one K-step of one co half
constexpr int WM_BYTES = STEP_BYTES / 2;
constexpr int LDS_BYTES = 2 * H_BYTES;     // two chunk buffers (the epilogue's 96 KB tile fits)
static_assert(384 * 256 <= LDS_BYTES, "epilogue staging");

struct LayerArgs {
  const char* A;         // fragment-ordered weights [C/128 h][9 C/64 steps][2][2][4][64] x 8
  const bf16_t* pbias;   // EPI_FWD: bf16 bias + pos-bias, stack fragment order [h][24][2][4][64]
  const char* X;         // input frame [B][21][21][C] bf16
  char* Y;               // output frame [B][21][21][C] bf16 (interior written)
  uint8_t* mask;         // [B][361][C/8]: EPI_FWD writes, EPI_DGRAD reads (layer below)
  int C;
};

DG_DEV int fsig(int f) { return ((f % F) + 3 * (f / F)) & 7; }

DG_DEV void lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
DG_DEV uint32_t bf16x2_bits(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
}
DG_DEV uint32_t relu_bf16x2(f32x2 v) {
  const s16x2 h = __builtin_bit_cast(s16x2, __builtin_convertvector(v, bf16x2v));
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(h, s16x2{0, 0}));
}
DG_DEV f32x2 bf16x2_f32(uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xFFFF0000u)};
}
DG_DEV uint32_t pair_mask(uint32_t nib) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_sbfe((int)nib, 0, 1);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int)nib, 1, 1);
  return __builtin_amdgcn_perm(hi, lo, 0x07060100u);
}

template <int EPI>
__global__ void __launch_bounds__(NT) conv_layer2_kernel(LayerArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int b = blockIdx.x, h = blockIdx.y;
  const int C = a.C, nch = C / 64, nsteps = nch * T;
  const char* Xb = a.X + (size_t)b * FF * C * 2;
  const char* Ah = a.A + (size_t)h * nsteps * STEP_BYTES;

  // chunk-image DMA instruction j (rows 8j .. 8j+7) of chunk c into buffer buf
  auto stage_H = [&](int buf, int c, int j) {
    const int rl = j * 8 + (lane >> 3);
    const int r = rl < FF ? rl : FF - 1;
    const int gs = (lane & 7) ^ fsig(rl);
    glds16(Xb + ((size_t)r * C + c * 64 + gs * 8) * 2, (LDS_AS void*)(smem + buf * H_BYTES + j * 1024));
  };
  for (int j = wave; j < HROWS / 8; j += NW) stage_H(0, 0, j);

  const int lr = lane & 15;
  const int lq = lane >> 4;
  uint32_t pk[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = wn * NF * 16 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int hh = p / BOARD, w = p - (p / BOARD) * BOARD;
    pk[j] = (uint32_t)(((hh + 1) * F + (w + 1)) * 128) | ((uint32_t)(((w + 1) + 3 * (hh + 1)) & 7) << 16);
  }
  const uint32_t a_lane = (uint32_t)(wm * WM_BYTES + lane * 16);
  auto load_A = [&](const char* A, int kk, bf16x8 (&r)[MF]) {
    const char* p = A + a_lane + kk * MF * 1024;
#pragma unroll
    for (int i = 0; i < MF; ++i) r[i] = *(const bf16x8*)(p + i * 1024);
  };
  auto read_B = [&](const char* sHc, int t, int kk, bf16x8 (&bfr)[NF]) {
    const int toff = (t / 3 - 1) * F + (t % 3 - 1);
    const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int off = (int)(pk[j] & 0xFFFFu) + toff * 128 +
                      ((lq ^ (((int)(pk[j] >> 16) + tsig) & 7)) * 16);
      bfr[j] = lds_read_b128((const LDS_AS char*)(sHc + (off ^ (kk * 64))));
    }
  };
  auto mma = [&](const bf16x8 (&af)[MF], const bf16x8 (&bfr)[NF], f32x4 (&acc)[MF][NF]) {
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  };

  __syncthreads();  // chunk 0 landed (the compiler waits for the LDS-DMA before the barrier)

  bf16x8 Ak[2][MF];
  load_A(Ah, 0, Ak[0]);
  load_A(Ah, 1, Ak[1]);
  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nch; ++c) {
    const char* sHc = smem + (c & 1) * H_BYTES;
#pragma unroll 1
    for (int t = 0; t < T; ++t) {
      const int s = c * T + t;
      const char* An = s + 1 < nsteps ? Ah + (s + 1) * STEP_BYTES : Ah;  // (harmless at the end)
      bf16x8 bfr[NF];
      read_B(sHc, t, 0, bfr);
      mma(Ak[0], bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      load_A(An, 0, Ak[0]);
      read_B(sHc, t, 1, bfr);
      __builtin_amdgcn_sched_barrier(0);
      mma(Ak[1], bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      load_A(An, 1, Ak[1]);
      // the next chunk's image: one DMA instruction per wave and tap step (7 x 8 = 56),
      // last in the step, into the buffer the previous chunk used
      if (c + 1 < nch && t < HROWS / 8 / NW) stage_H((c + 1) & 1, c + 1, wave * (HROWS / 8 / NW) + t);
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();  // chunk c+1 landed; every wave is past chunk c's reads
  }

  // ---- epilogue ----
  int z0 = 0;
  asm volatile("" : "+v"(z0));
  uint2 eb[NF][EPI == EPI_FWD ? MF : 1];
  uint2 em[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
    if constexpr (EPI == EPI_FWD) {
      const uint2* pf = (const uint2*)a.pbias + (((h * 24 + wn * NF + j) * 2 + wm) * 4) * 64 + lane + z0;
#pragma unroll
      for (int i = 0; i < MF; ++i) eb[j][i] = pf[i * 64];
    } else {
      em[j] = *(const uint2*)(a.mask + ((size_t)b * NPTS + p) * (C / 8) + h * 16 + wm * 8 + z0);
    }
  }
  // the tile, pixel-major: row p = 256 B (this half's 128 channels), 16-B slot q ^ (p & 15)
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int p = wn * NF * 16 + j * 16 + lr;
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int cl = wm * 64 + i * 16 + lq * 4;   // channel within the half
      const f32x4 v = acc[i][j];
      uint2 o;
      if constexpr (EPI == EPI_FWD) {
        o.x = relu_bf16x2(f32x2{v[0], v[1]} + bf16x2_f32(eb[j][i].x));
        o.y = relu_bf16x2(f32x2{v[2], v[3]} + bf16x2_f32(eb[j][i].y));
      } else {
        const int cw = i * 16 + lq * 4;
        const uint32_t word = (i < 2) ? em[j].x : em[j].y;
        const uint32_t nib = word >> ((cw & 31) >> 3 << 3) >> (cw & 4);
        o.x = bf16x2_bits(f32x2{v[0], v[1]}) & pair_mask(nib);
        o.y = bf16x2_bits(f32x2{v[2], v[3]}) & pair_mask(nib >> 2);
      }
      if (p < NPTS) *(uint2*)(smem + z0 + p * 256 + (((cl >> 3) ^ (p & 15)) * 16) + (cl & 4) * 2) = o;
    }
  }
  lds_barrier();
  for (int u = tid; u < NPTS * 16; u += NT) {
    const int p = u >> 4, q = u & 15;
    const uint4 v = *(const uint4*)(smem + p * 256 + ((q ^ (p & 15)) * 16));
    const int hh = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (hh + 1) * F + (w + 1);
    *(uint4*)(a.Y + ((size_t)(b * FF + f) * C + h * 128 + q * 8) * 2) = v;
    if (EPI == EPI_FWD && a.mask) {
      const uint32_t m = (((v.x + 0x7fff7fffu) >> 15) & 0x10001u) |
                         (((v.y + 0x7fff7fffu) >> 13) & 0x40004u) |
                         (((v.z + 0x7fff7fffu) >> 11) & 0x100010u) |
                         (((v.w + 0x7fff7fffu) >> 9) & 0x400040u);
      a.mask[((size_t)b * NPTS + p) * (C / 8) + h * 16 + q] = (uint8_t)(m | (m >> 15));
    }
  }
}

template <int EPI>
hipError_t launch_layer2(const LayerArgs& a, int B, hipStream_t stream) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_layer2_kernel<EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    done = true;
  }
  hipLaunchKernelGGL((conv_layer2_kernel<EPI>), dim3(B, a.C / 128), dim3(NT), LDS_BYTES, stream, a);
  return hipGetLastError();
}


// ------------------------------------------------------------------------------------
// conv_layer2_multi: a RUN of nl hidden layers (forward: X_l+1 = Y_l; backward-data: the
// dZ chain top -> down) in ONE launch, one workgroup per board (grid B), on the same K loop.
// A board's next layer only reads that board's own output, which this workgroup wrote
// (L2-resident; every wave retires its stores with vmcnt(0) at the next item's chunk-0
// barrier, before any DMA of the channels they hold), so the layers need no grid-wide
// synchronisation.  Per layer the workgroup runs the C/128 output halves back to back.  The
// next item's chunk 0 is staged into buffer 0 during the current item's last chunk (which
// sits in buffer 1): the same frame for the second half, the next layer's channels 0..63
// (written by the first half) at a layer change; the epilogue stages in buffer 1 + a 35 KB
// extension.  No item after the first waits for a chunk-0 DMA, and the epilogue stores drain
// under the next item's MFMAs.  Per-item math is the single-layer kernel's (bit-identical).
constexpr int MAXL2 = 16;
struct MultiArgs {
  LayerArgs L[MAXL2];
  int nl;
  dghead::HeadMArgs head;   // HEAD: the policy head on the run's last output (X = last Y)
};
constexpr int STG_OFF = H_BYTES;                       // epilogue staging: buffer 1 + ext
constexpr int LDS_MULTI = H_BYTES + NPTS * 256;        // 149760 B
static_assert(LDS_MULTI <= 160 * 1024, "LDS");
static_assert(dghead::frame_head_lds(256) <= LDS_MULTI, "fused head LDS");

// HEAD (forward, C = 256): after the run's last layer the workgroup runs the policy head of
// its board (head_body.h: forward, log-softmax / NLL / argmax, and the head's backward) on
// the output frame it has just written — no separate head launch (its 56 us at 12x256 sat
// between the forward and backward-data runs) and the frame is read back from L2 / MALL.
template <int EPI, int BPF, bool HEAD>
__global__ void __launch_bounds__(NT) conv_layer2_multi_kernel(MultiArgs m) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int b = blockIdx.x;
  const int C = m.L[0].C, nch = C / 64, nsteps = nch * T, nh = C / 128;
  const int nitems = m.nl * nh;

  auto stage_H = [&](const char* Xb, int buf, int c, int j) {
    const int rl = j * 8 + (lane >> 3);
    const int r = rl < FF ? rl : FF - 1;
    const int gs = (lane & 7) ^ fsig(rl);
    glds16(Xb + ((size_t)r * C + c * 64 + gs * 8) * 2, (LDS_AS void*)(smem + buf * H_BYTES + j * 1024));
  };
  const int lr = lane & 15;
  const int lq = lane >> 4;
  uint32_t pk[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = wn * NF * 16 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int hh = p / BOARD, w = p - (p / BOARD) * BOARD;
    pk[j] = (uint32_t)(((hh + 1) * F + (w + 1)) * 128) | ((uint32_t)(((w + 1) + 3 * (hh + 1)) & 7) << 16);
  }
  const uint32_t a_lane = (uint32_t)(wm * WM_BYTES + lane * 16);
  auto load_A = [&](const char* A, int kk, bf16x8 (&r)[MF]) {
    const char* p = A + a_lane + kk * MF * 1024;
#pragma unroll
    for (int i = 0; i < MF; ++i) r[i] = *(const bf16x8*)(p + i * 1024);
  };
  auto read_B = [&](const char* sHc, int t, int kk, bf16x8 (&bfr)[NF]) {
    const int toff = (t / 3 - 1) * F + (t % 3 - 1);
    const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int off = (int)(pk[j] & 0xFFFFu) + toff * 128 +
                      ((lq ^ (((int)(pk[j] >> 16) + tsig) & 7)) * 16);
      bfr[j] = lds_read_b128((const LDS_AS char*)(sHc + (off ^ (kk * 64))));
    }
  };
  auto mma = [&](const bf16x8 (&af)[MF], const bf16x8 (&bfr)[NF], f32x4 (&acc)[MF][NF]) {
    // each k-half's MFMA cluster at wave priority 1: the SIMD's other wave then issues its
    // LDS reads / loads around the cluster instead of between its MFMAs (12x256 bf16 +0.4%,
    // profiles/r4_s2_wave_priority_ab.txt)
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
  };

  bool staged = false;   // buffer 0 already holds this item's chunk 0
#pragma unroll 1
  for (int it = 0; it < nitems; ++it) {
    const int l = it / nh, h = it - (it / nh) * nh;
    const bool next_same = h + 1 < nh;     // the next item reads the same input frame
    const char* Xb = m.L[l].X + (size_t)b * FF * C * 2;
    const char* Ah = m.L[l].A + (size_t)h * nsteps * STEP_BYTES;
    // the next item's chunk 0 (channels 0..63) is staged during this item's last chunk: the
    // same frame, or — at a layer change with two output halves — the next layer's input,
    // whose channels 0..63 the FIRST half of this layer wrote (its stores completed at this
    // item's chunk-0 barrier)
    const bool pf_next = next_same || (nh > 1 && l + 1 < m.nl);
    const char* Xn = next_same ? Xb : (l + 1 < m.nl ? m.L[l + 1].X + (size_t)b * FF * C * 2 : Xb);
    if (!staged) {
      if (it > 0) {   // (C = 128: this layer's input is the previous item's output)
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
      }
      for (int j = wave; j < HROWS / 8; j += NW) stage_H(Xb, 0, 0, j);
      __syncthreads();  // chunk 0 landed
    }  // (else it landed at the previous item's last-chunk barrier)

    bf16x8 Ak[2][MF];
    load_A(Ah, 0, Ak[0]);
    load_A(Ah, 1, Ak[1]);
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c = 0; c < nch; ++c) {
      const char* sHc = smem + (c & 1) * H_BYTES;
      const bool dma = c + 1 < nch || pf_next;
      const int cn = c + 1 < nch ? c + 1 : 0;       // chunk (of this or the next item) to stage
      const char* Xs = c + 1 < nch ? Xb : Xn;
#pragma unroll 1
      for (int t = 0; t < T; ++t) {
        const int s = c * T + t;
        const char* An = s + 1 < nsteps ? Ah + (s + 1) * STEP_BYTES : Ah;
        if constexpr (BPF == 1) {
          // k-half 1's B fragments read before k-half 0's MFMAs (+24 VGPRs): their LDS
          // latency hides under this wave's own MFMAs, not only the SIMD partner's
          bf16x8 bfr[NF], bfr1[NF];
          read_B(sHc, t, 0, bfr);
          read_B(sHc, t, 1, bfr1);
          mma(Ak[0], bfr, acc);
          __builtin_amdgcn_sched_barrier(0);
          load_A(An, 0, Ak[0]);
          __builtin_amdgcn_sched_barrier(0);
          mma(Ak[1], bfr1, acc);
        } else {
          bf16x8 bfr[NF];
          read_B(sHc, t, 0, bfr);
          mma(Ak[0], bfr, acc);
          __builtin_amdgcn_sched_barrier(0);
          load_A(An, 0, Ak[0]);
          read_B(sHc, t, 1, bfr);
          __builtin_amdgcn_sched_barrier(0);
          mma(Ak[1], bfr, acc);
        }
        __builtin_amdgcn_sched_barrier(0);
        load_A(An, 1, Ak[1]);
        if (dma && t < HROWS / 8 / NW) stage_H(Xs, (c + 1) & 1, cn, wave * (HROWS / 8 / NW) + t);
        __builtin_amdgcn_sched_barrier(0);
      }
      // chunk 0's barrier also retires the previous item's epilogue stores (vmcnt(0) in every
      // wave): chunk 2+ of a new layer read them, and their DMAs issue after this barrier
      if (c == 0) __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();  // the staged chunk landed; every wave is past chunk c's reads
    }

    // ---- epilogue (the single-layer kernel's, staged at STG_OFF) ----
    const LayerArgs& a = m.L[l];
    int z0 = 0;
    asm volatile("" : "+v"(z0));
    uint2 eb[NF][EPI == EPI_FWD ? MF : 1];
    uint2 em[NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
      if constexpr (EPI == EPI_FWD) {
        const uint2* pf = (const uint2*)a.pbias + (((h * 24 + wn * NF + j) * 2 + wm) * 4) * 64 + lane + z0;
#pragma unroll
        for (int i = 0; i < MF; ++i) eb[j][i] = pf[i * 64];
      } else {
        em[j] = *(const uint2*)(a.mask + ((size_t)b * NPTS + p) * (C / 8) + h * 16 + wm * 8 + z0);
      }
    }
    char* stg = smem + STG_OFF;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = wn * NF * 16 + j * 16 + lr;
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int cl = wm * 64 + i * 16 + lq * 4;
        const f32x4 v = acc[i][j];
        uint2 o;
        if constexpr (EPI == EPI_FWD) {
          o.x = relu_bf16x2(f32x2{v[0], v[1]} + bf16x2_f32(eb[j][i].x));
          o.y = relu_bf16x2(f32x2{v[2], v[3]} + bf16x2_f32(eb[j][i].y));
        } else {
          const int cw = i * 16 + lq * 4;
          const uint32_t word = (i < 2) ? em[j].x : em[j].y;
          const uint32_t nib = word >> ((cw & 31) >> 3 << 3) >> (cw & 4);
          o.x = bf16x2_bits(f32x2{v[0], v[1]}) & pair_mask(nib);
          o.y = bf16x2_bits(f32x2{v[2], v[3]}) & pair_mask(nib >> 2);
        }
        if (p < NPTS) *(uint2*)(stg + z0 + p * 256 + (((cl >> 3) ^ (p & 15)) * 16) + (cl & 4) * 2) = o;
      }
    }
    lds_barrier();
    char* Yb = a.Y + (size_t)b * FF * C * 2;
    uint8_t* mk = a.mask ? a.mask + (size_t)b * NPTS * (C / 8) : nullptr;
    for (int u = tid; u < NPTS * 16; u += NT) {
      const int p = u >> 4, q = u & 15;
      const uint4 v = *(const uint4*)(stg + p * 256 + ((q ^ (p & 15)) * 16));
      const int hh = p / BOARD, w = p - (p / BOARD) * BOARD;
      const int f = (hh + 1) * F + (w + 1);
      *(uint4*)(Yb + ((size_t)f * C + h * 128 + q * 8) * 2) = v;
      if (EPI == EPI_FWD && mk) {
        const uint32_t mm = (((v.x + 0x7fff7fffu) >> 15) & 0x10001u) |
                            (((v.y + 0x7fff7fffu) >> 13) & 0x40004u) |
                            (((v.z + 0x7fff7fffu) >> 11) & 0x100010u) |
                            (((v.w + 0x7fff7fffu) >> 9) & 0x400040u);
        mk[(size_t)p * (C / 8) + h * 16 + q] = (uint8_t)(mm | (mm >> 15));
      }
    }
    // staging reads done (LDS only) before the next item's chunk-1 DMA into buffer 1; the
    // global stores keep draining under the next item's MFMAs
    lds_barrier();
    staged = pf_next;
  }
  if constexpr (HEAD) {
    __builtin_amdgcn_s_waitcnt(0x0F70);   // this workgroup's last-layer stores retired
    __syncthreads();
    dghead::head_from_frame<256>(m.head, b, smem);
  }
}

template <int EPI, int BPF, bool HEAD = false>
hipError_t launch_layer2_multi(const MultiArgs& m, int B, hipStream_t stream) {
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_layer2_multi_kernel<EPI, BPF, HEAD>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MULTI);
    done = true;
  }
  hipLaunchKernelGGL((conv_layer2_multi_kernel<EPI, BPF, HEAD>), dim3(B), dim3(NT), LDS_MULTI,
                     stream, m);
  return hipGetLastError();
}

// BPF = 1 (the only instantiation): the K loop reads k-half 1's B fragments before k-half
// 0's MFMAs (+0.5% at 12x256 over no read-ahead, which round 3 removed).  (Also reading the
// next step's k-half 0 under k-half 1's MFMAs, 242-252 VGPRs, measured -4.5%:
// profiles/r2_layer2_multi_ab.txt.)

}  // namespace

extern "C" {

// epi 1: forward (pbias required, mask written if given); 2: backward-data (mask of the
// layer below required).  C = 256 (128 works too: 2 chunks, one workgroup per board).
hipError_t dg_conv_layer2(int epi, const void* A, const void* pbias, const void* X, void* Y,
                          void* mask, int C, int B, hipStream_t stream) {
  if ((C != 128 && C != 256) || B <= 0 || !A || !X || !Y) return hipErrorInvalidValue;
  if (epi == EPI_FWD && !pbias) return hipErrorInvalidValue;
  if (epi == EPI_DGRAD && !mask) return hipErrorInvalidValue;
  LayerArgs a{(const char*)A, (const bf16_t*)pbias, (const char*)X, (char*)Y, (uint8_t*)mask, C};
  if (epi == EPI_FWD) return launch_layer2<EPI_FWD>(a, B, stream);
  if (epi == EPI_DGRAD) return launch_layer2<EPI_DGRAD>(a, B, stream);
  return hipErrorInvalidValue;
}

// nl layers in one launch: table = nl rows of {A, pbias, X, Y, mask} (int64); row l + 1's X
// must be row l's Y (checked).  C = 256 | 128 as above.  head (forward, C = 256 only, or
// null): the fused policy head on the last Y (head->X is set here).
static hipError_t layer2_multi(int epi, const long long* table, int nl, int C, int B,
                               const dghead::HeadMArgs* head, hipStream_t stream) {
  if ((C != 128 && C != 256) || B <= 0 || nl <= 0 || nl > MAXL2) return hipErrorInvalidValue;
  if (head && (epi != EPI_FWD || C != 256 || !head->dZ || !head->gw_part || !head->dzb))
    return hipErrorInvalidValue;
  MultiArgs m{};
  m.nl = nl;
  for (int i = 0; i < nl; ++i) {
    const long long* t = table + 5 * i;
    LayerArgs& a = m.L[i];
    a = LayerArgs{(const char*)t[0], (const bf16_t*)t[1], (const char*)t[2], (char*)t[3],
                  (uint8_t*)t[4], C};
    if (!a.A || !a.X || !a.Y) return hipErrorInvalidValue;
    if (epi == EPI_FWD && !a.pbias) return hipErrorInvalidValue;
    if (epi == EPI_DGRAD && !a.mask) return hipErrorInvalidValue;
    if (i > 0 && a.X != m.L[i - 1].Y) return hipErrorInvalidValue;
  }
  if (head) {
    m.head = *head;
    m.head.X = m.L[nl - 1].Y;
    return launch_layer2_multi<EPI_FWD, 1, true>(m, B, stream);
  }
  if (epi == EPI_FWD) return launch_layer2_multi<EPI_FWD, 1>(m, B, stream);
  if (epi == EPI_DGRAD) return launch_layer2_multi<EPI_DGRAD, 1>(m, B, stream);
  return hipErrorInvalidValue;
}

hipError_t dg_conv_layer2_multi(int epi, const long long* table, int nl, int C, int B,
                                hipStream_t stream) {
  return layer2_multi(epi, table, nl, C, B, nullptr, stream);
}

// the forward run + the fused policy head (3x3 / 256-channel head on the run's last output)
hipError_t dg_conv_layer2_multi_head(const long long* table, int nl, int B, const float* w,
                                     const float* bias, const float* posb, const int* labels,
                                     float* loss, int* pred, void* dZ, float* gw_part,
                                     float* dzb, int head_relu, float grad_scale,
                                     hipStream_t stream) {
  const dghead::HeadMArgs h{nullptr, w, bias, posb, labels, loss, pred, nullptr, (char*)dZ,
                            gw_part, dzb, head_relu, grad_scale};
  return layer2_multi(EPI_FWD, table, nl, 256, B, &h, stream);
}

}  // extern "C"
