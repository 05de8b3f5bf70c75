// Board-resident first layer: the k x k (5 x 5) convolution over the expanded input planes
// (37 planes padded to 40 channels), bias + untied position bias + ReLU, one board x 128
// output channels per workgroup.
//
// The pixel-tiled im2col kernel (conv_mfma.hip conv_nt_kernel) re-stages every pixel's
// 5x5x40 patch per tile: 40 KB of LDS-DMA per 192 MFMAs (213 B/MFMA) for a K of only 1000,
// ~25% of the MFMA rate.  Here the board's whole zero-bordered 23x23x40 input frame (42 KB)
// is staged ONCE by a linear LDS-DMA copy, and every B fragment is read straight out of it:
// the K axis is the 125 8-channel chunks (tap, c8) of the layer — a lane's 8 K values are
// one chunk, so a 32-wide K step may mix taps freely (padded to 128 chunks: K = 1024, 2.4%
// waste instead of the 60% of a 64-channel image).  The weights [128 co][64 k] stream
// through a 3-deep LDS ring by inline-asm LDS-DMA two steps ahead (conv_stack's scheme).
//
// 8 waves: 2 (64 co) x 4 (96 px, 6 fragments of 16); v_mfma_f32_16x16x32_bf16.
// Reference: layer 1 of getBasicModel (experiments.lua:137-147: SpatialZeroPadding(2),
// SpatialConvolutionMM(37 -> d, 5x5), Add (per-position bias), ReLU).
#include <stdlib.h>

#include "dg_common.h"
#include "dg_features.h"

using namespace dg;

namespace {

constexpr int BM = 128;
constexpr int A_BYTES = BM * 128;  // [128 co][64 k] bf16
constexpr int MF = 4, NF = 6;

struct L1Args {
  const bf16_t* A;     // [Mpad][KP] weights, k = tap * x_C + c (conv_nt layout)
  const char* X;       // input frame [B][F][F][x_C] bf16, F = 19 + 2 * pad
  char* Y;             // output frame [B][19 + 2 y_pad]^2[M] bf16
  const float* bias;   // [M]
  const float* posb;   // [361][M]
  int KP, M, x_C, y_pad, B;
  int ngroups;         // valid chunks = KW * KW * x_C / 8
  int img_bytes;       // LDS image bytes (whole KB)
  uint8_t* mask;       // optional ReLU bitmask [B][361][M/8] (bit k of byte q: channel 8q+k
                       // nonzero) — lets the backward-data stack reach layer 1
  const bf16_t* pbias; // optional: bf16(bias + posb) [361][M] in place of bias / posb (the
                       // other forward epilogues' table: the same values as the forward
                       // stack's fused first layer)
};

// NW = 8: one workgroup (board x 128 co) per CU, 3-deep weight ring.  NW = 4: a workgroup
// computes half the board's pixels (the whole input frame is still staged), 2-deep ring,
// 74 KB of LDS: two independent workgroups per CU, so one's frame load / epilogue overlaps
// the other's MFMAs.
template <int KW, int NW>
__global__ void __launch_bounds__(64 * NW, 8 / NW) conv_l1_kernel(L1Args a) {
  constexpr int R = (KW - 1) / 2;
  constexpr int F = BOARD + 2 * R;
  constexpr int NRING = NW == 8 ? 3 : 2;
  constexpr int DPW = 16 / NW;          // weight-tile DMA instructions per wave
  constexpr int WN = NW / 2;            // pixel groups (96 px each) per workgroup
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int b = blockIdx.x / (8 / NW);
  const int px0 = (blockIdx.x % (8 / NW)) * WN * 96 + wn * 96;
  const int m_tile = blockIdx.y * BM;
  char* img = smem;
  char* ring = smem + a.img_bytes;
  const uint32_t ring_u = (uint32_t)(uintptr_t)(LDS_AS char*)ring;
  const int xcb = a.x_C * 2;
  const int KS = a.KP / 64;

  // weight tile of K-step s -> ring slot s % NRING: DPW LDS-DMA instructions per wave
  const int g_src = (lane & 7) ^ (lane >> 3);
  const char* a_lane = (const char*)a.A +
                       ((size_t)(m_tile + wave * DPW * 8 + (lane >> 3)) * a.KP + g_src * 8) * 2;
  auto stage_A = [&](int s) {
    const char* src = a_lane + s * 128;
    const uint32_t dst = ring_u + (s % NRING) * A_BYTES + wave * DPW * 1024;
#pragma unroll
    for (int i = 0; i < DPW; ++i)
      dma16(src + (size_t)i * 8 * a.KP * 2, __builtin_amdgcn_readfirstlane(dst + i * 1024));
  };

  // ---- prologue: the board's input frame, a linear copy (whole 1-KB blocks; the tail
  // of the last block re-reads the frame's last 16 B into the image padding) ----
  {
    const int fbytes = F * F * xcb;
    const char* Xb = a.X + (size_t)b * fbytes;
    for (int blk = wave; blk < a.img_bytes / 1024; blk += NW) {
      int off = blk * 1024 + lane * 16;
      const int src = off < fbytes ? off : fbytes - 16;
      glds16(Xb + src, (LDS_AS void*)(img + blk * 1024));
    }
    stage_A(0);
    if (NRING == 3 && KS > 1) stage_A(1);
  }
  dma_wait<0>();
  __syncthreads();

  const int lr = lane & 15, lq = lane >> 4;
  int fpb[NF];  // byte offset of this lane's pixel (centre) in the image
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = px0 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    fpb[j] = ((h + R) * F + (w + R)) * xcb;
  }
  const int gpt = a.x_C / 8;

  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = 0; s < KS; ++s) {
    if (s + NRING - 1 < KS) stage_A(s + NRING - 1);
    const char* sA = ring + (s % NRING) * A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      // this lane's K chunk: (tap, c8) -> byte offset relative to the pixel centre
      int kc = s * 8 + kk * 4 + lq;
      if (kc >= a.ngroups) kc = 0;  // padding chunks: zero weights, any finite image value
      const int t = kc / gpt, c8 = kc - t * gpt;
      const int dy = t / KW - R, dx = t - (t / KW) * KW - R;
      const int koff = (dy * F + dx) * xcb + c8 * 16;
      const int g = kk * 4 + lq;
      bf16x8 af[MF], bfr[NF];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int row = wm * 64 + i * 16 + lr;
        af[i] = lds_read_b128((const LDS_AS char*)(sA + row * 128 + ((g ^ (row & 7)) * 16)));
      }
#pragma unroll
      for (int j = 0; j < NF; ++j)
        bfr[j] = lds_read_b128((const LDS_AS char*)(img + fpb[j] + koff));
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    // tile s+1 landed for this wave (with a 3-deep ring tile s+2 may stay in flight), then
    // for all waves
    if (NRING == 3 && s + 2 < KS) dma_wait<DPW>(); else dma_wait<0>();
    __builtin_amdgcn_s_barrier();
  }

  // ---- epilogue: + bias + position bias, ReLU, bf16 -> output frame ----
  // (no divergent exits before the mask shuffle: every lane computes, stores are guarded)
  const int yF = BOARD + 2 * a.y_pad;
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int co = m_tile + wm * 64 + i * 16 + lq * 4;
    const bool co_ok = co < a.M;
    const int coc = co_ok ? co : 0;
    const f32x4 bv = a.pbias ? f32x4{0.f, 0.f, 0.f, 0.f} : *(const f32x4*)(a.bias + coc);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = px0 + j * 16 + lr;
      const bool ok = co_ok && p < NPTS;
      const int pc = p < NPTS ? p : 0;
      f32x4 v = acc[i][j];
      if (a.pbias) {
        const uint2 u = *(const uint2*)(a.pbias + (size_t)pc * a.M + coc);
        v[0] = fmaxf(v[0] + __uint_as_float(u.x << 16), 0.f);
        v[1] = fmaxf(v[1] + __uint_as_float(u.x & 0xFFFF0000u), 0.f);
        v[2] = fmaxf(v[2] + __uint_as_float(u.y << 16), 0.f);
        v[3] = fmaxf(v[3] + __uint_as_float(u.y & 0xFFFF0000u), 0.f);
      } else {
        const f32x4 pv = *(const f32x4*)(a.posb + (size_t)pc * a.M + coc);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + bv[r] + pv[r], 0.f);
      }
      uint2 o;
      o.x = pack_bf16x2(v[0], v[1]);
      o.y = pack_bf16x2(v[2], v[3]);
      if (a.mask) {
        // lanes l and l ^ 16 hold channels co..co+3 and co+4..co+7 of one pixel: one byte
        const uint32_t nib = ((o.x & 0xFFFFu) ? 1u : 0u) | ((o.x >> 16) ? 2u : 0u) |
                             ((o.y & 0xFFFFu) ? 4u : 0u) | ((o.y >> 16) ? 8u : 0u);
        const uint32_t hi = (uint32_t)__shfl_xor((int)nib, 16, 64);
        if (ok && !(lq & 1))
          a.mask[((size_t)b * NPTS + p) * (a.M >> 3) + (co >> 3)] = (uint8_t)(nib | (hi << 4));
      }
      if (ok) {
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
        const size_t yo = (((size_t)b * yF + h + a.y_pad) * yF + (w + a.y_pad)) * a.M + co;
        *(uint2*)(a.Y + yo * 2) = o;
      }
    }
  }
}

template <int KW, int NW>
hipError_t launch_l1(const L1Args& a, int Mpad, hipStream_t stream) {
  const size_t lds = (size_t)a.img_bytes + (NW == 8 ? 3 : 2) * A_BYTES;
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_l1_kernel<KW, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL((conv_l1_kernel<KW, NW>), dim3(a.B * (8 / NW), Mpad / BM), dim3(64 * NW),
                     lds, stream, a);
  return hipGetLastError();
}


// ---- the 5x5 / 40-channel first layer on the forward stack's K loop (conv_l1_frag) ----
// The generic kernel above stages the weights through an LDS ring (one barrier per K-step)
// and reads the input frame in its linear 80-B-per-pixel layout (4.6M LDS bank-conflict
// cycles per launch at d = 256, 26% MFMA busy; profiles/r2_s4_pmc_12x256.txt).  This one
// is conv_stack2.hip's fused-first-layer scheme as a kernel of its own, for the shapes the
// stack cannot take (d = 256, fp8 models):
//   * one workgroup (8 waves) per board; the 23x23x40 frame is gathered ONCE into the
//     conflict-free plane layout cell(c8, y, x) = c8 * 816 + 35 y + x (16-B cells) and serves
//     every 128-channel output pass (h loop), so a board's frame is staged once instead of
//     once per (half board, 128 channels) workgroup;
//   * the weights stream from L2 into VGPRs in fragment order ([h][16 steps][2][2][4][64] x
//     8 bf16, written by weight_refresh), half a K-step ahead, with no barrier in the K loop;
//   * the epilogue adds the stack-order bias table (bf16 bias + position bias), applies
//     ReLU and stores straight from the accumulators (four 32-B pieces of a pixel's 64
//     channels back to back), plus the ReLU bitmask the backward-data chain reads.
constexpr int PF_RP = 35, PF_PS = 816, PF_CELLS = 5 * PF_PS;  // conv_stack2.hip L1RP / L1PS
constexpr int PF_F = 23, PF_XB = 80, PF_BYTES = PF_F * PF_F * PF_XB;
constexpr int PF_STEPS = 16, PF_CHUNKS = 125;
constexpr int PF_STEP_BYTES = 2 * 2 * MF * 64 * 16;   // 16 KB per K-step and 128-co pass
constexpr int PF_LDS = (PF_CELLS + 63) / 64 * 1024;   // whole 1-KB DMA blocks (65,536 B)

struct L1FragArgs {
  const char* A;          // fragment-ordered weights, nh passes of 16 x 16 KB
  const uint2* pbias;     // stack-order bf16 (bias + pos-bias): [h][24][2][4][64] x 4 bf16
  char* X;                // input frame [B][23][23][40] bf16 (written when in_planes is set)
  char* Y;                // output frame [B][21][21][M] bf16 (interior written)
  uint8_t* mask;          // optional ReLU bits [B][361][M/8]
  int M, nh;
  // optional: the feature expansion fused into the prologue — the staged planes are built from
  // the packed uint8 batch and the expanded frame X is written for the layer's weight gradient
  const uint8_t* in_planes;   // [B][9][361]
  const uint8_t* in_player;   // [B]
  const uint8_t* in_rank;     // [B]
};

// NFX = 6: one workgroup per board (4 x 96 pixels).  (NFX = 3, two half-board workgroups per
// board and two per CU, measured neutral in the step and was removed in round 6:
// profiles/r5_l1_half_ab.txt)
template <int NFX>
__global__ void __launch_bounds__(512, NFX == 6 ? 1 : 2) conv_l1_frag_kernel(L1FragArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int b = NFX == 6 ? blockIdx.x : blockIdx.x >> 1;
  const int f0 = NFX == 6 ? 0 : (blockIdx.x & 1) * 4 * NFX;   // first pixel fragment

  if (a.in_planes) {
    // fused expansion (dg_features.h, as expand_features): border pixels zero, interior
    // pixels also written to the expanded frame X (its border is zero from allocation)
    const uint8_t* plb = a.in_planes + (size_t)b * 9 * NPTS;
    const int pi = a.in_player[b], rk = a.in_rank[b];
    char* Xw = a.X + (size_t)b * PF_BYTES;
    for (int f = tid; f < PF_F * PF_F; f += 512) {
      const int y = f / PF_F, x = f - (f / PF_F) * PF_F;
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
          if (f0 == 0) *(uint4*)(Xw + f * PF_XB + c8 * 16) = cell[c8];
        }
      }
#pragma unroll
      for (int c8 = 0; c8 < 5; ++c8)
        *(uint4*)(smem + (c8 * PF_PS + y * PF_RP + x) * 16) = cell[c8];
    }
  } else {
    // gather: cell -> (chunk, frame row, column); padding cells re-read pixel 0 (never used)
    const char* Xb = a.X + (size_t)b * PF_BYTES;
    for (int blk = wave; blk < PF_LDS / 1024; blk += 8) {
      const int cell = blk * 64 + lane;
      const int c8 = cell / PF_PS, rem = cell - c8 * PF_PS;
      const int y = rem / PF_RP, x = rem - y * PF_RP;
      const int off = (c8 < 5 && y < PF_F && x < PF_F) ? (y * PF_F + x) * PF_XB + c8 * 16 : 0;
      glds16(Xb + off, (LDS_AS void*)(smem + blk * 1024));
    }
  }
  const int lr = lane & 15, lq = lane >> 4;
  int pbase[NFX];   // this lane's pixel centre in the plane layout (bytes)
#pragma unroll
  for (int j = 0; j < NFX; ++j) {
    int p = (f0 + wn * NFX + j) * 16 + lr;
    if (p >= NPTS) p = 0;
    const int hh = p / BOARD, w = p - (p / BOARD) * BOARD;
    pbase[j] = ((hh + 2) * PF_RP + (w + 2)) * 16;
  }
  const uint32_t a_lane = (uint32_t)(wm * (PF_STEP_BYTES / 2) + lane * 16);
  auto load_A = [&](const char* A, int kk, bf16x8 (&r)[MF]) {
    const char* p = A + a_lane + kk * MF * 1024;
#pragma unroll
    for (int i = 0; i < MF; ++i) r[i] = *(const bf16x8*)(p + i * 1024);
  };
  auto read_B = [&](int s, int kk, bf16x8 (&bfr)[NFX]) {
    int kc = s * 8 + kk * 4 + lq;          // this lane group's (tap, c8) chunk
    if (kc >= PF_CHUNKS) kc = 0;           // padding chunks: zero weights
    const int t = kc / 5, c8 = kc - (kc / 5) * 5;
    const int koff = (c8 * PF_PS + (t / 5 - 2) * PF_RP + (t % 5 - 2)) * 16;
#pragma unroll
    for (int j = 0; j < NFX; ++j)
      bfr[j] = lds_read_b128((const LDS_AS char*)(smem + pbase[j] + koff));
  };
  __syncthreads();   // frame landed

  bf16x8 Ak[2][MF];
  load_A(a.A, 0, Ak[0]);
  load_A(a.A, 1, Ak[1]);
  for (int h = 0; h < a.nh; ++h) {
    const char* Ah = a.A + (size_t)h * PF_STEPS * PF_STEP_BYTES;
    const char* A_next = h + 1 < a.nh ? Ah + PF_STEPS * PF_STEP_BYTES : Ah;
    f32x4 acc[MF][NFX];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NFX; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int s = 0; s < PF_STEPS; ++s) {
      // (past the last step of the last pass: a harmless re-load of its step 0)
      const char* An = s + 1 < PF_STEPS ? Ah + (s + 1) * PF_STEP_BYTES : A_next;
      bf16x8 bfr[NFX];
      read_B(s, 0, bfr);
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NFX; ++j) acc[i][j] = mfma16(Ak[0][i], bfr[j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      load_A(An, 0, Ak[0]);
      read_B(s, 1, bfr);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NFX; ++j) acc[i][j] = mfma16(Ak[1][i], bfr[j], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
      load_A(An, 1, Ak[1]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // epilogue: + bias table, ReLU, bf16 -> output frame (interior), ReLU bits
    int z0 = 0;
    asm volatile("" : "+v"(z0));
#pragma unroll
    for (int j = 0; j < NFX; ++j) {
      const int p = (f0 + wn * NFX + j) * 16 + lr;
      const int pc = p < NPTS ? p : NPTS - 1;
      const int hh = pc / BOARD, w = pc - (pc / BOARD) * BOARD;
      const uint2* pf = a.pbias + (((size_t)(h * 24 + f0 + wn * NFX + j) * 2 + wm) * 4) * 64 + lane + z0;
      char* yrow = a.Y + (((size_t)b * 21 + hh + 1) * 21 + (w + 1)) * a.M * 2;
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const uint2 eb = pf[i * 64];
        const f32x4 v = acc[i][j];
        const float y0 = fmaxf(v[0] + __uint_as_float(eb.x << 16), 0.f);
        const float y1 = fmaxf(v[1] + __uint_as_float(eb.x & 0xFFFF0000u), 0.f);
        const float y2 = fmaxf(v[2] + __uint_as_float(eb.y << 16), 0.f);
        const float y3 = fmaxf(v[3] + __uint_as_float(eb.y & 0xFFFF0000u), 0.f);
        uint2 o;
        o.x = pack_bf16x2(y0, y1);
        o.y = pack_bf16x2(y2, y3);
        const int co = h * 128 + wm * 64 + i * 16 + lq * 4;
        if (a.mask) {
          // lanes l and l ^ 16 hold channels co..co+3 / co+4..co+7 of one pixel: one byte
          const uint32_t nib = ((o.x & 0xFFFFu) ? 1u : 0u) | ((o.x >> 16) ? 2u : 0u) |
                               ((o.y & 0xFFFFu) ? 4u : 0u) | ((o.y >> 16) ? 8u : 0u);
          const uint32_t hi = (uint32_t)__shfl_xor((int)nib, 16, 64);
          if (p < NPTS && !(lq & 1))
            a.mask[((size_t)b * NPTS + p) * (a.M >> 3) + (co >> 3)] = (uint8_t)(nib | (hi << 4));
        }
        if (p < NPTS) *(uint2*)(yrow + co * 2) = o;
      }
    }
  }
}

}  // namespace

extern "C" {

// Usable for: 3x3 / 5x5, pad (k-1)/2 input frame with x_C <= 64 channels (multiple of 8),
// output channels padded to 128, K padded to 64 with zero weights.
int dg_conv_l1_ok(int kw, int x_pad, int x_C, int Mpad, int KP) {
  if (!(kw == 3 || kw == 5) || x_pad != (kw - 1) / 2 || x_C % 8 != 0 || x_C > 64 ||
      Mpad % BM != 0 || KP % 64 != 0 || KP < kw * kw * x_C)
    return 0;
  const int F = BOARD + 2 * x_pad;
  const int img = (F * F * x_C * 2 + 1023) / 1024 * 1024;
  return img + 3 * A_BYTES <= 160 * 1024 ? 1 : 0;
}

hipError_t dg_conv_l1(int kw, const void* A, int KP, int M, int Mpad, const void* X, int x_pad,
                      int x_C, int B, void* Y, int y_pad, const float* bias, const float* posb,
                      void* mask, const void* pbias, hipStream_t stream) {
  if (!dg_conv_l1_ok(kw, x_pad, x_C, Mpad, KP) || B <= 0 || M % 4 != 0 || M > Mpad ||
      (mask && M % 8 != 0))
    return hipErrorInvalidValue;
  const int F = BOARD + 2 * x_pad;
  L1Args a{(const bf16_t*)A, (const char*)X, (char*)Y, bias, posb, KP, M, x_C, y_pad, B,
           kw * kw * x_C / 8, (F * F * x_C * 2 + 1023) / 1024 * 1024, (uint8_t*)mask,
           (const bf16_t*)pbias};
  if (!pbias && (!bias || !posb)) return hipErrorInvalidValue;
  // 4-wave half-board workgroups when two fit on a CU
  const bool w4 = 2 * (a.img_bytes + 2 * A_BYTES) <= 160 * 1024;
  if (kw == 5) return w4 ? launch_l1<5, 4>(a, Mpad, stream) : launch_l1<5, 8>(a, Mpad, stream);
  return w4 ? launch_l1<3, 4>(a, Mpad, stream) : launch_l1<3, 8>(a, Mpad, stream);
}


// conv_l1_frag: 5x5 over the [B][23][23][40] input frame -> [B][21][21][M] (pad 1), M a
// multiple of 128; A = weight_refresh's fragment-ordered first-layer operand, pbias = its
// stack-order bias table; mask optional.
int dg_conv_l1_frag_ok(int kw, int x_pad, int x_C, int M, int y_pad) {
  return kw == 5 && x_pad == 2 && x_C == 40 && M % 128 == 0 && M <= 512 && y_pad == 1;
}

hipError_t dg_conv_l1_frag(const void* A, const void* pbias, void* X, int B, int M,
                           void* Y, void* mask, const void* planes, const void* player,
                           const void* rank, hipStream_t stream) {
  if (planes && (!player || !rank)) return hipErrorInvalidValue;
  if (!A || !pbias || !X || !Y || B <= 0 || M % 128 != 0 || M > 512)
    return hipErrorInvalidValue;
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_l1_frag_kernel<6>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, PF_LDS);
    done = true;
  }
  L1FragArgs a{(const char*)A, (const uint2*)pbias, (char*)X, (char*)Y, (uint8_t*)mask, M,
               M / 128, (const uint8_t*)planes, (const uint8_t*)player, (const uint8_t*)rank};
  hipLaunchKernelGGL(conv_l1_frag_kernel<6>, dim3(B), dim3(512), PF_LDS, stream, a);
  return hipGetLastError();
}

}  // extern "C"
