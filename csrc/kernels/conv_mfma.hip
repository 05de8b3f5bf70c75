// Implicit-GEMM 19x19 convolutions on CDNA4 MFMA (bf16 in, fp32 accumulate).
//
// Replaces the reference's nn.SpatialZeroPadding + nn.SpatialConvolutionMM (+ nn.Add +
// nn.ReLU) stack (experiments.lua:137-147; im2col + cuBLAS SGEMM in cunn, EXTERNAL).
//
// Design (MI355X-first, not a port):
//  * Activations live in zero-bordered NHWC frames [B][19+2p][19+2p][C] (bf16), so a
//    conv tap is a constant byte offset from the output pixel's centre and halo loads
//    need no predicates (zero padding = the frame border, written once, never touched).
//  * The GEMM N dimension is the flattened valid pixel index n = b*361 + h*19 + w
//    (no frame-border compute waste); every lane computes its own pixel's frame offset,
//    so im2col is implicit in the per-lane SOURCE address of global_load_lds_dwordx4.
//  * K = (tap, channel) in 8-channel (16 B) groups.  LDS tiles are lane-linear 128-B rows
//    (64 k) with an XOR swizzle applied on the source side (slot ^= row&7): conflict-free
//    ds_read_b128 for the 16x16x32 fragment pattern (checked with tools/lds_banks.py).
//  * conv_nt_kernel: D[co][n] = sum_k W[co][k] * im2col(X)[n][k]  (forward and dgrad).
//      EPI_FWD   : + bias[co] + pos_bias[p][co], ReLU, bf16 store into the output frame.
//      EPI_DGRAD : * (aux_activation > 0)  (ReLU backward fused), bf16 store.
//      EPI_LINEAR: plain store (tests).
//  * conv_wgrad_kernel: dW[co][k] = sum_n dZ[n][co] * im2col(X)[n][k] with split-K over
//    pixels into fp32 slabs; both operands are staged pixel-major and read with the
//    CDNA4 transposing LDS read ds_read_b64_tr_b16.
#include <stdlib.h>

#include "dg_common.h"

using namespace dg;

namespace {

constexpr int EPI_LINEAR = 0;
constexpr int EPI_FWD = 1;
constexpr int EPI_DGRAD = 2;

struct ConvNTArgs {
  const bf16_t* A;     // [Mpad][KP] bf16 weights (K contiguous)
  const char* X;       // input frame (bytes)
  char* Y;             // output frame (bytes)
  const float* bias;   // [M]           (EPI_FWD)
  const float* posb;   // [361][M]      (EPI_FWD)
  const char* aux;     // mask frame    (EPI_DGRAD), channels = M
  int KP;              // padded K (multiple of 64)
  int M;               // real output channels
  int Npix;            // B*361
  int x_pad, x_C;      // input frame pad and channels (multiple of 8)
  int y_pad;           // output frame pad (channels = M)
  int aux_pad;
  int ngroups;         // valid k-groups = KW*KW*x_C/8
  int gpt;             // k-groups per tap = x_C/8
  uint64_t gpt_magic;  // fastdiv magic for gpt
  uint8_t* mask;       // EPI_FWD (optional): ReLU bitmask [Npix][M/8], bit k = channel 8q+k
};

// Byte offset (relative to the pixel centre) of k-group kg.
template <int KW>
DG_DEV int koff_of(int kg, const ConvNTArgs& a) {
  if (kg >= a.ngroups) return 0;
  const int t = (int)fastdiv((uint32_t)kg, a.gpt_magic);
  const int c8 = kg - t * a.gpt;
  constexpr int R = (KW - 1) / 2;
  const int dh = t / KW - R;
  const int dw = t % KW - R;
  const int F = BOARD + 2 * a.x_pad;
  return ((dh * F + dw) * a.x_C + c8 * 8) * 2;
}

// MF: 16-row fragments per wave along M (BM = 2*16*MF); NF: along N (BN = 2*16*NF).
template <int KW, int MF, int NF, int EPI>
__global__ void __launch_bounds__(256)
conv_nt_kernel(ConvNTArgs a) {
  constexpr int BM = 32 * MF;
  constexpr int BN = 32 * NF;
  constexpr int A_BYTES = BM * 128;
  constexpr int B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int A_INSTR = BM / 32;  // glds per wave per K-step (BM rows / 8 rows / 4 waves)
  constexpr int B_INSTR = BN / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int n_tile = blockIdx.x * BN;
  const int m_tile = blockIdx.y * BM;

  // ---- per-lane staging constants ----
  const int g_src = (lane & 7) ^ (lane >> 3);   // k-group this lane fetches (source swizzle)
  const int row_in_instr = lane >> 3;
  uint32_t pix_off[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int r = (wave * B_INSTR + i) * 8 + row_in_instr;
    int n = n_tile + r;
    if (n >= a.Npix) n = 0;
    pix_off[i] = pixel_frame_off(n, a.x_pad, a.x_C);
  }
  const char* a_row[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int r = (wave * A_INSTR + i) * 8 + row_in_instr;
    a_row[i] = (const char*)a.A + (size_t)(m_tile + r) * a.KP * 2 + g_src * 16;
  }

  auto stage = [&](int buf, int ks) {
    char* sA = smem + buf * STAGE;
    char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i)
      glds16(a_row[i] + ks * 128, (LDS_AS void*)(sA + (wave * A_INSTR + i) * 1024));
    const int ko = koff_of<KW>(ks * 8 + g_src, a);
#pragma unroll
    for (int i = 0; i < B_INSTR; ++i)
      glds16(a.X + (int)pix_off[i] + ko, (LDS_AS void*)(sB + (wave * B_INSTR + i) * 1024));
  };

  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.KP / 64;
  stage(0, 0);
  __syncthreads();

  const int lr = lane & 15;
  const int lq = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) stage(buf ^ 1, ks + 1);
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int slot = ((kk * 4 + lq) ^ (lane & 7)) * 16;
      bf16x8 af[MF], bfr[NF];
#pragma unroll
      for (int i = 0; i < MF; ++i)
        af[i] = lds_read_b128((const LDS_AS char*)(sA + (wm * MF * 16 + i * 16 + lr) * 128 + slot));
#pragma unroll
      for (int j = 0; j < NF; ++j)
        bfr[j] = lds_read_b128((const LDS_AS char*)(sB + (wn * NF * 16 + j * 16 + lr) * 128 + slot));
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    __syncthreads();
  }

  // ---- epilogue ----
  // all global loads (bias / pos_bias / ReLU mask) issued before any use (see conv_board)
  const int y_C = a.M;
  int pb_[NF], bb_[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int n = n_tile + wn * NF * 16 + j * 16 + lr;
    const int nn = n < a.Npix ? n : 0;
    bb_[j] = nn / NPTS;
    pb_[j] = n < a.Npix ? nn - bb_[j] * NPTS : -1;
  }
  f32x4 bias_v[MF];
  f32x4 pos_v[NF][MF];
  uint2 mask_v[NF][MF];
#pragma unroll
  for (int i = 0; i < MF; ++i) {
    const int co = m_tile + wm * MF * 16 + i * 16 + lq * 4;
    const int coc = co < a.M ? co : 0;
    if constexpr (EPI == EPI_FWD) bias_v[i] = *(const f32x4*)(a.bias + coc);
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = pb_[j] < 0 ? 0 : pb_[j];
      if constexpr (EPI == EPI_FWD) pos_v[j][i] = *(const f32x4*)(a.posb + p * a.M + coc);
      if constexpr (EPI == EPI_DGRAD) {
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
        mask_v[j][i] = *(const uint2*)(a.aux + frame_off(bb_[j], h, w, a.aux_pad, y_C) + coc * 2);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    if constexpr (EPI == EPI_FWD) {
      // ReLU bitmask (what the board dgrad / dgrad stack gate with): lanes l and l ^ 16
      // hold channels co..co+3 and co+4..co+7 of the same pixel -> one byte; computed by
      // every lane before the divergent stores below (the shuffle needs them all)
      if (a.mask) {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int co = m_tile + wm * MF * 16 + i * 16 + lq * 4;
          const int coc = co < a.M ? co : 0;
          uint32_t nib = 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float y = fmaxf(acc[i][j][r] + bias_v[i][r] + pos_v[j][i][r], 0.f);
            nib |= (f2bf(y) != 0 ? 1u : 0u) << r;
          }
          const uint32_t hi = (uint32_t)__shfl_xor((int)nib, 16, 64);
          if (!(lq & 1) && pb_[j] >= 0 && co < a.M)
            a.mask[(size_t)(bb_[j] * NPTS + pb_[j]) * (a.M >> 3) + (coc >> 3)] =
                (uint8_t)(nib | (hi << 4));
        }
      }
    }
    if (pb_[j] < 0) continue;
    const int b = bb_[j];
    const int p = pb_[j];
    const int h = p / BOARD;
    const int w = p - h * BOARD;
    const uint32_t yo = frame_off(b, h, w, a.y_pad, y_C);
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int co = m_tile + wm * MF * 16 + i * 16 + lq * 4;
      if (co >= a.M) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI == EPI_FWD) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r] + bias_v[i][r] + pos_v[j][i][r], 0.f);
      } else if constexpr (EPI == EPI_DGRAD) {
        const uint2 m = mask_v[j][i];
        if ((m.x & 0xFFFFu) == 0 || (m.x & 0x8000u)) v[0] = 0.f;
        if ((m.x >> 16) == 0 || (m.x & 0x80000000u)) v[1] = 0.f;
        if ((m.y & 0xFFFFu) == 0 || (m.y & 0x8000u)) v[2] = 0.f;
        if ((m.y >> 16) == 0 || (m.y & 0x80000000u)) v[3] = 0.f;
      }
      uint2 o;
      o.x = pack_bf16x2(v[0], v[1]);
      o.y = pack_bf16x2(v[2], v[3]);
      *(uint2*)(a.Y + yo + co * 2) = o;
    }
  }
}

// ------------------------------------------------------------------------------------
// Weight gradient: dW[co][k] = sum_n dZ[n][co] * im2col(X)[n][k]
// Tile: BM co x BN k per workgroup, 4 waves (2x2), each 64x64 (4x4 fragments).
// Reduction over pixels in steps of 64, split across blockIdx.z into fp32 slabs
// slab[z][co][k] (co < Mpad, k < KP).
struct WgradArgs {
  const char* dZ;   // gradient frame, channels = M
  const char* X;    // input frame of the layer
  float* slab;      // [splits][Mpad][KP]
  int dz_pad;
  int M, Mpad;      // output channels (real, padded to 128)
  int KP;           // padded K (multiple of 128)
  int Npix;
  int px_per_split; // multiple of 64
  int x_pad, x_C;
  int ngroups, gpt;
  uint64_t gpt_magic;
  int ablate;  // diagnostics: 1 no MFMA, 2 no LDS reads, 4 no DMA, 8 no slab store, 16 no barrier
  int ktiles, mtiles, splits;  // logical grid (launched flat, XCD-remapped)
  int nlayers;                 // t3 kernel: layers of identical geometry in one launch
};

// Per-layer operands of a multi-layer weight-gradient launch (conv_wgrad_t3_kernel).
constexpr int MAXWL = 16;
struct WgradLayers {
  const char* dZ[MAXWL];
  const char* X[MAXWL];
  float* slab[MAXWL];
};

DG_DEV int wg_swz(int r) { return 2 * ((r & 3) | (((r >> 3) & 1) << 2)); }

template <int KW>
DG_DEV int koff_wg(int kg, const WgradArgs& a) {
  if (kg >= a.ngroups) return 0;
  const int t = (int)fastdiv((uint32_t)kg, a.gpt_magic);
  const int c8 = kg - t * a.gpt;
  constexpr int R = (KW - 1) / 2;
  const int dh = t / KW - R;
  const int dw = t % KW - R;
  const int F = BOARD + 2 * a.x_pad;
  return ((dh * F + dw) * a.x_C + c8 * 8) * 2;
}

template <int KW>
__global__ void __launch_bounds__(256, 2)
conv_wgrad_kernel(WgradArgs a) {
  constexpr int BM = 128, BN = 128, BKN = 64;  // BKN pixels per step
  constexpr int T_BYTES = BKN * 256;           // 64 rows x 256 B
  constexpr int STAGE = 2 * T_BYTES;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware remap (cdna guide T1): hardware dispatch round-robins flat block ids over the
  // 8 XCDs (private L2 each).  Give every XCD a contiguous range of logical work items so
  // the k-tiles sharing a pixel split (same dZ rows, overlapping X rows) run together on
  // one XCD and hit its L2, instead of re-streaming from the Infinity Cache.
  const int nwg = a.ktiles * a.mtiles * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, xslot = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + xslot;
  const int kt = lid % a.ktiles;
  const int rest = lid / a.ktiles;
  const int mt = rest % a.mtiles;
  const int zsplit = rest / a.mtiles;
  const int k_tile = kt * BN;
  const int m_tile = mt * BM;
  const int n_begin = zsplit * a.px_per_split;
  int n_end = n_begin + a.px_per_split;
  if (n_end > a.Npix) n_end = a.Npix;
  const int nsteps = (n_end - n_begin + BKN - 1) / BKN;

  // staging: each wave-instruction = 4 rows x 16 slots of 16 B; 4 instr per wave per tile
  const int r_in = lane >> 4;
  const int slot = lane & 15;
  // source chunk (16 B unit along the 256-B row) for each of the 4 rows this lane fills
  int koffs[4];
  int dz_chunk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (wave * 4 + i) * 4 + r_in;  // row within tile (pixel)
    const int c = slot ^ wg_swz(r);
    dz_chunk[i] = (m_tile * 2) + c * 16;
    koffs[i] = koff_wg<KW>(k_tile / 8 + c, a);
  }

  auto stage = [&](int buf, int step) {
    if (a.ablate & 4) return;
    char* sA = smem + buf * STAGE;
    char* sB = sA + T_BYTES;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = (wave * 4 + i) * 4 + r_in;
      int n = n_begin + step * BKN + r;
      const bool ok = n < n_end;
      if (!ok) n = n_begin;  // valid address; the dZ row reads the zero border instead
      const int b = n / NPTS;
      const int p = n - b * NPTS;
      const int h = p / BOARD;
      const int w = p - h * BOARD;
      const uint32_t dzo = frame_off(b, h, w, a.dz_pad, a.M);
      const uint32_t xo = frame_off(b, h, w, a.x_pad, a.x_C);
      // out-of-range rows read the zero border (offset 0 of the frame is border) for dZ
      const char* src_dz = ok ? (a.dZ + dzo + dz_chunk[i]) : (a.dZ + (slot * 16));
      glds16(src_dz, (LDS_AS void*)(sA + (wave * 4 + i) * 1024));
      glds16(a.X + xo + koffs[i], (LDS_AS void*)(sB + (wave * 4 + i) * 1024));
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    stage(0, 0);
    __syncthreads();
  }
  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + T_BYTES;
    // all 32 transposed fragment reads of the step first (distinct registers), then the
    // 32 MFMAs: the scheduler may not interleave them back into read->wait->mfma bursts.
    s16x4 ta[2][2][4], tb[2][2][4];
    if (a.ablate & 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) ta[kk][half][i] = tb[kk][half][i] = s16x4{};
    } else
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int row = kk * 32 + 8 * g + 4 * half + q;
        const int sw = wg_swz(row);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = (wm * 64 + i * 16) / 8 + (pp >> 1);
          ta[kk][half][i] =
              lds_read_tr((const LDS_AS char*)(sA + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int c = (wn * 64 + j * 16) / 8 + (pp >> 1);
          tb[kk][half][j] =
              lds_read_tr((const LDS_AS char*)(sB + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // next step's DMA after the tr-reads (else the compiler waits vmcnt(0) before them)
    if (st + 1 < nsteps) stage(buf ^ 1, st + 1);
    __builtin_amdgcn_sched_barrier(0);
    if (a.ablate & 1) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half)
#pragma unroll
          for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(ta[kk][half][i]), "v"(tb[kk][half][i]));
    } else
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x4 lo = ta[kk][0][i], hi = ta[kk][1][i];
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const s16x4 lo = tb[kk][0][j], hi = tb[kk][1][j];
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);  // DMA wait + barrier stay below the MFMAs
    if (!(a.ablate & 16)) __syncthreads();
  }
  if (a.ablate & 8) {
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) keep += acc[i][j][0];
    if (keep == 1234.5f) a.slab[0] = keep;
    return;
  }

  // slab store: D rows = co, cols = k
  float* slab = a.slab + (size_t)zsplit * a.Mpad * a.KP;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m_tile + wm * 64 + i * 16 + g * 4 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k_tile + wn * 64 + j * 16 + li;
        slab[(size_t)co * a.KP + k] = acc[i][j][r];
      }
    }
  }
}

// The same tile and the same summation order as conv_wgrad_kernel (so bit-identical slabs),
// with a deeper LDS-DMA pipeline: 32-pixel K-steps, NS stage buffers of 16 KB (dZ 32 x 256 B
// + X 32 x 256 B) and PD = NS - 1 steps in flight, issued from inline asm (dma16) with exact
// vmcnt accounting (every wave issues exactly 4 DMAs per stage: 2 dZ + 2 X blocks of 4 rows).
// Why: the first layer's 5x5 weight gradient (K = 25 taps x 40 channels, 64 pixel splits)
// is latency-bound in conv_wgrad_kernel — one 32-KB stage in flight per workgroup, 32 MFMAs
// (~256 cycles) per wave between a DMA issue and its wait — and it sits on the step's critical
// tail after the window weight gradient in every configuration.  Each wave also reads half
// as many fragments per step (one 32-row k-half), so its registers stay below
// conv_wgrad_kernel's.
template <int KW, int NS>
__global__ void __launch_bounds__(256, 2)
conv_wgrad_pipe_kernel(WgradArgs a) {
  constexpr int BKN = 32;                      // pixels per K-step
  constexpr int T_BYTES = BKN * 256;           // 32 rows x 256 B
  constexpr int STAGE = 2 * T_BYTES;           // dZ tile + X tile: 16 KB
  constexpr int PD = NS - 1;                   // K-steps in flight beyond the current one
  static_assert(NS >= 2 && NS <= 4, "stages");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const uint32_t smem_u = (uint32_t)(uintptr_t)(LDS_AS char*)smem;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int nwg = a.ktiles * a.mtiles * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, xslot = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + xslot;
  const int kt = lid % a.ktiles;
  const int rest = lid / a.ktiles;
  const int mt = rest % a.mtiles;
  const int zsplit = rest / a.mtiles;
  const int k_tile = kt * 128;
  const int m_tile = mt * 128;
  const int n_begin = zsplit * a.px_per_split;
  int n_end = n_begin + a.px_per_split;
  if (n_end > a.Npix) n_end = a.Npix;
  const int nsteps = n_end > n_begin ? (n_end - n_begin + BKN - 1) / BKN : 0;

  // staging: a DMA instruction = 4 rows x 16 slots of 16 B; wave w fills rows (2w + i) * 4 ..
  const int r_in = lane >> 4;
  const int slot = lane & 15;
  int koffs[2], dz_chunk[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * 2 + i) * 4 + r_in;
    const int c = slot ^ wg_swz(r);
    dz_chunk[i] = (m_tile * 2) + c * 16;
    koffs[i] = koff_wg<KW>(k_tile / 8 + c, a);
  }
  auto issue = [&](int buf, int step) {
    const uint32_t base = smem_u + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * 2 + i) * 4 + r_in;
      int n = n_begin + step * BKN + r;
      const bool ok = n < n_end;
      if (!ok) n = n_begin;  // valid address; the dZ row reads the zero border instead
      const int b = n / NPTS;
      const int p = n - b * NPTS;
      const int h = p / BOARD;
      const int w = p - h * BOARD;
      const uint32_t dzo = frame_off(b, h, w, a.dz_pad, a.M);
      const uint32_t xo = frame_off(b, h, w, a.x_pad, a.x_C);
      const char* src_dz = ok ? (a.dZ + dzo + dz_chunk[i]) : (a.dZ + (slot * 16));
      const uint32_t dst = base + (wave * 2 + i) * 1024;
      dma16(src_dz, __builtin_amdgcn_readfirstlane(dst));
      dma16(a.X + xo + koffs[i], __builtin_amdgcn_readfirstlane(dst + T_BYTES));
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < nsteps) issue(p % NS, p);
  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  for (int st = 0; st < nsteps; ++st) {
    // this wave's DMAs of step st landed (those of st + 1 .. st + PD - 1 may remain), then
    // every wave's (barrier) — which also retires every wave's reads of step st - 1, whose
    // buffer the issue below refills
    const int ahead = min(PD - 1, nsteps - 1 - st);
    if (ahead >= 2) dma_wait<8>();
    else if (ahead == 1) dma_wait<4>();
    else dma_wait<0>();
    __syncthreads();
    if (st + PD < nsteps) issue((st + PD) % NS, st + PD);
    const char* sA = smem + (st % NS) * STAGE;
    const char* sB = sA + T_BYTES;
    s16x4 ta[2][4], tb[2][4];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int row = 8 * g + 4 * half + q;
      const int sw = wg_swz(row);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = (wm * 64 + i * 16) / 8 + (pp >> 1);
        ta[half][i] =
            lds_read_tr((const LDS_AS char*)(sA + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = (wn * 64 + j * 16) / 8 + (pp >> 1);
        tb[half][j] =
            lds_read_tr((const LDS_AS char*)(sB + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
      }
    }
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s16x4 lo = ta[0][i], hi = ta[1][i];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const s16x4 lo = tb[0][j], hi = tb[1][j];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      bfr[j] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  }

  float* slab = a.slab + (size_t)zsplit * a.Mpad * a.KP;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m_tile + wm * 64 + i * 16 + g * 4 + r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k_tile + wn * 64 + j * 16 + li;
        slab[(size_t)co * a.KP + k] = acc[i][j][r];
      }
    }
  }
}

// Three-tap variant of conv_wgrad_kernel: one workgroup (8 waves) owns a 128 co x 384 k
// tile — three consecutive 128-k slices (e.g. the three dw taps of one kernel row) — so the
// dZ rows staged for a 64-pixel step serve three slices instead of one: 64 KB of LDS-DMA
// per step feed 384 MFMAs (171 B/MFMA vs 256 for the 128 x 128 tile, the limiter of the
// im2col wgrad per the no-DMA ablation).  Wave (wm, wn) owns 64 co x 96 k (4 x 6
// fragments); one workgroup per CU (2 x 64 KB stages).  Same swizzle, transposing reads,
// XCD remap and slab layout as conv_wgrad_kernel.
template <int KW>
__global__ void __launch_bounds__(512, 1)
conv_wgrad_t3_kernel(WgradArgs a, WgradLayers Ls) {
  constexpr int BKN = 64;
  constexpr int T_BYTES = BKN * 256;           // one 64 x 128 (bf16) tile
  constexpr int STAGE = 4 * T_BYTES;           // dZ tile + 3 X slices
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;
  const int nwg = a.ktiles * a.mtiles * a.splits * a.nlayers;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, xslot = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + xslot;
  const int kt = lid % a.ktiles;
  const int rest = lid / a.ktiles;
  const int mt = rest % a.mtiles;
  const int rest2 = rest / a.mtiles;
  const int zsplit = rest2 % a.splits;
  const int layer = rest2 / a.splits;
  const char* __restrict__ dZl = Ls.dZ[layer];
  const char* __restrict__ Xl = Ls.X[layer];
  const int k_tile = kt * 384;
  const int m_tile = mt * 128;
  const int n_begin = zsplit * a.px_per_split;
  int n_end = n_begin + a.px_per_split;
  if (n_end > a.Npix) n_end = a.Npix;
  const int nsteps = n_end > n_begin ? (n_end - n_begin + BKN - 1) / BKN : 0;

  // staging: each wave-instruction = 4 rows x 16 slots of 16 B; rows (wave*2 + i)*4 + r_in
  const int r_in = lane >> 4;
  const int slot = lane & 15;
  int koffs[3][2];
  int dz_chunk[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * 2 + i) * 4 + r_in;
    const int c = slot ^ wg_swz(r);
    dz_chunk[i] = (m_tile * 2) + c * 16;
#pragma unroll
    for (int j = 0; j < 3; ++j) koffs[j][i] = koff_wg<KW>((k_tile + j * 128) / 8 + c, a);
  }

  auto stage = [&](int buf, int step) {
    if (a.ablate & 4) return;
    char* sA = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * 2 + i) * 4 + r_in;
      int n = n_begin + step * BKN + r;
      const bool ok = n < n_end;
      if (!ok) n = n_begin;
      const int b = n / NPTS;
      const int p = n - b * NPTS;
      const int h = p / BOARD;
      const int w = p - h * BOARD;
      const uint32_t dzo = frame_off(b, h, w, a.dz_pad, a.M);
      const uint32_t xo = frame_off(b, h, w, a.x_pad, a.x_C);
      const char* src_dz = ok ? (dZl + dzo + dz_chunk[i]) : (dZl + (slot * 16));
      glds16(src_dz, (LDS_AS void*)(sA + (wave * 2 + i) * 1024));
#pragma unroll
      for (int j = 0; j < 3; ++j)
        glds16(Xl + xo + koffs[j][i],
               (LDS_AS void*)(sA + (j + 1) * T_BYTES + (wave * 2 + i) * 1024));
    }
  };

  f32x4 acc[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nsteps > 0) {
    stage(0, 0);
    __syncthreads();
  }
  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  for (int st = 0; st < nsteps; ++st) {
    const int buf = st & 1;
    const char* sA = smem + buf * STAGE;
    s16x4 ta[2][2][4], tb[2][2][6];
    if (a.ablate & 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int i = 0; i < 4; ++i) ta[kk][half][i] = s16x4{};
#pragma unroll
          for (int j = 0; j < 6; ++j) tb[kk][half][j] = s16x4{};
        }
    } else
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int row = kk * 32 + 8 * g + 4 * half + q;
        const int sw = wg_swz(row);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = (wm * 64 + i * 16) / 8 + (pp >> 1);
          ta[kk][half][i] =
              lds_read_tr((const LDS_AS char*)(sA + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
        }
#pragma unroll
        for (int j = 0; j < 6; ++j) {
          const int col = wn * 96 + j * 16;  // within the 384-k tile
          const int c = (col & 127) / 8 + (pp >> 1);
          tb[kk][half][j] = lds_read_tr((const LDS_AS char*)(
              sA + (1 + (col >> 7)) * T_BYTES + row * 256 + ((c ^ sw) * 16) + (pp & 1) * 8));
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // next step's DMA after the tr-reads (else the compiler waits vmcnt(0) before them)
    if (st + 1 < nsteps) stage(buf ^ 1, st + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[6];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const s16x4 lo = ta[kk][0][i], hi = ta[kk][1][i];
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const s16x4 lo = tb[kk][0][j], hi = tb[kk][1][j];
        const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bfr[j] = __builtin_bit_cast(bf16x8, v);
      }
      if (a.ablate & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
        for (int j = 0; j < 6; ++j) asm volatile("" ::"v"(bfr[j]));
      } else
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 6; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();
  }

  if (a.ablate & 8) {
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 6; ++j) keep += acc[i][j][0];
    if (keep == 1234.5f) Ls.slab[layer][0] = keep;
    return;
  }
  float* slab = Ls.slab[layer] + (size_t)zsplit * a.Mpad * a.KP;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = m_tile + wm * 64 + i * 16 + g * 4 + r;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const int k = k_tile + wn * 96 + j * 16 + li;
        slab[(size_t)co * a.KP + k] = acc[i][j][r];
      }
    }
  }
}

// Sum the split-K slabs and scatter into the fp32 master-gradient layout OHWI
// [co][kh][kw][ci] (only ci < Cin, co < M).  out is overwritten.  Each thread owns 4
// consecutive k of one co (16-byte slab loads), the split loop is unrolled by 4 so
// several loads are in flight; the slabs are normally still resident in the Infinity
// Cache when this runs.
constexpr int RD_MAXL = 16;
struct ReduceLayers {  // blockIdx.y = layer (several layers, each with its own shape)
  const float* slab[RD_MAXL];
  float* out[RD_MAXL];
  const float* bpart[RD_MAXL];
  float* gposb[RD_MAXL];
  float* gbias[RD_MAXL];
  // optional bf16 twins of out / gposb / gbias (the data-parallel bf16 wire format: the
  // bucket all-reduce runs on them directly, no conversion kernels; null = fp32 only)
  bf16_t* out16[RD_MAXL];
  bf16_t* gposb16[RD_MAXL];
  bf16_t* gbias16[RD_MAXL];
  int splits[RD_MAXL], M[RD_MAXL], Mpad[RD_MAXL], KP[RD_MAXL], taps[RD_MAXL], cin[RD_MAXL],
      cinp[RD_MAXL], bchunks[RD_MAXL], main_blocks[RD_MAXL];
  long long* sf;   // the fused update's step tag (dg_common.h): an output out of range sets it
};
__global__ void __launch_bounds__(256) wgrad_reduce_kernel(ReduceLayers Ls) {
  const int ly = blockIdx.y;
  const float* __restrict__ slab = Ls.slab[ly];
  float* __restrict__ out = Ls.out[ly];
  const float* __restrict__ bpart = Ls.bpart[ly];
  float* __restrict__ gposb = Ls.gposb[ly];
  float* __restrict__ gbias = Ls.gbias[ly];
  const int splits = Ls.splits[ly], M = Ls.M[ly], Mpad = Ls.Mpad[ly], KP = Ls.KP[ly];
  const int taps = Ls.taps[ly], cin = Ls.cin[ly], cinp = Ls.cinp[ly];
  const int bchunks = Ls.bchunks[ly], main_blocks = Ls.main_blocks[ly];
  const int pos_blocks = bpart ? (NPTS * M + 255) / 256 : 0;
  if ((int)blockIdx.x >= main_blocks + pos_blocks + (bpart ? M : 0)) return;  // (shorter layer)
  if ((int)blockIdx.x >= main_blocks + pos_blocks) {
    // gbias[c] = sum over (chunk, row) of rowpart (the fixed-order rows_sum4 on one lane
    // quad, shared with the fused grad_update kernel); one workgroup per channel
    const int c = blockIdx.x - main_blocks - pos_blocks;
    const float* rp = bpart + (size_t)bchunks * NPTS * M;  // rowpart [bchunks][19][M]
    if (threadIdx.x < 4) {
      const float v = rows_sum4(rp, bchunks * BOARD, M, c, threadIdx.x);
      if (threadIdx.x == 0) {
        gbias[c] = v;
        if (Ls.gbias16[ly]) Ls.gbias16[ly][c] = f2bf(v);
        if (Ls.sf && grad_out_of_range(v)) flag_bad_step(Ls.sf);
      }
    }
    return;
  }
  if ((int)blockIdx.x >= main_blocks) {
    // second pass of the bias gradients (see bias_grad_partial_kernel):
    //   gposb[p][c] = sum_chunks part[chunk][p][c]; gbias[c] = sum_{chunk,h} rowpart[chunk][h][c]
    const int j = (blockIdx.x - main_blocks) * 256 + threadIdx.x;
    const int np = NPTS * M;
    if (j < np) {
      const float v = chunk_sum(bpart + j, bchunks, (size_t)np);
      gposb[j] = v;
      if (Ls.gposb16[ly]) Ls.gposb16[ly][j] = f2bf(v);
      if (Ls.sf && grad_out_of_range(v)) flag_bad_step(Ls.sf);
    }
    return;
  }
  const int kq = KP / 4;
  const int total = M * kq;
  const size_t zstride = (size_t)Mpad * KP;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += main_blocks * blockDim.x) {
    const int co = idx / kq;
    const int k = (idx - co * kq) * 4;
    const f32x4 s = slab_sum4(slab + (size_t)co * KP + k, splits, zstride);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int kk = k + e;
      const int t = kk / cinp;
      const int ci = kk - t * cinp;
      if (t < taps && ci < cin) {
        const size_t o = ((size_t)co * taps + t) * cin + ci;
        out[o] = s[e];
        if (Ls.out16[ly]) Ls.out16[ly][o] = f2bf(s[e]);
      }
    }
    if (Ls.sf && (grad_out_of_range(s[0]) || grad_out_of_range(s[1]) ||
                  grad_out_of_range(s[2]) || grad_out_of_range(s[3])))
      flag_bad_step(Ls.sf);
  }
}

}  // namespace

// ------------------------------------------------------------------------------------
// Host launchers (C ABI used by the pybind11 module).

static uint64_t magic_for(int d) { return fastdiv_magic((uint32_t)d); }

// Allow > 64 KiB of dynamic LDS (gfx950 has 160 KiB per CU); set once per kernel.
template <typename K>
static void allow_lds(K kernel, size_t bytes) {
  static bool done = false;  // one flag per template instantiation
  if (!done && bytes > 65536) {
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    done = true;
  }
}

static hipError_t launch_t3(int kw, WgradArgs a, const WgradLayers& Ls, hipStream_t stream) {
  a.ktiles = a.KP / 384;
  dim3 grid3(a.ktiles * a.mtiles * a.splits * a.nlayers);
  constexpr size_t lds3 = 2 * 4 * 64 * 256;
  if (kw == 3) {
    allow_lds(conv_wgrad_t3_kernel<3>, lds3);
    hipLaunchKernelGGL(conv_wgrad_t3_kernel<3>, grid3, dim3(512), lds3, stream, a, Ls);
  } else {
    allow_lds(conv_wgrad_t3_kernel<5>, lds3);
    hipLaunchKernelGGL(conv_wgrad_t3_kernel<5>, grid3, dim3(512), lds3, stream, a, Ls);
  }
  return hipGetLastError();
}

template <int KW, int MF, int NF, int EPI>
static void launch_nt_epi(const ConvNTArgs& a, int Mpad, hipStream_t s) {
  constexpr int BM = 32 * MF, BN = 32 * NF;
  const size_t lds = 2 * (size_t)(BM * 128 + BN * 128);
  dim3 grid((a.Npix + BN - 1) / BN, Mpad / BM);
  allow_lds(conv_nt_kernel<KW, MF, NF, EPI>, lds);
  hipLaunchKernelGGL((conv_nt_kernel<KW, MF, NF, EPI>), grid, dim3(256), lds, s, a);
}

template <int KW, int MF, int NF>
static hipError_t launch_nt(int epi, const ConvNTArgs& a, int Mpad, hipStream_t s) {
  switch (epi) {
    case EPI_FWD: launch_nt_epi<KW, MF, NF, EPI_FWD>(a, Mpad, s); break;
    case EPI_DGRAD: launch_nt_epi<KW, MF, NF, EPI_DGRAD>(a, Mpad, s); break;
    default: launch_nt_epi<KW, MF, NF, EPI_LINEAR>(a, Mpad, s);
  }
  return hipGetLastError();
}

template <int KW>
static hipError_t dispatch_tile(int epi, const ConvNTArgs& a, int Mpad, int bm, int bn,
                                hipStream_t s) {
  if (bm == 128 && bn == 128) return launch_nt<KW, 4, 4>(epi, a, Mpad, s);
  if (bm == 128 && bn == 192) return launch_nt<KW, 4, 6>(epi, a, Mpad, s);
  if (bm == 64 && bn == 128) return launch_nt<KW, 2, 4>(epi, a, Mpad, s);
  if (bm == 64 && bn == 256) return launch_nt<KW, 2, 8>(epi, a, Mpad, s);
  return hipErrorInvalidValue;
}

extern "C" {

// Conv (forward / dgrad / linear) via the NT implicit-GEMM kernel.
hipError_t dg_conv_nt_ex(int epi, int kw, int bm, int bn, const void* A, int KP, int M,
                         int Mpad, const void* X, int x_pad, int x_C, int Npix, void* Y,
                         int y_pad, const float* bias, const float* posb, const void* aux,
                         int aux_pad, void* mask, hipStream_t stream) {
  if (KP % 64 != 0 || x_C % 8 != 0 || M % 4 != 0 || Mpad % bm != 0 || Npix <= 0)
    return hipErrorInvalidValue;
  ConvNTArgs a;
  a.A = (const bf16_t*)A;
  a.X = (const char*)X;
  a.Y = (char*)Y;
  a.bias = bias;
  a.posb = posb;
  a.aux = (const char*)aux;
  a.KP = KP;
  a.M = M;
  a.Npix = Npix;
  a.x_pad = x_pad;
  a.x_C = x_C;
  a.y_pad = y_pad;
  a.aux_pad = aux_pad;
  a.gpt = x_C / 8;
  a.ngroups = kw * kw * a.gpt;
  a.gpt_magic = magic_for(a.gpt);
  a.mask = (uint8_t*)mask;
  if (mask && (epi != EPI_FWD || M % 8 != 0)) return hipErrorInvalidValue;
  if (a.ngroups * 8 > KP) return hipErrorInvalidValue;
  switch (kw) {
    case 1: return dispatch_tile<1>(epi, a, Mpad, bm, bn, stream);
    case 3: return dispatch_tile<3>(epi, a, Mpad, bm, bn, stream);
    case 5: return dispatch_tile<5>(epi, a, Mpad, bm, bn, stream);
    default: return hipErrorInvalidValue;
  }
}

hipError_t dg_conv_nt(int epi, int kw, int bm, int bn, const void* A, int KP, int M, int Mpad,
                      const void* X, int x_pad, int x_C, int Npix, void* Y, int y_pad,
                      const float* bias, const float* posb, const void* aux, int aux_pad,
                      hipStream_t stream) {
  return dg_conv_nt_ex(epi, kw, bm, bn, A, KP, M, Mpad, X, x_pad, x_C, Npix, Y, y_pad, bias,
                       posb, aux, aux_pad, nullptr, stream);
}

static int g_wgrad_ablate = 0;
void dg_conv_wgrad_set_ablate(int m) { g_wgrad_ablate = m; }
// the 5x5 weight gradient's kernel: 4 = conv_wgrad_pipe_kernel with four 32-pixel stages
// (default: 32.0 vs 32.9 us alone, +0.1..+0.7% in the four configurations' steps, 108 vs 165
// VGPRs; five stages measured slower, 37 us: profiles/r6_wgrad5_pipe.txt), 0 =
// conv_wgrad_kernel (two 64-pixel stages; bit-identical slabs).  DG_WGRAD5_NS=0 | 4
static int g_wgrad5_ns = [] {
  const char* e = getenv("DG_WGRAD5_NS");
  return e && atoi(e) == 0 ? 0 : 4;
}();
void dg_conv_wgrad5_set_ns(int ns) { g_wgrad5_ns = ns == 4 ? 4 : 0; }
int dg_conv_wgrad_wgs_per_cu() { return 2; }
// k-tile width / workgroups per CU of the kernel dg_conv_wgrad will use for this K: the
// three-slice kernel wherever K is a multiple of 384
int dg_conv_wgrad_ktile(int KP) { return KP % 384 == 0 ? 384 : 128; }
int dg_conv_wgrad_wgs_per_cu_for(int KP) {
  return dg_conv_wgrad_ktile(KP) == 384 ? 1 : dg_conv_wgrad_wgs_per_cu();
}

hipError_t dg_conv_wgrad(int kw, const void* dZ, int dz_pad, int M, int Mpad, const void* X,
                         int x_pad, int x_C, int B, int KP, int splits, float* slab,
                         hipStream_t stream) {
  const int Npix = B * NPTS;
  if (KP % 128 != 0 || Mpad % 128 != 0 || x_C % 8 != 0 || M % 8 != 0 || splits <= 0)
    return hipErrorInvalidValue;
  WgradArgs a;
  a.dZ = (const char*)dZ;
  a.X = (const char*)X;
  a.slab = slab;
  a.dz_pad = dz_pad;
  a.M = M;
  a.Mpad = Mpad;
  a.KP = KP;
  a.Npix = Npix;
  int per = (Npix + splits - 1) / splits;
  per = (per + 63) / 64 * 64;
  a.px_per_split = per;
  a.x_pad = x_pad;
  a.x_C = x_C;
  a.gpt = x_C / 8;
  a.ngroups = kw * kw * a.gpt;
  a.gpt_magic = magic_for(a.gpt);
  a.ablate = g_wgrad_ablate;
  if (a.ngroups * 8 > KP) return hipErrorInvalidValue;
  // dZ channel tile must stay inside the dZ rows: for M < Mpad the extra co rows read
  // neighbouring channels/pixels of valid memory and land in unused slab rows.
  a.ktiles = KP / 128;
  a.mtiles = Mpad / 128;
  a.splits = splits;
  a.nlayers = 1;
  if (dg_conv_wgrad_ktile(KP) == 384 && (kw == 3 || kw == 5)) {
    WgradLayers Ls{};
    Ls.dZ[0] = a.dZ;
    Ls.X[0] = a.X;
    Ls.slab[0] = a.slab;
    return launch_t3(kw, a, Ls, stream);
  }
  dim3 grid(a.ktiles * a.mtiles * splits);
  const size_t lds = 2 * 2 * 64 * 256;
  switch (kw) {
    case 1: hipLaunchKernelGGL(conv_wgrad_kernel<1>, grid, dim3(256), lds, stream, a); break;
    case 3: hipLaunchKernelGGL(conv_wgrad_kernel<3>, grid, dim3(256), lds, stream, a); break;
    case 5:
      if (g_wgrad5_ns == 4 && g_wgrad_ablate == 0) {
        constexpr size_t lds4 = 4 * 16 * 1024;
        allow_lds(conv_wgrad_pipe_kernel<5, 4>, lds4);
        hipLaunchKernelGGL((conv_wgrad_pipe_kernel<5, 4>), grid, dim3(256), lds4, stream, a);
      } else {
        allow_lds(conv_wgrad_kernel<5>, lds);
        hipLaunchKernelGGL(conv_wgrad_kernel<5>, grid, dim3(256), lds, stream, a);
      }
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Weight gradients of nl layers of identical geometry in ONE launch (three-slice tiles):
// table = nl rows of {dZ frame, X frame, slab} pointers; each layer gets `splits` pixel
// splits.  Fewer splits per layer than a one-layer launch at the same machine fill, so
// proportionally fewer fp32 partial slabs to write and reduce.
hipError_t dg_conv_wgrad_multi(int kw, const long long* table, int nl, int dz_pad, int M,
                               int Mpad, int x_pad, int x_C, int B, int KP, int splits,
                               hipStream_t stream) {
  const int Npix = B * NPTS;
  if (nl <= 0 || nl > MAXWL || KP % 384 != 0 || Mpad % 128 != 0 || x_C % 8 != 0 ||
      M % 8 != 0 || splits <= 0 || (kw != 3 && kw != 5))
    return hipErrorInvalidValue;
  WgradArgs a{};
  a.dz_pad = dz_pad;
  a.M = M;
  a.Mpad = Mpad;
  a.KP = KP;
  a.Npix = Npix;
  int per = (Npix + splits - 1) / splits;
  a.px_per_split = (per + 63) / 64 * 64;
  a.x_pad = x_pad;
  a.x_C = x_C;
  a.gpt = x_C / 8;
  a.ngroups = kw * kw * a.gpt;
  a.gpt_magic = magic_for(a.gpt);
  a.ablate = g_wgrad_ablate;
  if (a.ngroups * 8 > KP) return hipErrorInvalidValue;
  a.mtiles = Mpad / 128;
  a.splits = splits;
  a.nlayers = nl;
  WgradLayers Ls{};
  for (int i = 0; i < nl; ++i) {
    Ls.dZ[i] = (const char*)table[3 * i];
    Ls.X[i] = (const char*)table[3 * i + 1];
    Ls.slab[i] = (float*)table[3 * i + 2];
    if (!Ls.dZ[i] || !Ls.X[i] || !Ls.slab[i]) return hipErrorInvalidValue;
  }
  a.dZ = Ls.dZ[0];
  a.X = Ls.X[0];
  a.slab = Ls.slab[0];
  return launch_t3(kw, a, Ls, stream);
}

static void reduce_layer(ReduceLayers& Ls, int i, const float* slab, float* out,
                         const float* bpart, float* gposb, float* gbias, int splits, int M,
                         int Mpad, int KP, int taps, int cin, int cinp, int bchunks) {
  int blocks = (M * (KP / 4) + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  Ls.slab[i] = slab;
  Ls.out[i] = out;
  Ls.bpart[i] = bpart;
  Ls.gposb[i] = gposb;
  Ls.gbias[i] = gbias;
  Ls.splits[i] = splits;
  Ls.M[i] = M;
  Ls.Mpad[i] = Mpad;
  Ls.KP[i] = KP;
  Ls.taps[i] = taps;
  Ls.cin[i] = cin;
  Ls.cinp[i] = cinp;
  Ls.bchunks[i] = bchunks;
  Ls.main_blocks[i] = blocks;
}
static int reduce_grid_x(const ReduceLayers& Ls, int i) {
  return Ls.main_blocks[i] + (Ls.bpart[i] ? (NPTS * Ls.M[i] + 255) / 256 + Ls.M[i] : 0);
}

hipError_t dg_wgrad_reduce(const float* slab, float* out, int splits, int M, int Mpad, int KP,
                           int taps, int cin, int cinp, const float* bpart, int bchunks,
                           float* gposb, float* gbias, void* out16, void* gposb16, void* gbias16,
                           long long* sf, hipStream_t stream) {
  ReduceLayers Ls{};
  Ls.sf = sf;
  reduce_layer(Ls, 0, slab, out, bpart, gposb, gbias, splits, M, Mpad, KP, taps, cin, cinp,
               bchunks);
  Ls.out16[0] = (bf16_t*)out16;
  Ls.gposb16[0] = (bf16_t*)gposb16;
  Ls.gbias16[0] = (bf16_t*)gbias16;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(reduce_grid_x(Ls, 0), 1), dim3(256), 0, stream,
                     Ls);
  return hipGetLastError();
}

// Slab reduce + bias-gradient pass 2 of nl layers (any shapes) in one launch: table = nl
// rows of `cols` int64 {slab, out (weight grad), bpart, gposb, gbias, splits, M, Mpad, KP,
// taps, cin, cinp, bchunks[, out16, gposb16, gbias16]} (cols 13, or 16 with bf16 twins).
hipError_t dg_wgrad_reduce_multi(const long long* table, int nl, int cols, hipStream_t stream) {
  if (nl <= 0 || nl > RD_MAXL || (cols != 13 && cols != 16)) return hipErrorInvalidValue;
  ReduceLayers Ls{};
  int gx = 1;
  for (int i = 0; i < nl; ++i) {
    const long long* t = table + cols * i;
    if (cols == 16) {
      Ls.out16[i] = (bf16_t*)t[13];
      Ls.gposb16[i] = (bf16_t*)t[14];
      Ls.gbias16[i] = (bf16_t*)t[15];
    }
    if (!t[0] || !t[1] || !t[2] || t[5] <= 0 || t[6] <= 0 || t[8] % 4 != 0)
      return hipErrorInvalidValue;
    reduce_layer(Ls, i, (const float*)t[0], (float*)t[1], (const float*)t[2], (float*)t[3],
                 (float*)t[4], (int)t[5], (int)t[6], (int)t[7], (int)t[8], (int)t[9],
                 (int)t[10], (int)t[11], (int)t[12]);
    gx = gx > reduce_grid_x(Ls, i) ? gx : reduce_grid_x(Ls, i);
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(gx, nl), dim3(256), 0, stream, Ls);
  return hipGetLastError();
}

}  // extern "C"
