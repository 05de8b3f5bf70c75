// Row-stripe weight gradient for 3x3 stride-1 layers (the hidden layers of the Go CNN).
//
//   dW[co][dh][dw][ci] = sum_{b,p} dZ[b][p][co] * X[b][p + (dh-1, dw-1)][ci]
//
// The im2col wgrad (conv_mfma.hip) stages one 128-wide k tile (= one tap) per 64-pixel
// step, so every input row is fetched once per tap (9x) and the whole kernel is bound by
// global->LDS traffic per CU (profiles/README.md).  Here a workgroup owns a
// 128 co x (3 taps x CK channels) tile — one kernel row dh, all three dw — and per 64-pixel
// step stages
//   * the 64 dZ rows (256 B each, 128 co), and
//   * ONE X stripe: the contiguous frame rows that the 64 pixels' three horizontal taps
//     touch (<= 74 rows for a pad-1 frame instead of 3 x 64),
// then the three dw fragments read the same stripe at a +dw row offset.  That is 3x the
// MFMA work per staged byte of the im2col kernel (CK = 128: 36 KB per 6.3 MFLOP).
//
// Pixels are processed per board in NSUB = 6 steps of 64 (the last has 41 valid; missing
// dZ rows read the frame's zero border, so they contribute nothing).  The (board, step)
// sequence is split over `splits` workgroups per tile (fp32 slabs, reduced by
// wgrad_reduce_kernel in conv_mfma.hip — same slab layout [split][Mpad][KP], k = tap*x_C+ci).
//
// Operands are staged pixel-major with LDS-DMA and read with the CDNA4 transposing
// ds_read_b64_tr_b16; 8 waves = 2 (co) x 4 (k), each 64 co x 3CK/4 k of 16x16 fragments
// of v_mfma_f32_16x16x32_bf16.  LDS rows are padded (see RS_A) rather than swizzled, so
// fragment addresses cost no VALU in the loop (the swizzled first version was VALU-issue
// bound: ~250 address ops per 48 MFMAs per wave and step).
//
// Reference op: nn.SpatialConvolutionMM accGradParameters (SURVEY.md N4;
// /root/reference/experiments.lua:138).
#include <stdlib.h>

#include "dg_common.h"

using namespace dg;

namespace {

constexpr int PSTEP = 64;
constexpr int NSUB = (NPTS + PSTEP - 1) / PSTEP;  // 6

DG_DEV int div19(int p) { return (p * 3450) >> 16; }  // exact for 0 <= p < 400

struct W3Args {
  const char* dZ;  // gradient frame [B][Fz][Fz][M] bf16
  const char* X;   // input frame [B][F][F][x_C] bf16
  float* slab;     // [splits][Mpad][KP]
  int dz_pad, M, Mpad, KP;
  int x_pad, x_C;
  int total_steps;  // B * NSUB
  int splits, tiles, mtiles;
  int ablate;       // 1 no MFMA, 2 no LDS reads, 4 no DMA, 8 no slab store (tools/kbench.py)
};

// LDS geometry.  Rows are PADDED instead of XOR-swizzled: a 288-B (256 + 32) stride puts
// row r at bank group 8r mod 64, so the 8 consecutive pixel rows that one 32-lane
// ds_read_b64_tr_b16 group reads (32 B each) hit 8 disjoint bank groups, and every fragment
// address is one per-lane VGPR base plus a compile-time immediate (no per-read VALU).
// 160-B rows (CK = 64) give groups {0,40,16,56,32,8,48,24} — also disjoint.
constexpr int RS_A = 288;                         // dZ rows: 128 co = 256 B + pad
constexpr int A_BYTES = PSTEP * RS_A;             // 18 KiB = 18 DMA instructions
template <int CK> struct XGeo {
  static constexpr int RS = CK * 2 + 32;          // stripe row stride
  static constexpr int BYTES = CK == 128 ? 24 * 1024 : 14 * 1024;  // >= 84 rows (F <= 23)
};

// NW waves per workgroup: 8 (one workgroup per CU, 3-stage ring) or 4 (two independent
// workgroups per CU — one's reads / barrier / slab store run under the other's MFMAs —
// with a 2-stage ring in 64 KB of LDS).
template <int CK, int NW>
__global__ void __launch_bounds__(NW * 64, NW == 4 ? 2 : 1)
conv_wgrad3_kernel(W3Args a) {
  constexpr int NSTAGE = NW == 8 ? 3 : 2;
  constexpr int LOOK = NSTAGE - 1;           // stages in flight ahead of the one read
  constexpr int WN = NW / 2;
  constexpr int RS_X = XGeo<CK>::RS;
  constexpr int X_BYTES = XGeo<CK>::BYTES;
  constexpr int STAGE = A_BYTES + X_BYTES;
  constexpr int NKT = 3 * CK;                // k width of the tile
  constexpr int WK = NKT / WN;               // k per wave
  constexpr int NF = WK / 16;                // 6 (CK 128 / NW 8, CK 64 / NW 4) or 3
  constexpr int MF = 4;
  constexpr int A_INSTR = A_BYTES / 1024;    // 18
  constexpr int X_INSTR_MAX = X_BYTES / 1024;
  constexpr int A_PW = (A_INSTR + NW - 1) / NW;      // dZ DMA instructions per wave
  constexpr int X_PW = (X_INSTR_MAX + NW - 1) / NW;  // stripe DMA instructions per wave
  constexpr int DMA_PER_STEP = A_PW + X_PW;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware remap (cdna guide T1): consecutive logical ids (the tiles of one split, which
  // share every dZ row and most X rows) land on one XCD and hit its L2.
  const int nwg = a.splits * a.tiles;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, xslot = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + xslot;
  const int split = lid / a.tiles;
  const int tile = lid - split * a.tiles;
  const int mt = tile % a.mtiles;
  const int rest = tile / a.mtiles;
  const int dh = rest % 3;
  const int cc = rest / 3;
  const int st_begin = (int)(((long long)split * a.total_steps) / a.splits);
  const int st_end = (int)(((long long)(split + 1) * a.total_steps) / a.splits);

  const int F = BOARD + 2 * a.x_pad;
  const int FF = F * F;
  const int Fz = BOARD + 2 * a.dz_pad;
  const size_t zrow = (size_t)a.M * 2;     // dZ frame row bytes
  const size_t xrow = (size_t)a.x_C * 2;   // X frame row bytes

  // per-step geometry (wave-uniform)
  struct Geo {
    int b, p0, pc, h0, w0, nr, fr0;
  };
  auto geo = [&](int st) {
    Geo g;
    g.b = st / NSUB;
    const int sub = st - g.b * NSUB;
    g.p0 = sub * PSTEP;
    g.pc = min(PSTEP, NPTS - g.p0);
    const int pl = g.p0 + g.pc - 1;
    g.h0 = div19(g.p0);
    g.w0 = g.p0 - 19 * g.h0;
    const int hl = div19(pl), wl = pl - 19 * hl;
    g.nr = (hl - g.h0) * F + (wl - g.w0) + 3;
    g.fr0 = (g.h0 + a.x_pad + dh - 1) * F + (g.w0 + a.x_pad) - 1;
    return g;
  };

  // DMA lane geometry (loop invariant): instruction j of a stage covers LDS bytes
  // [j*1024, j*1024+1024); lane -> (row, col) of the padded image.  Pad lanes re-read
  // column 0 of their row (any valid address).
  int a_row[A_PW], a_col[A_PW], x_row[X_PW], x_col[X_PW];
#pragma unroll
  for (int m = 0; m < A_PW; ++m) {
    const int d = (wave + NW * m) * 1024 + lane * 16;
    a_row[m] = d / RS_A;
    const int ca = d - a_row[m] * RS_A;
    a_col[m] = ca < 256 ? ca : 0;
  }
#pragma unroll
  for (int m = 0; m < X_PW; ++m) {
    const int d = (wave + NW * m) * 1024 + lane * 16;
    x_row[m] = d / RS_X;
    const int cx = d - x_row[m] * RS_X;
    x_col[m] = cx < CK * 2 ? cx : 0;
  }

  const bool no_dma = a.ablate & 4;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_AS char*)smem;
  // Exactly A_PW dZ + X_PW X instructions per wave and step (DMA_PER_STEP): instructions past
  // the real count repeat one of the step's real ones (same source, same destination,
  // identical bytes), so vmcnt arithmetic is static.
  auto stage = [&](int buf, const Geo& g) {
    if (no_dma) return;
    const uint32_t sA = lds0 + buf * STAGE;
    const uint32_t sX = sA + A_BYTES;
    const char* zb = a.dZ + (size_t)g.b * Fz * Fz * zrow;
#pragma unroll
    for (int m = 0; m < A_PW; ++m) {
      // (no runtime-indexed register arrays here: they would go to scratch, and a scratch
      // load's vmcnt wait would also wait for the in-flight DMA)
      const bool real = wave + NW * m < A_INSTR;  // past the 18 pieces: repeat piece m = 0
      const int j = real ? wave + NW * m : wave;
      const int r = real ? a_row[m] : a_row[0];
      const int acol = real ? a_col[m] : a_col[0];
      const char* src;
      if (r < g.pc) {
        const int p = g.p0 + r;
        const int h = div19(p), w = p - 19 * h;
        src = zb + ((h + a.dz_pad) * Fz + w + a.dz_pad) * zrow + mt * 256 + acol;
      } else {
        src = zb + (acol & 255);  // zero border row 0 of the frame
      }
      dma16(src, __builtin_amdgcn_readfirstlane(sA + j * 1024));
    }
    const int ninstr = min((g.nr * RS_X + 1023) / 1024, X_INSTR_MAX);
    const char* xb = a.X + (size_t)g.b * FF * xrow + cc * (CK * 2);
#pragma unroll
    for (int m = 0; m < X_PW; ++m) {
      int j = wave + NW * m;
      int rr = x_row[m], col = x_col[m];
      if (j >= ninstr) {  // repeat a real instruction of this step (identical bytes)
        j = wave % ninstr;
        const int d = j * 1024 + lane * 16;
        rr = d / RS_X;
        col = d - rr * RS_X;
        col = col < CK * 2 ? col : 0;
      }
      int fr = g.fr0 + rr;
      fr = fr < FF ? fr : FF - 1;
      dma16(xb + (size_t)fr * xrow + col, __builtin_amdgcn_readfirstlane(sX + j * 1024));
    }
  };

  f32x4 acc[MF][NF];
#pragma unroll
  for (int i = 0; i < MF; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int g4 = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  // MFMA k-slot -> pixel permutation: k-slot 8*g4 + 4*half + q of 32-slot block kk reads
  // pixel row kk*32 + 16*(g4>>1) + 8*half + 4*(g4&1) + q, so lanes 0-31 (g4 0/1) of each
  // tr-read touch 8 CONSECUTIVE pixel rows (both operands use the same permutation, the
  // contraction over pixels is unchanged).
  const int prow0 = 16 * (g4 >> 1) + 4 * (g4 & 1) + q;
  const int lane_col = (pp >> 1) * 16 + (pp & 1) * 8;
  const int a_base = prow0 * RS_A + wm * 128 + lane_col;

  const int nst = st_end - st_begin;
  Geo cur = geo(st_begin);
  if (nst > 0) stage(0, cur);
  if (LOOK == 2 && nst > 1) stage(1, geo(st_begin + 1));
  if (LOOK == 2 && nst > 1) dma_wait<DMA_PER_STEP>(); else dma_wait<0>();
  __builtin_amdgcn_s_barrier();
  for (int st = st_begin; st < st_end; ++st) {
    const int ls = st - st_begin;
    const int buf = ls % NSTAGE;
    const bool more = ls + LOOK < nst;
    if (more) stage((ls + LOOK) % NSTAGE, geo(st + LOOK));  // into the stage read at ls - 1
    const LDS_AS char* sA = (const LDS_AS char*)(smem + buf * STAGE) + a_base;
    const LDS_AS char* sX = (const LDS_AS char*)(smem + buf * STAGE + A_BYTES) + lane_col;
    // stripe row of each pixel row this lane reads: rel = frame(p) - frame(p0)
    const LDS_AS char* xbase[2][2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        int p = cur.p0 + kk * 32 + 8 * half + prow0;
        p = p < cur.p0 + cur.pc ? p : cur.p0 + cur.pc - 1;
        const int h = div19(p), w = p - 19 * h;
        xbase[kk][half] = sX + ((h - cur.h0) * F + (w - cur.w0)) * RS_X;
      }
    s16x4 ta[2][2][MF], tb[2][2][NF];
    if (a.ablate & 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int i = 0; i < MF; ++i) ta[kk][half][i] = s16x4{};
#pragma unroll
          for (int j = 0; j < NF; ++j) tb[kk][half][j] = s16x4{};
        }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int i = 0; i < MF; ++i)
            ta[kk][half][i] = lds_read_tr(sA + (kk * 32 + 8 * half) * RS_A + i * 32);
#pragma unroll
          for (int j = 0; j < NF; ++j) {
            const int kf = wn * WK + j * 16;  // wave-uniform
            tb[kk][half][j] =
                lds_read_tr(xbase[kk][half] + (kf / CK) * RS_X + ((kf % CK) / 8) * 16);
          }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (a.ablate & 1) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int i = 0; i < MF; ++i) asm volatile("" ::"v"(ta[kk][half][i]));
#pragma unroll
          for (int j = 0; j < NF; ++j) asm volatile("" ::"v"(tb[kk][half][j]));
        }
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[MF], bfr[NF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const s16x4 lo = ta[kk][0][i], hi = ta[kk][1][i];
          const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          af[i] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const s16x4 lo = tb[kk][0][j], hi = tb[kk][1][j];
          const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          bfr[j] = __builtin_bit_cast(bf16x8, v);
        }
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // DMA wait + barrier stay below the MFMAs
    // stage ls+1 must have landed (every wave's part) before anyone reads it; stage ls+2
    // (issued this step) stays in flight
    if (LOOK == 2 && more) dma_wait<DMA_PER_STEP>(); else dma_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (ls + 1 < nst) cur = geo(st + 1);
  }

  if (a.ablate & 8) {
    float keep = 0.f;
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) keep += acc[i][j][0];
    if (keep == 1234.5f) a.slab[0] = keep;
    return;
  }
  float* slab = a.slab + (size_t)split * a.Mpad * a.KP;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int kf = wn * WK + j * 16 + li;
    const int dw = kf / CK;
    const int k = (dh * 3 + dw) * a.x_C + cc * CK + (kf % CK);
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = mt * 128 + wm * 64 + i * 16 + g4 * 4 + r;
        slab[(size_t)co * a.KP + k] = acc[i][j][r];
      }
  }
}

template <int CK, int NW>
hipError_t launch3(const W3Args& a, hipStream_t s) {
  constexpr size_t lds = (NW == 8 ? 3 : 2) * (size_t)(A_BYTES + XGeo<CK>::BYTES);
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_wgrad3_kernel<CK, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL((conv_wgrad3_kernel<CK, NW>), dim3(a.splits * a.tiles), dim3(NW * 64), lds,
                     s, a);
  return hipGetLastError();
}

// variant: 0 = CK 128 / 8 waves (x_C % 128 == 0), 1 = CK 64 / 4 waves, 2 = CK 64 / 8 waves
int g_variant = -1;
int variant_for(int x_C) {
  int& v = g_variant;
  if (v < 0) {
    const char* e = getenv("DG_WGRAD3_VARIANT");
    v = e ? atoi(e) : 1;
  }
  if (v == 0 && x_C % 128 != 0) return 2;
  return v;
}

}  // namespace

static int g_wgrad3_ablate = 0;
extern "C" void dg_conv_wgrad3_set_ablate(int m) { g_wgrad3_ablate = m; }

// Tiles per split for a layer (host helper shared with the Python split picker).
extern "C" int dg_wgrad3_tiles(int Mpad, int x_C) {
  const int ck = variant_for(x_C) == 0 ? 128 : 64;
  return (Mpad / 128) * 3 * (x_C / ck);
}
// workgroups that fit on one CU (LDS / registers): splits = num_cus * this / tiles
extern "C" void dg_wgrad3_set_variant(int v) { g_variant = v; }
extern "C" int dg_wgrad3_wgs_per_cu(int x_C) { return variant_for(x_C) == 1 ? 2 : 1; }

extern "C" hipError_t dg_conv_wgrad3(const void* dZ, int dz_pad, int M, int Mpad, const void* X,
                                     int x_pad, int x_C, int B, int KP, int splits, float* slab,
                                     hipStream_t stream) {
  if (x_C % 64 != 0 || M % 8 != 0 || Mpad % 128 != 0 || M > Mpad || splits <= 0 || B <= 0)
    return hipErrorInvalidValue;
  if (x_pad < 1 || x_pad > 2 || dz_pad < 1 || KP < 9 * x_C) return hipErrorInvalidValue;
  W3Args a;
  a.dZ = (const char*)dZ;
  a.X = (const char*)X;
  a.slab = slab;
  a.dz_pad = dz_pad;
  a.M = M;
  a.Mpad = Mpad;
  a.KP = KP;
  a.x_pad = x_pad;
  a.x_C = x_C;
  a.total_steps = B * NSUB;
  a.splits = splits < a.total_steps ? splits : a.total_steps;
  a.mtiles = Mpad / 128;
  a.tiles = dg_wgrad3_tiles(Mpad, x_C);
  a.ablate = g_wgrad3_ablate;
  if (splits != a.splits) return hipErrorInvalidValue;  // caller sized the slab for `splits`
  switch (variant_for(x_C)) {
    case 0: return launch3<128, 8>(a, stream);
    case 1: return launch3<64, 4>(a, stream);
    default: return launch3<64, 8>(a, stream);
  }
}
