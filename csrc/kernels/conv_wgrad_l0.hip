// Sliding-window weight gradient of the FIRST layer (5x5 taps, 37/38 input planes padded to
// 40 channels): the hidden layers' window trick (conv_wgrad_win.hip) on the 23 x 23 frame of
// the expanded input.
//
//   dW[co][t][ci] = sum_G dZ[G][co] * X[G + off_t][ci],   off_t = (kh - 2) * 23 + (kw - 2)
//
// G runs over the rows of the zero-bordered 23 x 23 input frames (pad 2) of consecutive
// boards.  dZ lives in the 21 x 21 frames (pad 1) of the layer's output gradient, so each
// staged dZ row is GATHERED: frame-23 row (b, r, c) -> dZ row b*441 + (r-1)*21 + (c-1) when
// (r, c) is on the board, else a zero row — dZ is then zero wherever an X window would reach
// past its board's 2-pixel border, and the 25 taps are 25 constant row shifts of one X window.
// Per board the K-steps cover frame rows 2..20 (G = b*529 + 46 + 32j, j < 14: 448 of 529
// rows).
//
// The GEMM's N dimension is the FLAT (tap, channel) index k = t * 40 + ci (1000 columns, 63
// fragments of 16 and one zero one): a 16-column B fragment may straddle two taps — the
// transposing LDS read takes a per-lane row address, and 4-column lane groups never straddle
// one (40 = 10 x 4) — so the 40-channel input is not padded to a power of two (the
// three-slice im2col kernel it replaces, conv_mfma.hip conv_wgrad_kernel<5>, staged 25 taps x
// 40 channels of im2col rows per 64 pixels: 256 B of LDS-DMA per MFMA; here a K-step stages 32
// dZ rows and 32 new X rows for 32 MFMAs per wave: 32 B per MFMA).
//
// Workgroup = 8 waves: 64 co x all 1024 columns; wave w owns fragments 8w .. 8w+7 (4 x 8
// accumulator fragments, 128 registers).  One workgroup per CU (X ring 64 KB: the board-to-
// board jump of 81 rows plus the 5x5 reach needs more than 256 rows in flight).
// Output: fp32 split slabs slab[z][co][t*40 + ci] in the layout wgrad_reduce sums (the same
// as conv_wgrad_kernel<5>'s).
//
// Reference semantics: SpatialConvolutionMM accGradParameters of the first 5x5 convolution of
// getBasicModel (experiments.lua:135-149).
#include "dg_common.h"

using namespace dg;

namespace {

constexpr int WF = 23;               // frame width (pad 2)
constexpr int WFF = WF * WF;         // 529 rows per board
constexpr int DZF = 21;              // the dZ frame (pad 1)
constexpr int DZFF = DZF * DZF;      // 441
constexpr int SPB = 14;              // K-steps per board: 14 x 32 = 448 rows from frame row 2
constexpr int G_FIRST = 2 * WF;      // 46: first row of a board's K range
constexpr int REACH = 2 * WF + 2;    // 48: the largest |off_t|
constexpr int XR = 512;              // X ring rows (128 B each: 40 channels + zero pad)
constexpr int XRING = XR * 128;      // 64 KB
constexpr int CIN = 40;              // input channels (37/38 planes padded)
constexpr int NCOL = 25 * CIN;       // 1000 flat (tap, channel) columns
constexpr int NW = 8;
constexpr int PD = 3;                // LDS-DMA prefetch distance (K-steps)
constexpr int DZR = 128;             // dZ LDS row bytes (64 co)
constexpr int DZB = 32 * DZR;        // one dZ step

struct L0Args {
  const char* dZ;     // [B][441][M] bf16
  const char* X;      // [B][529][40] bf16
  const char* zero;   // >= 128 zero bytes
  float* slab;        // [splits][Mpad][KP]
  int M, Mpad, KP, B, splits;
};

// the window kernel's 16-B slot swizzle of a 128-B ring row (bits 1 and 3 of the row)
DG_DEV int xswz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

DG_DEV int step_g0(int s) {
  const int b = s / SPB;
  return b * WFF + G_FIRST + 32 * (s - b * SPB);
}

__global__ void __launch_bounds__(64 * NW, 1) conv_wgrad_l0_kernel(L0Args a) {
  __shared__ __attribute__((aligned(16))) char smem[XRING + (PD + 1) * DZB];
  char* xring = smem;
  char* dzbuf = smem + XRING;
  const uint32_t xring_u = (uint32_t)(uintptr_t)(LDS_AS char*)smem;
  const uint32_t dz_u = xring_u + XRING;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nco = a.M / 64;
  const int coch = blockIdx.x % nco;
  const int zsplit = blockIdx.x / nco;
  const char* __restrict__ dZl = a.dZ + coch * 128;
  const int Mb = a.M * 2;
  const int Gmax = a.B * WFF;
  const int T = a.B * SPB;
  const int s0 = (int)((long long)zsplit * T / a.splits);
  const int s1 = (int)((long long)(zsplit + 1) * T / a.splits);

  // one 1-KB block of X ring rows r0 .. r0+7: lane -> (row, LDS slot lane & 7), source piece
  // (lane & 7) ^ swizzle; pieces 5..7 (channels 40..63) are zeros
  auto x_block = [&](int r0) {
    const int row = r0 + (lane >> 3);
    const int c = (lane & 7) ^ xswz(row & (XR - 1));
    int gr = row < 0 ? 0 : row;
    gr = gr >= Gmax ? Gmax - 1 : gr;
    const char* src = c < 5 ? a.X + (size_t)gr * (CIN * 2) + c * 16 : a.zero;
    dma16(src, __builtin_amdgcn_readfirstlane(xring_u + (r0 & (XR - 1)) * 128));
  };
  // 8 dZ rows (block k of the 32 rows of step g0) into buffer buf, gathered from the 21 x 21
  // frames (zero rows off the board)
  auto dz_block = [&](int buf, int g0, int k) {
    const int r = k * 8 + (lane >> 3);
    const int c = (lane & 7) ^ xswz(r);
    const int G = g0 + r;
    const int b = G / WFF;                       // (per lane; a few VALU per DMA)
    const int rc = G - b * WFF;
    const int fr = (rc * 2850) >> 16;            // rc / 23, exact for rc < 529
    const int fc = rc - fr * WF;
    const bool on = fr >= 2 && fr <= 20 && fc >= 2 && fc <= 20 && b < a.B;
    const char* src = on ? dZl + ((size_t)b * DZFF + (fr - 1) * DZF + (fc - 1)) * Mb + c * 16
                         : a.zero + c * 16;
    dma16(src, __builtin_amdgcn_readfirstlane(dz_u + buf * DZB + k * 1024));
  };
  int loaded_hi = 0;
  // steady-state issue for step sn into dZ buffer buf: 2 DMAs per wave (3 at a board's first
  // step): X blocks lo.. (a wave past the last new block re-loads the first, same bytes), and
  // dZ block (wave & 3) (waves 4..7 repeat waves 0..3's, same bytes)
  auto issue = [&](int sn, int buf) {
    const int g0n = step_g0(sn);
    int lo = (g0n - REACH) & ~7;
    if (lo < loaded_hi) lo = loaded_hi;
    const int hi = (g0n + 32 + REACH + 7) & ~7;
    const int nblk = (hi - lo) >> 3;            // 4 inside a board, <= 16 at a board start
    x_block(lo + 8 * (wave < nblk ? wave : 0));
    if (nblk > NW) x_block(lo + 8 * (wave + NW < nblk ? wave + NW : 0));
    loaded_hi = hi;
    dz_block(buf, g0n, wave & 3);
  };

  f32x4 acc[4][8];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[i][u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  const int p1 = pp >> 1, p0 = (pp & 1) * 8;

  if (s0 < s1) {
    const int g0 = step_g0(s0);
    const int lo = (g0 - REACH) & ~7;
    loaded_hi = (g0 + 32 + REACH + 7) & ~7;
    for (int k = wave; k < ((loaded_hi - lo) >> 3); k += NW) x_block(lo + 8 * k);
    dz_block(0, g0, wave & 3);
    dma_wait<0>();
    __syncthreads();
#pragma unroll
    for (int p = 1; p < PD; ++p)
      if (s0 + p < s1) issue(s0 + p, p);
  }
  // Per-lane LDS read addresses.  dZ (A, the 64 co): as the window kernel.  X (B): fragment
  // 8 * wave + u, column group pp -> flat column k = 16 f + 4 pp -> (tap, channel); the ring
  // slot of row q / half h is (g0 + off_t + rl) & (XR - 1); inside a board g0 advances by 32
  // (bits 1 and 3 of the slot, the swizzle's, unchanged), so per step the address is
  // (rel + 4096 j) & (XRING - 1) with rel computed once per board.  Columns past 1000 read
  // channels 40..43 (zeros).
  int rel_d[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rl = 8 * g + 4 * h + q;
    const int sw = xswz(rl);
#pragma unroll
    for (int i = 0; i < 4; ++i) rel_d[h][i] = rl * DZR + (((2 * i + p1) ^ sw) * 16) + p0;
  }
  int col_off[8], col_ci[8];   // per fragment: the lane group's tap offset and channel
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int k = 16 * (8 * wave + u) + 4 * pp;
    const int t = k < NCOL ? k / CIN : 0;
    col_ci[u] = k < NCOL ? k - t * CIN : CIN;
    col_off[u] = (t / 5 - 2) * WF + (t % 5 - 2);
  }
  int rel_x[8][2];
  auto board_rel = [&](int gb) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int slot = (gb + col_off[u] + 8 * g + 4 * h + q) & (XR - 1);
        const int ci = col_ci[u];
        rel_x[u][h] = slot * 128 + (((ci >> 3) ^ xswz(slot)) * 16) + (ci & 7) * 2;
      }
  };
  int bsteps = s0 / SPB;
  int j = s0 - bsteps * SPB;
  board_rel(bsteps * WFF + G_FIRST);
  int buf = 0, buf_pd = PD;
  auto wait_next = [&](int st) {
    if (st + PD < s1) {
      const int r = (st + 2) % SPB;   // a board-first step among st+2 .. st+PD: one more DMA
      if (r == 0 || r + PD - 2 >= SPB)
        dma_wait<2 * (PD - 1) + 1>();
      else
        dma_wait<2 * (PD - 1)>();
    } else {
      dma_wait<0>();
    }
  };
  for (int st = s0; st < s1; ++st) {
    if (st + PD < s1) issue(st + PD, buf_pd);
    if (j == SPB) {
      j = 0;
      ++bsteps;
      board_rel(bsteps * WFF + G_FIRST);
    }
    const int jo = j * 4096;
    const char* sD = dzbuf + buf * DZB;
    s16x4 ta[2][4], tb[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) ta[h][i] = lds_read_tr((const LDS_AS char*)(sD + rel_d[h][i]));
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        tb[h][u] = lds_read_tr((const LDS_AS char*)(xring + ((rel_x[u][h] + jo) & (XRING - 1))));
    bf16x8 af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s16x4 lo = ta[0][i], hi = ta[1][i];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const s16x4 lo = tb[0][u], hi = tb[1][u];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][u] = mfma16(af[i], bfr, acc[i][u]);
    }
    wait_next(st);
    __syncthreads();
    buf = buf == PD ? 0 : buf + 1;
    buf_pd = buf_pd == PD ? 0 : buf_pd + 1;
    ++j;
  }

  float* slab = a.slab + (size_t)zsplit * a.Mpad * a.KP;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = coch * 64 + i * 16 + g * 4 + r;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = 16 * (8 * wave + u) + li;
        if (k < NCOL) slab[(size_t)co * a.KP + k] = acc[i][u][r];
      }
    }
}

}  // namespace

extern "C" {

// splits: workgroups per 64-co chunk (the slab count); one workgroup per CU
int dg_conv_wgrad_l0_splits(int M, int B, int num_cus) {
  int s = num_cus / (M / 64);
  if (s > 64) s = 64;            // the slab volume wgrad_reduce sums (64 x Mpad x KP floats)
  const int smax = B * SPB / 4;  // at least 4 K-steps each
  if (s > smax) s = smax;
  return s < 1 ? 1 : s;
}

// dZ: [B][21][21][M] bf16 (the layer's output gradient frames, pad 1); X: [B][23][23][40] bf16
// (the expanded input frames, pad 2); zero: >= 128 zero bytes; slab: [splits][Mpad][KP] fp32
// with k = t * 40 + ci (KP >= 1000).
hipError_t dg_conv_wgrad_l0(const void* dZ, const void* X, const void* zero, float* slab,
                            int M, int Mpad, int KP, int B, int splits, hipStream_t stream) {
  if (!dZ || !X || !zero || !slab || M % 64 != 0 || Mpad < M || KP < NCOL || B <= 0 ||
      splits <= 0 || splits > B * SPB)
    return hipErrorInvalidValue;
  L0Args a{(const char*)dZ, (const char*)X, (const char*)zero, slab, M, Mpad, KP, B, splits};
  hipLaunchKernelGGL(conv_wgrad_l0_kernel, dim3((M / 64) * splits), dim3(64 * NW), 0, stream, a);
  return hipGetLastError();
}

}  // extern "C"
