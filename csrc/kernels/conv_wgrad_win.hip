// Sliding-window weight gradient of 3x3 layers on the frame-linear pixel axis.
//
//   dW[co][t][ci] = sum_G dZ[G][co] * X[G + off_t][ci],   off_t = (kh-1)*21 + (kw-1)
//
// G runs over the rows of the zero-bordered 21x21 frames of consecutive boards (frames are
// contiguous in memory, so G is a plain row index into both the dZ and the X frame
// arrays).  dZ is zero on every border position, so the product never leaks across a board
// edge and the 9 taps are 9 constant row shifts of ONE X window: per 32-row K-step a
// workgroup stages 32 new dZ rows and ~32 new X rows (a ring indexed by G mod 256) and runs
// all 9 taps against them.  The im2col wgrad (conv_mfma.hip, conv_wgrad_t3_kernel) stages
// X once per kernel row instead (64 KB of LDS-DMA per 384 MFMAs = 171 B/MFMA, its measured
// limiter); here it is 12 KB per 288 MFMAs = 43 B/MFMA.
//
// Per board the K-steps cover frame rows 1..19 only (G = b*441 + 21 + 32j, j < 13, 416 of
// 441 rows; the last step's tail is border row 20, zero in dZ), so the MFMA work is 416/361
// of the useful products.  Both operands are read with transposing LDS reads
// (ds_read_b64_tr_b16): rows = pixels (K), columns = channels.
//
// Workgroup = 4 waves, tile 64 co x 9 taps x 64 ci (wave wn: 64 co x 9 taps x 16 ci, 4 x 9
// accumulator fragments); grid = layers x co-chunks x ci-chunks x pixel splits, two
// workgroups per CU, XCD-remapped so the chunks of one (layer, split) share an L2.  Output:
// fp32 split slabs slab[z][co][t*Cx + ci] in the layout wgrad_reduce_multi sums.
//
// Reference semantics: SpatialConvolutionMM accGradParameters (experiments.lua:138, EXTERNAL
// nn) — the gradient of the 3x3 hidden convolutions of getBasicModel (experiments.lua:135-149).
#include "dg_common.h"

using namespace dg;

namespace {

constexpr int WF = 21;              // frame width (pad 1)
constexpr int WFF = WF * WF;        // 441 rows per board
constexpr int STEPS_PER_BOARD = 13; // 13 x 32 = 416 rows from frame row 1
constexpr int XR = 256;             // X ring rows (128 B each)
constexpr int XRING = XR * 128;     // 32 KB
constexpr int MAXL = 16;

struct WinLayers {
  const char* dZ[MAXL];
  const char* X[MAXL];
  float* slab[MAXL];
};

struct WinArgs {
  long long* sf;  // the fused update's step tag (dg_common.h): a slab value out of range sets it
  int M;       // dZ channels (co), multiple of 128
  int Mpad;    // slab rows
  int Cx;      // X channels (ci), multiple of 64
  int KP;      // slab row length (>= 9 * Cx)
  int B;       // boards
  int splits;  // pixel splits per (layer, chunk pair)
  int nl;      // layers
};

// 16-B slot swizzle of a 128-B X ring row: a 32-lane half of a transposing read takes rows
// {s..s+3, s+8..s+11} for ANY shift s (the 9 taps); this keeps its 256 B on 64 distinct
// banks (checked exhaustively over s and the chunk pair).
DG_DEV int xswz(int r) { return 2 * (((r >> 1) & 1) | (((r >> 3) & 1) << 1)); }

DG_DEV int step_g0(int s) {
  const int b = s / STEPS_PER_BOARD;
  return b * WFF + WF + 32 * (s - b * STEPS_PER_BOARD);
}

// ABL: ablation bits (diagnostics; 0 in production): 1 no MFMA, 2 no LDS reads, 4 no DMA,
// 8 X read addresses fixed per board (no per-step address VALU; wrong data), 16 no K-step
// barrier (races; timing only).
// PD: LDS-DMA prefetch distance in K-steps (dZ buffers = PD + 1; the X ring holds the
// current window plus PD steps ahead: <= 22 + 54 + 57 + 32 (PD - 1) + 8 rows < 256 for
// PD <= 4).  The DMAs are issued from inline asm (dma16) with hand vmcnt accounting: every
// wave issues exactly 2 per steady-state step (one dZ block, one X block; a wave with no
// new X block re-loads one that another wave loads, same bytes), so "DMAs of step st+1
// landed" = vmcnt(2 (PD - 1)).
//
// NW = 4 waves per workgroup: 64-co chunks, two independent workgroups per CU (their K-step
// barriers are not in lockstep, so one's LDS reads overlap the other's MFMAs); every wave
// owns 64 co x 9 taps x 16 ci.  (Measured and removed in round 4: 8-wave / 128-co
// workgroups, a software-pipelined K loop and prefetch distance 2 — all slower or equal,
// profiles/r1_kbench_wgrad_win_v5_swp.json, r3_wgrad_win_stream_experiments.txt.)
template <int ABL, int PD, int NW>
__global__ void __launch_bounds__(64 * NW, 8 / NW) conv_wgrad_win_kernel(WinArgs a, WinLayers Ls) {
  static_assert(PD >= 1 && PD <= 4, "prefetch distance");
  static_assert(NW == 4, "waves");
  constexpr int COCH = 16 * NW;        // co per workgroup (64 or 128)
  constexpr int DZR = 2 * COCH;        // dZ LDS row bytes
  constexpr int DZB = 32 * DZR;        // one dZ step (32 rows); NW 1-KB blocks
  __shared__ __attribute__((aligned(16))) char smem[XRING + (PD + 1) * DZB];
  char* xring = smem;
  char* dzbuf = smem + XRING;
  const uint32_t xring_u = (uint32_t)(uintptr_t)(LDS_AS char*)smem;
  const uint32_t dz_u = xring_u + XRING;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = 0, wn = wave;

  const int nci = a.Cx / 64, nco = a.M / COCH;
  const int nwg = a.nl * nco * nci * a.splits;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, xslot = bid >> 3;
  const int q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + xslot;
  const int coch = lid % nco;   // co chunks of one (layer, split) adjacent: same XCD / L2
  int rest = lid / nco;
  const int cich = rest % nci;
  rest /= nci;
  const int zsplit = rest % a.splits;
  const int layer = rest / a.splits;

  const char* __restrict__ dZl = Ls.dZ[layer] + coch * DZR;
  const char* __restrict__ Xl = Ls.X[layer] + cich * 128;
  const int Mb = a.M * 2, Xb = a.Cx * 2;
  const int Gmax = a.B * WFF;
  const int T = a.B * STEPS_PER_BOARD;
  const int s0 = (int)((long long)zsplit * T / a.splits);
  const int s1 = (int)((long long)(zsplit + 1) * T / a.splits);

  // one 1-KB block of X ring rows r0 .. r0+7
  auto x_block = [&](int r0) {
    if constexpr (ABL & 4) return;
    const int row = r0 + (lane >> 3);
    const int c = (lane & 7) ^ xswz(row & (XR - 1));
    int gr = row < 0 ? 0 : row;
    gr = gr >= Gmax ? Gmax - 1 : gr;
    dma16(Xl + (size_t)gr * Xb + c * 16,
          __builtin_amdgcn_readfirstlane(xring_u + (r0 & (XR - 1)) * 128));
  };
  // 32 dZ rows of step g0 into buffer buf: one 1-KB block per wave
  auto dz_block = [&](int buf, int g0) {
    if constexpr (ABL & 4) return;
    const int r = wave * 8 + (lane >> 3);
    const int c = (lane & 7) ^ xswz(r);
    dma16(dZl + (size_t)(g0 + r) * Mb + c * 16,
          __builtin_amdgcn_readfirstlane(dz_u + buf * DZB + wave * 1024));
  };
  int loaded_hi = 0;
  // steady-state issue for step sn into dZ buffer buf: 2 DMAs per wave (3 at a board's
  // first step)
  auto issue = [&](int sn, int buf) {
    const int g0n = step_g0(sn);
    int lo = (g0n - 22) & ~7;
    if (lo < loaded_hi) lo = loaded_hi;
    const int hi = (g0n + 54 + 7) & ~7;
    const int nblk = (hi - lo) >> 3;  // 4 .. 8 (4 inside a board, 7-8 across boards)
    // 1 X block per wave inside a board, 2 at a board's first step (7-8 new blocks; a wave
    // without an 8th block re-loads block 0, same bytes)
    x_block(lo + 8 * wave);
    if (nblk > 4) x_block(lo + 8 * (wave + 4 < nblk ? wave + 4 : 0));
    loaded_hi = hi;
    dz_block(buf, g0n);
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 2, pp = li & 3;
  const int p1 = pp >> 1, p0 = (pp & 1) * 8;

  if (s0 < s1) {
    const int g0 = step_g0(s0);
    const int lo = (g0 - 22) & ~7;
    loaded_hi = (g0 + 54 + 7) & ~7;
    for (int k = wave; k < ((loaded_hi - lo) >> 3); k += NW) x_block(lo + 8 * k);
    dz_block(0, g0);
    dma_wait<0>();
    __syncthreads();
#pragma unroll
    for (int p = 1; p < PD; ++p)
      if (s0 + p < s1) issue(s0 + p, p);
  }
  // Per-lane LDS read addresses.  dZ: fixed per (i, h) + the step's buffer base.  X: the
  // ring slot of tap t / half h is (g0 + off_t + rl) & 255 and its 16-B chunk is XOR-ed by
  // bits 1 and 3 of the slot; inside a board g0 advances by 32 (slot += 32 keeps bits 1, 3),
  // so the address is (rel + 4096 j) & 0x7fff with rel computed once per board.
  int rel_d[2][4];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rl = 8 * g + 4 * h + q;
    const int sw = xswz(rl);
#pragma unroll
    for (int i = 0; i < 4; ++i) rel_d[h][i] = rl * DZR + (((8 * wm + 2 * i + p1) ^ sw) * 16) + p0;
  }
  int rel_x[9][2];
  auto board_rel = [&](int gb) {
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int off = (t / 3 - 1) * WF + (t % 3 - 1);
        const int slot = (gb + off + 8 * g + 4 * h + q) & (XR - 1);
        rel_x[t][h] = slot * 128 + (((2 * wn + p1) ^ xswz(slot)) * 16) + p0;
      }
  };
  int bsteps = s0 / STEPS_PER_BOARD;           // board of step st
  int j = s0 - bsteps * STEPS_PER_BOARD;       // step within the board
  board_rel(bsteps * WFF + WF);
  int buf = 0;        // dZ buffer of step st
  int buf_pd = PD;    // dZ buffer of step st + PD
  // this wave's DMAs of step st+1 landed: the DMAs of steps st+2 .. st+PD may remain
  auto wait_next = [&](int st) {
    if (st + PD < s1) {
      // 2 per step, 3 at a board's first step (at most one in any 3 consecutive steps)
      const int r = (st + 2) % STEPS_PER_BOARD;
      if (r == 0 || r + PD - 2 >= STEPS_PER_BOARD)
        dma_wait<2 * (PD - 1) + 1>();
      else
        dma_wait<2 * (PD - 1)>();
    } else {
      dma_wait<0>();
    }
  };
  for (int st = s0; st < s1; ++st) {
    if (st + PD < s1) issue(st + PD, buf_pd);
    if (j == STEPS_PER_BOARD) {
      j = 0;
      ++bsteps;
      board_rel(bsteps * WFF + WF);
    }
    const int jo = j * 4096;
    const char* sD = dzbuf + buf * DZB;
    s16x4 ta[2][4], tb[2][9];
    if constexpr (ABL & 2) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int i = 0; i < 4; ++i) ta[h][i] = s16x4{};
#pragma unroll
        for (int t = 0; t < 9; ++t) tb[h][t] = s16x4{};
      }
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) ta[h][i] = lds_read_tr((const LDS_AS char*)(sD + rel_d[h][i]));
#pragma unroll
      for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          tb[h][t] = lds_read_tr((const LDS_AS char*)(
              xring + ((ABL & 8) ? rel_x[t][h] : ((rel_x[t][h] + jo) & (XRING - 1)))));
    }
    bf16x8 af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s16x4 lo = ta[0][i], hi = ta[1][i];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      af[i] = __builtin_bit_cast(bf16x8, v);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const s16x4 lo = tb[0][t], hi = tb[1][t];
      const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, v);
      if constexpr (ABL & 1) {
        asm volatile("" ::"v"(bfr));
      } else {
        if constexpr (ABL & 32) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i][t] = mfma16(af[i], bfr, acc[i][t]);
        if constexpr (ABL & 32) __builtin_amdgcn_s_setprio(0);
      }
    }
    wait_next(st);
    if constexpr (!(ABL & 16)) __syncthreads();
    buf = buf == PD ? 0 : buf + 1;
    buf_pd = buf_pd == PD ? 0 : buf_pd + 1;
    ++j;
  }

  float* slab = Ls.slab[layer] + (size_t)zsplit * a.Mpad * a.KP;
  // the step tag's range check: an unsigned max of the stored values' |v| bits, beside the
  // stores (NaN bits exceed every finite and infinite value)
  unsigned vmx = 0u;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = coch * COCH + wm * 64 + i * 16 + g * 4 + r;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int k = t * a.Cx + cich * 64 + wn * 16 + li;
        slab[(size_t)co * a.KP + k] = acc[i][t][r];
        vmx = max(vmx, __float_as_uint(acc[i][t][r]) & 0x7FFFFFFFu);
      }
    }
  }
  if (a.sf && vmx >= __float_as_uint(GRAD_BOUND)) flag_bad_step(a.sf);
}

int g_win_ablate = 0;
constexpr int WIN_NW = 4;
constexpr int WIN_PD = 4;

template <int ABL>
void launch_win(dim3 grid, const WinArgs& a, const WinLayers& Ls, hipStream_t stream) {
  hipLaunchKernelGGL((conv_wgrad_win_kernel<ABL, WIN_PD, WIN_NW>), grid, dim3(64 * WIN_NW), 0,
                     stream, a, Ls);
}

}  // namespace

extern "C" {

void dg_conv_wgrad_win_set_ablate(int mode) { g_win_ablate = mode; }

// Splits per (layer, chunk pair) that fill num_cus CUs in one round (8 / NW workgroups per
// CU).  At least 8 K-steps per split (the prologue loads a full window).
int dg_conv_wgrad_win_splits(int nl, int M, int Cx, int B, int num_cus) {
  const int pairs = nl * (M / (16 * WIN_NW)) * (Cx / 64);
  int s = pairs > 0 ? num_cus * (8 / WIN_NW) / pairs : 1;
  const int smax = B * STEPS_PER_BOARD / 8;
  if (s > smax) s = smax;
  return s < 1 ? 1 : s;
}

// table = nl rows of {dZ frame (pad 1, M channels), X frame (pad 1, Cx channels), slab}.
hipError_t dg_conv_wgrad_win(const long long* table, int nl, int M, int Mpad, int Cx, int B,
                             int KP, int splits, long long* sf, hipStream_t stream) {
  const int coch = 16 * WIN_NW;
  if (nl <= 0 || nl > MAXL || M % coch != 0 || Mpad < M || Cx % 64 != 0 || KP < 9 * Cx ||
      B <= 0 || splits <= 0 || splits > B * STEPS_PER_BOARD)
    return hipErrorInvalidValue;
  WinLayers Ls{};
  for (int i = 0; i < nl; ++i) {
    Ls.dZ[i] = (const char*)table[3 * i];
    Ls.X[i] = (const char*)table[3 * i + 1];
    Ls.slab[i] = (float*)table[3 * i + 2];
    if (!Ls.dZ[i] || !Ls.X[i] || !Ls.slab[i]) return hipErrorInvalidValue;
  }
  WinArgs a{sf, M, Mpad, Cx, KP, B, splits, nl};
  const dim3 grid(nl * (M / coch) * (Cx / 64) * splits);
  // d >= 256: s_setprio 1 around each tap's MFMAs (ABL bit 32).  This kernel is the step's
  // critical path there and the side stream's bias partials / 5x5 weight gradient share its
  // CUs: 12x256 bf16 +1.6%; at d = 128 the side chain is the critical one (-2.9%), and the
  // same priority on the MX-fp8 window kernel, the side kernels or the stacks measured equal
  // or slower (profiles/r4_s2_wave_priority_ab.txt)
  if (M >= 256 && (g_win_ablate & 31) == 0) {
    launch_win<32>(grid, a, Ls, stream);
    return hipGetLastError();
  }
  switch (g_win_ablate & 31) {
    case 0: launch_win<0>(grid, a, Ls, stream); break;
#define WIN_CASE(n) \
  case n:           \
    launch_win<n>(grid, a, Ls, stream); \
    break;
      WIN_CASE(1) WIN_CASE(2) WIN_CASE(3) WIN_CASE(4) WIN_CASE(5) WIN_CASE(6) WIN_CASE(7)
      WIN_CASE(8) WIN_CASE(12) WIN_CASE(16) WIN_CASE(20) WIN_CASE(22)
#undef WIN_CASE
  }
  return hipGetLastError();
}

}  // extern "C"
