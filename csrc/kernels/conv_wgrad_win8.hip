// MX-fp8 sliding-window weight gradient of 3x3 layers (BASELINE config 5's fp8 backward):
//
//   dW[co][t][ci] = s_dz * s_x * sum_G dz8[G][co] * x8[G + off_t][ci]
//
// on v_mfma_scale_f32_16x16x128_f8f6f4 (A = the e5m2 gradient frame dz8, B = the e4m3
// activation frame x8, fp32 accumulate; 2x the bf16 MFMA rate).  The fp8 frames are the
// bytes the fp8 layer stacks (conv_stack_f8.hip) already hold in their images — e4m3
// activations quantized with the next layer's input scale, e5m2 gradients with the layer's
// gradient scale, both powers of two — copied out beside the dequantized bf16 frames, so the
// weight gradient sees exactly the operands of the fp8 forward / backward-data chains; the
// per-tensor scales are applied to the fp32 sums at the slab write (exact: powers of two).
//
// Same geometry as the bf16 kernel (conv_wgrad_win.hip): G runs over the rows of the
// zero-bordered 21x21 frames of consecutive boards, dZ is zero on every border so the 9 taps
// are 9 row shifts of ONE X window, and a board is 13 sub-steps of 32 rows (frame rows 1..19).
// The fp8 frames are written with a pitch of 448 rows per board (441 + 7 zero rows): every
// sub-step then starts at a row = 21 (mod 32) and the LDS swizzle (bits 2..3 of the ring
// row) is the same for all of them, so a lane's 9 tap read offsets are fixed for the whole
// kernel and a sub-step only adds a wave-uniform row offset.
// One MFMA contracts K = 128 rows = 4 consecutive sub-steps (a "super-step", which may span
// two boards: the K order inside an MFMA is free as long as A and B agree):
//   MFMA K index 32 g + 8 r + q  <->  row 8 g + q of sub-step r of the super-step,
// for lane group g = lane >> 4 — exactly what one ds_read_b64_tr_b8 per sub-step r delivers
// (probed on gfx950, tools/tr8_probe.hip: per 16-lane group, lane 2q + p supplies the
// address of row q, bytes 8p..8p+7; lane i receives byte i of rows 0..7).
//
// LDS (one 8-wave workgroup = 64 co x 9 taps x 64 ci; wave (wm, wn) owns co half wm (32 co)
// x ci 16 wn .. +16; ~96 KB, one workgroup per CU, two waves per SIMD):
//   X ring   XR = 1024 rows x 64 B (64 ci) = 64 KB, slot = G & 1023, 16-B chunk c at
//            c ^ ((slot >> 2) & 3): any 16 consecutive rows hit 16 distinct 16-B bank groups
//            per chunk (the two tr-groups of a 32-lane half read rows 8g + q of one sub-step
//            = 16 consecutive rows), and +32 rows (the next sub-step of a board) keeps the
//            swizzle;
//   dZ       PD + 1 = 4 buffers of 128 rows x 64 B (64 co), row R = 32 r + i, same swizzle.
// DMA: every wave issues exactly PER = 3 LDS-DMAs per super-step (1 dZ + 2 X blocks of 1 KB;
// 8 dZ + 16 X blocks per workgroup, and a super-step needs at most 11 new X blocks: 128 rows,
// +32 across a board edge, +16 alignment — a wave without a block re-loads the first one,
// same bytes), so "super-step S+1 landed" with S+2 .. S+PD-1 still in flight =
// vmcnt(PER * (PD - 1)).  Prefetch distance PD = 3 (a template parameter, 2..4; 4 measured
// equal): the ring holds super-steps S .. S+PD, whose rows span at most (PD + 1) x (128 + 32)
// + 76 + 30 rows = 746 at PD 3, 906 at PD 4, < 1024 (static_assert below), so a DMA never
// overwrites rows a wave may still read.
// Output: fp32 split slabs slab[z][co][t*Cx + ci], the layout wgrad_reduce_multi sums (the
// bf16 kernel's), so the reduce, the bias gradients and the DP buckets are unchanged.
//
// Reference semantics: SpatialConvolutionMM accGradParameters of the hidden 3x3 layers
// (experiments.lua:135-149, EXTERNAL nn; the backward of train.lua:10).
#include <stdio.h>
#include <stdlib.h>

#include "dg_common.h"

using namespace dg;

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(2))) int i32x2;

namespace {

constexpr int WF = 21;
constexpr int FP = 448;           // fp8 frame pitch: rows per board (441 + 7 zero rows)
constexpr int SPB = 13;           // 32-row sub-steps per board (rows 21 .. 436)
constexpr int XR = 1024;          // X ring rows (64 B each)
constexpr int XRING = XR * 64;    // 64 KB
constexpr int PD_MAX = 4;         // DMA distance (super-steps): PD - 1 in flight beyond the next
constexpr int MAXL = 16;
// ring capacity at prefetch distance PD (see the header): PD + 1 super-steps of at most
// 128 + 32 rows each, plus the 76-row tap window and 30 rows of block alignment
static_assert((PD_MAX + 1) * (128 + 32) + 76 + 30 <= XR, "X ring capacity");

struct Win8Layers {
  const uint8_t* dZ[MAXL];   // e5m2 [B][448][M]
  const uint8_t* X[MAXL];    // e4m3 [B][448][Cx]
  float* slab[MAXL];
  const float* s_dz[MAXL];   // device scalars (powers of two)
  const float* s_x[MAXL];
};

struct Win8Args {
  long long* sf;   // the fused update's step tag (dg_common.h)
  int M, Mpad, Cx, KP, B, splits, nl;
};

DG_DEV int swz(int slot) { return (slot >> 2) & 3; }
DG_DEV int sub_g0(int s) {
  const int b = s / SPB;
  return b * FP + WF + 32 * (s - b * SPB);
}

DG_DEV i32x2 tr8(const LDS_AS char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((LDS_AS i32x2*)p);
}

// NW = 4: one wave per SIMD (the whole 512-register file), each wave 64 co x 9 taps x 16 ci;
// NW = 8: two waves per SIMD, each 32 co (co half wm) x 9 taps x 16 ci — a partner wave
// on the SIMD covers one wave's LDS reads / barrier.  The workgroup tile (64 co x 64 ci) and
// the DMA schedule (20 1-KB blocks per super-step: 8 dZ + 12 X) are the same.
// RA: B (X) fragments read RA taps ahead of their MFMAs (each tap's 4 tr8 reads then have
// RA x MI MFMAs to land)
// MODE: 0 in production; timing ablations (tools/kbench_win8.py, wrong results): 1 no MFMA,
// 2 no LDS fragment reads (register operands), 4 no LDS-DMA (nothing issued or waited for),
// 8 no slab store, 16 no per-super-step barrier.
// COT: the workgroup's co tile (64; the 128-co forms were removed in round 6, see WIN8_COT).
template <int NW, int RA, int PD, int MODE = 0, int COT = 64>
__global__ void __launch_bounds__(64 * NW, NW / 4) conv_wgrad_win8_kernel(Win8Args a, Win8Layers Ls) {
  static_assert(PD >= 2 && PD <= PD_MAX, "prefetch distance");
  static_assert(COT == 64, "co tile");
  constexpr int MI = COT / 16 / (NW / 4);   // 16-co accumulator fragments per wave
  constexpr int XPW = NW == 4 ? 3 : 2;   // X blocks per wave per super-step (12 | 16 >= 11)
  constexpr int DZB = 128 * COT;         // one super-step of dZ rows (8 | 16 KB)
  constexpr int DPW = COT / 8 / NW;      // dZ blocks (1 KB) per wave per super-step
  constexpr int PER = XPW + DPW;         // DMAs per wave per super-step
  constexpr int RPB = 1024 / COT;        // dZ rows per 1-KB block (16 | 8)
  constexpr int LPR = COT / 16;          // lanes per dZ row (4 | 8)
  static_assert(DPW * NW * RPB == 128, "dZ blocks");
  __shared__ __attribute__((aligned(16))) char smem[XRING + (PD + 1) * DZB];
  char* xring = smem;
  char* dzbuf = smem + XRING;
  const uint32_t xring_u = (uint32_t)(uintptr_t)(LDS_AS char*)smem;
  const uint32_t dz_u = xring_u + XRING;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave & 3;               // ci quarter (16 ci)
  const int wm = wave >> 2;              // co half (NW = 8)

  const int nci = a.Cx / 64, nco = a.M / COT;
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

  const uint8_t* __restrict__ dZl = Ls.dZ[layer] + coch * COT;
  // dZ ring-row swizzle (chunk c of buffer row R at c ^ dz_swz(R))
  auto dz_swz = [](int R) { return COT == 64 ? (R >> 2) & 3 : (R >> 1) & 7; };
  const uint8_t* __restrict__ Xl = Ls.X[layer] + cich * 64;
  const int Gmax = a.B * FP;
  const int TS = a.B * SPB / 4;                         // super-steps
  const int s0 = (int)((long long)zsplit * TS / a.splits);
  const int s1 = (int)((long long)(zsplit + 1) * TS / a.splits);

  // one 1-KB block of X ring rows r0 .. r0 + 15 (r0 a multiple of 16)
  auto x_block = [&](int r0) {
    const int row = r0 + (lane >> 2);
    const int slot = row & (XR - 1);
    const int c = (lane & 3) ^ swz(slot);
    int gr = row < 0 ? 0 : row;
    gr = gr >= Gmax ? Gmax - 1 : gr;
    dma16(Xl + (size_t)gr * a.Cx + c * 16,
          __builtin_amdgcn_readfirstlane(xring_u + (r0 & (XR - 1)) * 64));
  };
  // dZ rows of super-step S into buffer buf: 128 / RPB blocks of RPB rows (DPW per wave)
  auto dz_blocks = [&](int buf, int S) {
#pragma unroll
    for (int u = 0; u < DPW; ++u) {
      const int k = wave + NW * u;            // block: sub-step r, rows rr ..
      constexpr int BPS = 32 / RPB;           // blocks per 32-row sub-step
      const int r = k / BPS;
      const int rr = RPB * (k % BPS) + lane / LPR;
      const int R = 32 * r + rr;              // buffer row
      const int c = (lane % LPR) ^ dz_swz(R);
      const int g = sub_g0(4 * S + r) + rr;
      dma16(dZl + (size_t)g * a.M + c * 16,
            __builtin_amdgcn_readfirstlane(dz_u + buf * DZB + k * 1024));
    }
  };
  int loaded_hi = 0;
  // steady-state issue for super-step Sn into dZ buffer buf: exactly PER DMAs per wave
  auto issue = [&](int Sn, int buf) {
    const int lo0 = (sub_g0(4 * Sn) - 22) & ~15;
    const int lo = lo0 > loaded_hi ? lo0 : loaded_hi;
    const int hi = (sub_g0(4 * Sn + 3) + 54 + 15) & ~15;
    const int nblk = (hi - lo) >> 4;                       // <= 11
#pragma unroll
    for (int u = 0; u < XPW; ++u) {
      const int k = wave + NW * u;
      x_block(lo + 16 * (k < nblk ? k : 0));
    }
    loaded_hi = hi;
    dz_blocks(buf, Sn);
  };

  f32x4 acc[MI][9];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int li = lane & 15;
  const int g = lane >> 4;
  const int q = li >> 1, p = li & 1;

  // A (dZ) read addresses: buffer row R = 32 r + 8 g + q; its swizzle depends on bits 2..3
  // of 8 g + q only, so fragment i (chunk i) of sub-step r is at a_off ^ (16 i) + r * 2 KB
  int a_off;
  {
    const int R0 = 8 * g + q;
    a_off = R0 * COT + (dz_swz(R0) * 16) + 8 * p;
  }
  // B (X) read offsets: ring slot of row 21 + off_t + 8 g + q (board 0, sub-step 0); a
  // sub-step starting at row g0 adds (g0 - 21) rows (a multiple of 32: swizzle unchanged)
  const int rowq = WF + 8 * g + q;
  auto rel_of = [&](int t) {
    const int off = (t / 3 - 1) * WF + (t % 3 - 1);
    const int slot = (rowq + off) & (XR - 1);
    return slot * 64 + ((wn ^ swz(slot)) * 16) + 8 * p;
  };
  int rel[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) rel[t] = rel_of(t);

  if (s0 < s1 && !(MODE & 4)) {
    const int lo = (sub_g0(4 * s0) - 22) & ~15;
    loaded_hi = (sub_g0(4 * s0 + 3) + 54 + 15) & ~15;
    for (int k = wave; k < ((loaded_hi - lo) >> 4); k += NW) x_block(lo + 16 * k);
    dz_blocks(s0 % (PD + 1), s0);
    dma_wait<0>();
    __syncthreads();
#pragma unroll
    for (int pp = 1; pp < PD; ++pp)
      if (s0 + pp < s1) issue(s0 + pp, (s0 + pp) % (PD + 1));
  }

  for (int S = s0; S < s1; ++S) {
    if (!(MODE & 4) && S + PD < s1) issue(S + PD, (S + PD) % (PD + 1));
    int so[4];                             // wave-uniform ring byte offsets per sub-step
#pragma unroll
    for (int r = 0; r < 4; ++r)
      so[r] = __builtin_amdgcn_readfirstlane((sub_g0(4 * S + r) - WF) * 64);
    // A fragments: 4 chunks x 4 sub-steps
    const LDS_AS char* sD = (const LDS_AS char*)(dzbuf + (S % (PD + 1)) * DZB);
    i32x8 af[MI];
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int ig = wm * MI + i;          // the 16-co chunk of the 64-co tile
      i32x2 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = tr8(sD + (a_off ^ (16 * ig)) + r * 32 * COT);
      af[i] = i32x8{v[0].x, v[0].y, v[1].x, v[1].y, v[2].x, v[2].y, v[3].x, v[3].y};
      if constexpr ((MODE & 2) != 0) {
        int z = lane + ig;
        asm volatile("" : "+v"(z));
        af[i] = i32x8{z, z, z, z, z, z, z, z};
      }
    }
    auto read_b = [&](int t) -> i32x8 {
      if constexpr ((MODE & 2) != 0) {
        int z = lane + t;
        asm volatile("" : "+v"(z));
        return i32x8{z, z, z, z, z, z, z, z};
      }
      i32x2 v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        v[r] = tr8((const LDS_AS char*)(xring + ((rel[t] + so[r]) & (XRING - 1))));
      return i32x8{v[0].x, v[0].y, v[1].x, v[1].y, v[2].x, v[2].y, v[3].x, v[3].y};
    };
    // a tap's B reads issued RA taps ahead of its MFMAs (pinned by sched_barriers: left
    // alone the scheduler hoists all 36 reads to the top)
    i32x8 bb[9];
#pragma unroll
    for (int t = 0; t < RA; ++t) bb[t] = read_b(t);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + RA < 9) bb[t + RA] = read_b(t + RA);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        if constexpr ((MODE & 1) != 0)
          asm volatile("" ::"v"(af[i]), "v"(bb[t]));
        else
          acc[i][t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[i], bb[t], acc[i][t],
                                                                       1, 0, 0, 127, 0, 127);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // this wave's DMAs of super-step S + 1 landed (those of S + 2 .. S + PD may remain),
    // then every wave's (barrier): the next super-step's rows are visible and S's free
    if constexpr (!(MODE & 4)) {
      // in flight beyond S + 1: super-steps S + 2 .. min(S + PD, s1 - 1)
      const int ahead = min(PD - 1, s1 - S - 2);
      if (ahead >= PD - 1)
        dma_wait<PER * (PD - 1)>();
      else if (ahead == 2)
        dma_wait<2 * PER>();
      else if (ahead == 1)
        dma_wait<PER>();
      else
        dma_wait<0>();
    }
    if constexpr (!(MODE & 16)) __syncthreads();
  }

  const float scale = *Ls.s_dz[layer] * *Ls.s_x[layer];
  float* slab = Ls.slab[layer] + (size_t)zsplit * a.Mpad * a.KP;
  // the step tag's range check on the stored values themselves: an unsigned max of their |v|
  // bits (NaN bits exceed every finite and infinite value) — checked after the stores, the
  // accumulators stayed live past them (181 -> 212 VGPRs)
  unsigned vmx = 0u;
#pragma unroll
  for (int i = 0; i < MI; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int co = coch * COT + (wm * MI + i) * 16 + g * 4 + r;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int k = t * a.Cx + cich * 64 + wn * 16 + li;
        const float v = acc[i][t][r] * scale;
        if constexpr ((MODE & 8) != 0)
          asm volatile("" ::"v"(v));
        else
          slab[(size_t)co * a.KP + k] = v;
        vmx = max(vmx, __float_as_uint(v) & 0x7FFFFFFFu);
      }
    }
  }
  if (a.sf && vmx >= __float_as_uint(GRAD_BOUND)) flag_bad_step(a.sf);
}

}  // namespace

int g_win8_ablate = 0;
// workgroup co tile: 64.  (The 128-co tiles — 8 waves with 4 fragments each, or 4 waves with
// the whole register file — were 8-13% faster alone but 6-9% slower in the step: 128 KB of
// LDS per workgroup left no room for the side-stream kernels; removed in round 6,
// profiles/r5_win8_ablation.txt.)
constexpr int WIN8_COT = 64;

extern "C" {

// Splits per (layer, chunk pair): one 8-wave workgroup per CU, so the launch runs in
// rounds of num_cus workgroups.  Cost model in super-step times (~0.55 us): rounds x
// super-steps per workgroup, plus each workgroup's 147 KB fp32 slab written and reduced
// (~0.11 of a super-step of the whole machine).  d = 256 (160 pairs): 3 splits = 2 rounds
// (256 + 224) of 278 super-steps; d = 128 (40 pairs): 6 splits = 1 round of 139 (1 split
// would leave 96 CUs idle; a perfect fill at 8 / 32 splits writes 2.7x / 5x the slabs).
int dg_conv_wgrad_win8_splits(int nl, int M, int Cx, int B, int num_cus) {
  const int cot = WIN8_COT;
  const int pairs = nl * (M / cot) * (Cx / 64);
  const int TS = B * SPB / 4;
  if (pairs <= 0 || num_cus <= 0) return 1;
  int best = 1;
  double best_t = -1.0;
  for (int s = 1; s <= 32 && s <= TS / 4; ++s) {
    const long long rounds = (pairs * (long long)s + num_cus - 1) / num_cus;
    const double t = (double)(rounds * ((TS + s - 1) / s)) + 0.11 * (cot / 64) * pairs * s;
    if (best_t < 0 || t < best_t) {
      best_t = t;
      best = s;
    }
  }
  return best;
}

// table = nl rows of {dZ8 frame (pad 1, M channels, e5m2), X8 frame (pad 1, Cx channels,
// e4m3), slab, s_dz, s_x} (int64)
hipError_t dg_conv_wgrad_win8(const long long* table, int nl, int M, int Mpad, int Cx, int B,
                              int KP, int splits, long long* sf, hipStream_t stream) {
  const int cot = WIN8_COT;
  if (nl <= 0 || nl > MAXL || M % cot != 0 || Mpad < M || Cx % 64 != 0 || KP < 9 * Cx ||
      B <= 0 || B % 4 != 0 || splits <= 0 || splits > B * SPB / 4)
    return hipErrorInvalidValue;
  Win8Layers Ls{};
  for (int i = 0; i < nl; ++i) {
    const long long* r = table + 5 * i;
    Ls.dZ[i] = (const uint8_t*)r[0];
    Ls.X[i] = (const uint8_t*)r[1];
    Ls.slab[i] = (float*)r[2];
    Ls.s_dz[i] = (const float*)r[3];
    Ls.s_x[i] = (const float*)r[4];
    if (!Ls.dZ[i] || !Ls.X[i] || !Ls.slab[i] || !Ls.s_dz[i] || !Ls.s_x[i])
      return hipErrorInvalidValue;
  }
  Win8Args a{sf, M, Mpad, Cx, KP, B, splits, nl};
  const dim3 grid(nl * (M / cot) * (Cx / 64) * splits);
  // (8 waves: the 4-wave variant, 1 wave per SIMD with the whole register file, measured
  // the same — profiles/r3_fp8_wgrad_ab.txt)
  // (B reads 2 taps ahead measured the same as 1: profiles/r4_s1_fused_update_and_fp8_bisection.txt)
  // prefetch distance 3: 4 measured equal (12x256 fp8 133.7k vs 133.9k,
  // profiles/r4_s2_sr_hash_win8_pd_ab.txt)
  switch (g_win8_ablate) {   // (timing ablations: tools/kbench_win8.py)
#define DG_W8(m) \
  case m: hipLaunchKernelGGL((conv_wgrad_win8_kernel<8, 1, 3, m>), grid, dim3(512), 0, stream, a, Ls); break;
    DG_W8(1) DG_W8(2) DG_W8(3) DG_W8(4) DG_W8(6) DG_W8(7) DG_W8(8) DG_W8(16) DG_W8(20) DG_W8(31)
#undef DG_W8
    default:
      hipLaunchKernelGGL((conv_wgrad_win8_kernel<8, 1, 3>), grid, dim3(512), 0, stream, a, Ls);
  }
  return hipGetLastError();
}

void dg_conv_wgrad_win8_set_ablate(int mode) { g_win8_ablate = mode; }

}  // extern "C"
