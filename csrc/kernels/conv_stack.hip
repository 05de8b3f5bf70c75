// Fused run of hidden 3x3 layers (C -> C, C = 128, pad 1), board-resident in LDS: the
// whole forward stack, or the whole backward-data (dgrad) chain, in ONE launch.
//
// Per-layer kernels (conv_board.hip) end every layer with a burst of 23.6 MB of stores
// from all workgroups at once, plus a prologue that re-reads the same activation from HBM;
// ablations (profiles/) put that epilogue/prologue at ~14 of ~32 us per layer, and it
// cannot overlap with anything because every workgroup reaches it at the same time.
// A conv layer (and its transposed-weight dgrad) only mixes pixels of ONE board, so a
// workgroup that owns a board can run the next layer without any grid-wide sync.
//
// Here one workgroup owns one board for ALL layers of the run:
//   * the board's zero-bordered 21x21x128 frame lives in LDS (two 64-channel halo images,
//     112 KB, XOR-swizzled 128-B rows — the conv_board layout);
//   * each layer is 18 K-steps (2 chunks x 9 taps) of v_mfma_f32_16x16x32_bf16 over that
//     image; weight tiles [128 co][64 k] stream through a 3-deep LDS ring by LDS-DMA,
//     issued two steps ahead (across layer boundaries) and retired with a COUNTED
//     s_waitcnt vmcnt(2) + raw s_barrier, so a tile's L2 latency has two steps to land and
//     the barrier never drains the newest DMA (a __syncthreads() would: vmcnt(0));
//   * the epilogue writes the layer's bf16 output straight back INTO the LDS image (it is
//     the next layer's input):
//       EPI_FWD   : + (bias + pos-bias) table, ReLU          (forward; writes ReLU bitmask)
//       EPI_DGRAD : * ReLU bitmask of the layer below       (dZ_{i-1} = mask * W_i^T dZ_i)
//     and the global store of that output (activation / gradient frame for the wgrads,
//     plus the forward's bitmask) is spread over the next layer's first 12 K-steps,
//     underneath its MFMAs.
// Only the first input load and the last layer's stores are exposed.
//
// LDS: 3 x 16 KB weight ring + 2 x 56 KB images = 160 KB (the whole CU): one workgroup of
// 8 waves per CU, one board per workgroup.
//
// Reference ops: nn.SpatialZeroPadding + SpatialConvolutionMM + Add + ReLU per layer
// (experiments.lua:137-147) and their backward through the stack (train.lua:10).
#include <stdlib.h>

#include "dg_common.h"
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
constexpr int UNITS = NPTS * 16;          // 16-B output pieces of one board (5776)
constexpr int MAXL = 24;
constexpr int BM = 128;
constexpr int A_BYTES = BM * 128;         // [128 co][64 k] bf16
constexpr int MF = 4;                     // 64 co per wave (4 fragments of 16)

// Image swizzle: the 16-B slot of 8-channel group g in frame row f is g ^ sig(f) with
// sig(f) = (x + 3y) & 7, (y, x) = (f / 21, f % 21).  The plain f & 7 (conv_board) is
// conflict-free for 16 consecutive rows, but a 16-pixel B fragment crosses a board-row
// wrap (+2 frame rows) in 3 of 4 cases: 75% of the fragment reads were 2-way bank
// conflicts (avg 1.75 LDS cycles per lane group, modelled over every tap / fragment);
// (x + 3y) & 7 brings that to 1.04.  Linear in (x, y), so a tap shift (dh, dw) adds the
// uniform dw + 3 dh.
DG_DEV int fsig(int f) { return ((f % F) + 3 * (f / F)) & 7; }

struct StackLayer {
  const bf16_t* A;      // [128][KP] weights, k = tap*128 + ci (dgrad: flipped, transposed)
  const bf16_t* pbias;  // EPI_FWD: bf16 bias + pos-bias in fragment order (weight_refresh's
                        // pbias_frag: [24][2][4][64] x 4 bf16)
  char* Y;              // output frame [B][21][21][128] bf16
  uint8_t* mask;        // [B][361][16] ReLU bits: EPI_FWD writes (optional), EPI_DGRAD reads
};
struct StackArgs {
  const char* X0;       // input frame [B][21][21][128] bf16 of the first layer
  int nl, KP;
  StackLayer L[MAXL];
  unsigned long long* prof;  // ABL & 32: per-wave phase cycle sums [B][8 waves][8]
  int stagger;               // unused (copy-out reads are now pipelined one step ahead)
  int fuse_head;             // EPI_FWD, 8 waves: run the policy head on the final image
  dghead::HeadMArgs head;    // (head_body.h; X unused: the image is resident)
};

// NRING: weight-tile ring depth (tiles are issued NRING-1 steps ahead).
// ABL: timing ablations for tools/kbench_stack.py (0 in production): 1 no MFMA, 2 no
// fragment LDS reads, 4 no weight DMA, 8 no in-loop copy-out, 16 no per-step barrier.
template <int EPI, int NRING, int ABL, bool BPF = true, int NW = 8>
__global__ void __launch_bounds__(NW * 64) conv_stack_kernel(StackArgs a) {
  // NW waves: 2 (co halves) x NW/2 pixel groups; 8 waves: 64 co x 96 px per wave (2 per
  // SIMD), 16 waves: 64 co x 48 px per wave (4 per SIMD, half the accumulators)
  constexpr int NT = NW * 64;
  constexpr int WN = NW / 2;
  constexpr int NF = 24 / WN;
  constexpr int DMA_PER_TILE = 16 / NW;
  constexpr int AHEAD = NRING - 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int b = blockIdx.x;
  char* sA0 = smem;
  char* sH = smem + NRING * A_BYTES;  // image c at sH + c * H_BYTES
  const int g_src = (lane & 7) ^ (lane >> 3);
  const int total = a.nl * NSTEP;     // global K-steps over all layers

  // weight tile of global step g into ring slot g % NRING: exactly DMA_PER_TILE LDS-DMA
  // instructions per wave, issued from inline asm (dma16) so the compiler's waitcnt pass
  // does not drain them in front of the copy-out's LDS reads; retired by dma_wait below
  const uint32_t lds0 = (uint32_t)(uintptr_t)(LDS_AS char*)smem;
  // per-lane part of the weight-tile source address (row r of the tile, swizzled group)
  const uint32_t a_lane0 =
      (uint32_t)((((wave * DMA_PER_TILE) * 8 + (lane >> 3)) * a.KP + g_src * 8) * 2);
  const uint32_t a_lane1 = a_lane0 + (uint32_t)(8 * a.KP * 2);
  // tile (layer weights A, step s of that layer) into ring slot `slot`
  auto stage_A_at = [&](const bf16_t* A, int s, int slot) {
    if (ABL & 4) return;
    const int c = s / T, t = s - (s / T) * T;
    const char* Ak = (const char*)A + (t * C + c * 64) * 2;
    const uint32_t dst = lds0 + slot * A_BYTES;
    dma16(Ak + a_lane0, __builtin_amdgcn_readfirstlane(dst + (wave * DMA_PER_TILE) * 1024));
    if constexpr (DMA_PER_TILE == 2)
      dma16(Ak + a_lane1, __builtin_amdgcn_readfirstlane(dst + (wave * 2 + 1) * 1024));
  };
  auto stage_A = [&](int g) {
    if (ABL & 4) return;
    const int l = g / NSTEP, s = g - l * NSTEP;
    const int c = s / T, t = s - (s / T) * T;
    const int kcol = t * C + c * 64;
    const bf16_t* A = a.L[l].A;
    const uint32_t dst = lds0 + (g % NRING) * A_BYTES;
#pragma unroll
    for (int i = 0; i < DMA_PER_TILE; ++i) {
      const int r = (wave * DMA_PER_TILE + i) * 8 + (lane >> 3);
      dma16((const char*)A + ((size_t)r * a.KP + kcol + g_src * 8) * 2,
            __builtin_amdgcn_readfirstlane(dst + (wave * DMA_PER_TILE + i) * 1024));
    }
  };

  // ---- prologue: the first layer's input frame (both images) + weight tiles 0, 1 ----
  {
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
    for (int g = 0; g < AHEAD && g < total; ++g) stage_A(g);
  }
  __syncthreads();

  const int lr = lane & 15;
  const int lq = lane >> 4;
  int fp[NF], fs[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = wn * NF * 16 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    fp[j] = (h + 1) * F + (w + 1);
    fs[j] = (w + 1) + 3 * (h + 1);  // fsig(fp[j]) before the & 7
  }

  // Copy-out of the previous layer's output (resident in the image) to HBM, one 16-B piece
  // (8 channels of one pixel) per thread and K-step: the piece of step s is READ from LDS
  // during step s-1 and STORED in step s, so no wave blocks on that read's latency in front
  // of its MFMAs (a read+store in one step cost a full LDS round trip per step: ~10% of
  // the layer).  Thread tid always handles channel piece q = tid & 15 of pixels
  // p = tid / 16 + 32 s (NT = 512).
  const int co_q = tid & 15;
  auto co_addr = [&](int s_, int& f) {
    const int p = (tid >> 4) + 32 * s_;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    f = (h + 1) * F + (w + 1);
    return sH + (co_q >> 3) * H_BYTES + f * 128 + (((co_q & 7) ^ fsig(f)) * 16);
  };
  auto co_read = [&](int s_) -> uint4 {
    int f;
    return *(const uint4*)co_addr(s_, f);
  };
  auto co_store = [&](int s_, const uint4& v, const StackLayer& Lo) {
    const int p = (tid >> 4) + 32 * s_;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    *(uint4*)(Lo.Y + ((size_t)(b * FF + f) * C) * 2 + co_q * 16) = v;
    if (EPI == EPI_FWD && Lo.mask) {
      // bit per nonzero bf16 half (as the gates test it): packed min(x, 1) per half
      typedef unsigned short us2 __attribute__((ext_vector_type(2)));
      auto nz2 = [](uint32_t x) {
        const us2 m = __builtin_elementwise_min(__builtin_bit_cast(us2, x), us2{1, 1});
        const uint32_t t = __builtin_bit_cast(uint32_t, m);
        return (t | (t >> 15)) & 3u;
      };
      Lo.mask[((size_t)b * NPTS + p) * 16 + co_q] =
          (uint8_t)(nz2(v.x) | (nz2(v.y) << 2) | (nz2(v.z) << 4) | (nz2(v.w) << 6));
    }
  };
  auto copy_out = [&](int u, const StackLayer& Lo) {  // exposed (last layer): direct
    const int s_ = (u - tid) / NT;
    co_store(s_, co_read(s_), Lo);
  };
  constexpr int CO_STEPS = (UNITS + NT - 1) / NT;  // 12


  auto read_A = [&](const char* sA, int kk, bf16x8 (&af)[MF]) {
    const int g = kk * 4 + lq;
#pragma unroll
    for (int i = 0; i < MF; ++i) {
      const int row = wm * 64 + i * 16 + lr;
      af[i] = (ABL & 2) ? bf16x8{}
              : lds_read_b128((const LDS_AS char*)(sA + row * 128 + ((g ^ (row & 7)) * 16)));
    }
  };
  auto read_B = [&](int s_, int kk, bf16x8 (&bfr)[NF]) {
    const int c = s_ / T, t = s_ - (s_ / T) * T;
    const char* sHc = sH + c * H_BYTES;
    const int toff = (t / 3 - 1) * F + (t % 3 - 1);
    const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
    const int g = kk * 4 + lq;
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int row = fp[j] + toff;
      bfr[j] = (ABL & 2) ? bf16x8{}
               : lds_read_b128((const LDS_AS char*)(sHc + row * 128 +
                                                   ((g ^ ((fs[j] + tsig) & 7)) * 16)));
    }
  };
  auto mma = [&](const bf16x8 (&af)[MF], const bf16x8 (&bfr)[NF], f32x4 (&acc)[MF][NF]) {
    if constexpr ((ABL & 1) != 0) {
#pragma unroll
      for (int i = 0; i < MF; ++i) asm volatile("" ::"v"(af[i]));
#pragma unroll
      for (int j = 0; j < NF; ++j) asm volatile("" ::"v"(bfr[j]));
    } else {
#pragma unroll
      for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };
  bf16x8 bpre[NF];
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp0 = 0, te0 = 0;
  (void)tp0;
  (void)te0;

  int gs = 0;  // global step
  for (int l = 0; l < a.nl; ++l) {
    const StackLayer L = a.L[l];
    const bf16_t* A_next = l + 1 < a.nl ? a.L[l + 1].A : L.A;
    const StackLayer Lprev = a.L[l > 0 ? l - 1 : 0];
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (BPF) read_B(0, 0, bpre);  // image of this layer is ready (barrier)
    const bool co_on = !(ABL & 8) && l > 0;
    uint4 co_v = uint4{0, 0, 0, 0};
    if (co_on && (tid >> 4) < NPTS) co_v = co_read(0);
    for (int s = 0; s < NSTEP; ++s, ++gs) {
      if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); tp0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); }
      // k-half 0's A fragments first (tile gs landed: barrier above): their LDS latency hides
      // under the copy-out store and the weight-DMA issue below instead of stalling the
      // first MFMA (the DMA is inline asm: the compiler inserts no vmcnt wait for it)
      const char* sA = sA0 + (gs % NRING) * A_BYTES;
      bf16x8 af[MF], bfr[NF];
      read_A(sA, 0, af);
      // the previous layer's output (already in the image) goes to HBM under this layer's
      // MFMAs: 512 pieces per step over the first 12 steps.  Issued BEFORE the weight DMA:
      // hipcc puts an s_waitcnt vmcnt(0) in front of an LDS read that follows an LDS-DMA
      // (it cannot prove they do not alias), which would expose the DMA's latency.
      // waves 0-3 copy out before their k-half-0 MFMAs, waves 4-7 (the other wave of each
      // SIMD) after them: one wave of every SIMD always has MFMAs to issue meanwhile
      if (co_on && s < CO_STEPS && (tid >> 4) + 32 * s < NPTS) co_store(s, co_v, Lprev);
      // ring slot (gs+AHEAD)%NRING was last read in step gs-1: every wave passed the
      // barrier after it
      const bool more = gs + AHEAD < total;
      // (no dynamic kernel-argument indexing in the loop: a.L[l + 1].A is hoisted below)
      if (more) {
        if (s + AHEAD < NSTEP) stage_A_at(L.A, s + AHEAD, (gs + AHEAD) % NRING);
        else stage_A_at(A_next, s + AHEAD - NSTEP, (gs + AHEAD) % NRING);
      }
      if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[0] += t - tp0; tp0 = t; __builtin_amdgcn_sched_barrier(0); }
      // k-half 0: B fragments were prefetched during the previous step (BPF)
      if constexpr (BPF) {
#pragma unroll
        for (int j = 0; j < NF; ++j) bfr[j] = bpre[j];
      } else {
        read_B(s, 0, bfr);
      }
      mma(af, bfr, acc);
      // 16 waves (4 per SIMD, 128 VGPRs): keep k-half 1's reads below these MFMAs (the other
      // waves of the SIMD hide their latency) instead of two live fragment sets
      if constexpr (NW == 16) __builtin_amdgcn_sched_barrier(0);
      // next step's copy-out piece, read under this step's k-half-1 MFMAs
      if (co_on && s + 1 < CO_STEPS && (tid >> 4) + 32 * (s + 1) < NPTS) co_v = co_read(s + 1);
      if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[1] += t - tp0; tp0 = t; __builtin_amdgcn_sched_barrier(0); }
      // k-half 1, and the next step's k-half-0 B fragments (the image is resident: no DMA
      // dependency) issued before these MFMAs so their LDS latency hides under them
      read_A(sA, 1, af);
      read_B(s, 1, bfr);
      if (BPF && s + 1 < NSTEP) read_B(s + 1, 0, bpre);
      mma(af, bfr, acc);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((ABL & 32) != 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[2] += t - tp0; tp0 = t; __builtin_amdgcn_sched_barrier(0); }
      // tile gs+1 must have landed for every wave; the newer tiles (the newest
      // DMA_PER_TILE*(AHEAD-1) VMEM ops of this wave — the copy-out stores precede them)
      // may stay in flight
      if (more) dma_wait<DMA_PER_TILE * (AHEAD - 1)>(); else dma_wait<0>();
      if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[3] += t - tp0; tp0 = t; __builtin_amdgcn_sched_barrier(0); }
      if (!(ABL & 16)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((ABL & 32) != 0) { const unsigned long long t = __builtin_amdgcn_s_memtime(); ph[4] += t - tp0; tp0 = t; __builtin_amdgcn_sched_barrier(0); }
    }

    // ---- epilogue: write the layer's output back into the LDS image ----
    // (every wave is past its last read of the image: barrier above)
    if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); te0 = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); }
    // every global load of the epilogue is issued before the first use (one latency, not
    // 24 dependent ones: the phase timer put the old loop at 12.5k cycles per layer)
    uint2 eu[NF][EPI == EPI_FWD ? MF : 1];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = min(wn * NF * 16 + j * 16 + lr, NPTS - 1);
      if constexpr (EPI == EPI_FWD) {
        // fragment-ordered table (weight_refresh writes it): 512 contiguous bytes per load;
        // the [361][128] table read with this lane mapping touched 16 rows per load (4x
        // the L2 traffic; the phase timer put the epilogue at 12.5k cycles per layer)
        const uint2* pf = (const uint2*)L.pbias + ((wn * NF + j) * 2 + wm) * 4 * 64 + lane;
#pragma unroll
        for (int i = 0; i < MF; ++i) eu[j][i] = pf[i * 64];
      } else {  // 64 channel bits of this wave's image half
        eu[j][0] = *(const uint2*)(L.mask + ((size_t)b * NPTS + p) * 16 + wm * 8);
      }
    }
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = wn * NF * 16 + j * 16 + lr;
      const int f = fp[j];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int cl = i * 16 + lq * 4;  // channel within the wave's 64-channel image
        f32x4 v = acc[i][j];
        if constexpr (EPI == EPI_FWD) {
          const uint2 u = eu[j][i];
          v[0] = fmaxf(v[0] + __uint_as_float(u.x << 16), 0.f);
          v[1] = fmaxf(v[1] + __uint_as_float(u.x & 0xFFFF0000u), 0.f);
          v[2] = fmaxf(v[2] + __uint_as_float(u.y << 16), 0.f);
          v[3] = fmaxf(v[3] + __uint_as_float(u.y & 0xFFFF0000u), 0.f);
        } else {
          const uint32_t word = (cl < 32) ? eu[j][0].x : eu[j][0].y;
          const uint32_t bits = word >> ((cl & 31) >> 3 << 3) >> (cl & 4);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = ((bits >> r) & 1u) ? v[r] : 0.f;
        }
        uint2 o;
        o.x = pack_bf16x2(v[0], v[1]);
        o.y = pack_bf16x2(v[2], v[3]);
        const int slot = (cl >> 3) ^ (fs[j] & 7);
        if (p < NPTS) *(uint2*)(sH + wm * H_BYTES + f * 128 + slot * 16 + (cl & 4) * 2) = o;
      }
    }
    __syncthreads();
    if constexpr ((ABL & 32) != 0) { __builtin_amdgcn_sched_barrier(0); ph[5] += __builtin_amdgcn_s_memtime() - te0; __builtin_amdgcn_sched_barrier(0); }
  }
  // last layer's output: exposed copy-out
  for (int u = tid; u < UNITS; u += NT) copy_out(u, a.L[a.nl - 1]);
  // the policy head on the board image that is already in LDS (no re-staging, no launch):
  // its scratch (weights, logits, frame-shaped dz) goes into the idle weight ring
  if constexpr (EPI == EPI_FWD && NW == 8 && ABL == 0) {
    static_assert(dghead::scratch_bytes(C) <= NRING * (size_t)A_BYTES, "head scratch");
    if (a.fuse_head) dghead::head_body<C>(a.head, b, sH, smem, [](int) {});
  }
  if constexpr ((ABL & 32) != 0) {
    if (lane == 0 && a.prof) {
      ph[6] = (unsigned long long)a.nl * NSTEP;
#pragma unroll
      for (int k = 0; k < 8; ++k) a.prof[((size_t)b * 8 + wave) * 8 + k] = ph[k];
    }
  }
}

template <int EPI, int NRING, int ABL, bool BPF = true, int NW = 8>
hipError_t launch_stack(const StackArgs& a, int B, hipStream_t stream) {
  constexpr size_t lds = NRING * (size_t)A_BYTES + 2 * (size_t)H_BYTES;
  static_assert(lds <= 160 * 1024, "LDS");
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_stack_kernel<EPI, NRING, ABL, BPF, NW>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL((conv_stack_kernel<EPI, NRING, ABL, BPF, NW>), dim3(B), dim3(NW * 64), lds,
                     stream, a);
  return hipGetLastError();
}

template <int NRING>
hipError_t dispatch_ablate(int ablate, const StackArgs& a, int B, hipStream_t s) {
  switch (ablate) {  // forward only; see tools/kbench_stack.py
    case 1: return launch_stack<EPI_FWD, NRING, 1>(a, B, s);
    case 2: return launch_stack<EPI_FWD, NRING, 2>(a, B, s);
    case 4: return launch_stack<EPI_FWD, NRING, 4>(a, B, s);
    case 8: return launch_stack<EPI_FWD, NRING, 8>(a, B, s);
    case 16: return launch_stack<EPI_FWD, NRING, 16>(a, B, s);
    case 6: return launch_stack<EPI_FWD, NRING, 6>(a, B, s);
    case 12: return launch_stack<EPI_FWD, NRING, 12>(a, B, s);
    case 14: return launch_stack<EPI_FWD, NRING, 14>(a, B, s);
    case 32: return launch_stack<EPI_FWD, NRING, 32>(a, B, s);
    case 40: return launch_stack<EPI_FWD, NRING, 40>(a, B, s);
    default: return hipErrorInvalidValue;
  }
}


}  // namespace

static int g_stack_ablate = 0;
static int g_stack_stagger = -1;
static unsigned long long* g_stack_prof = nullptr;
static int g_stack_ring = 0;  // 0: default (2)
static int g_stack_bpf = 1;   // B-fragment prefetch across K-steps
static int g_stack_waves = 8; // waves per workgroup (8 or 16)

extern "C" {

void dg_conv_stack_set_ablate(int mode) { g_stack_ablate = mode; }
void dg_conv_stack_set_stagger(int on) { g_stack_stagger = on; }
void dg_conv_stack_set_prof(void* p) { g_stack_prof = (unsigned long long*)p; }
void dg_conv_stack_set_ring(int n) { g_stack_ring = n; }
void dg_conv_stack_set_bpf(int on) { g_stack_bpf = on; }
void dg_conv_stack_set_waves(int n) { g_stack_waves = n; }

// table: nl rows of {A, pbias, Y, mask} (int64 pointers)
//   epi 1 (forward): pbias required, mask optional (written)
//   epi 2 (dgrad)  : mask required (read; ReLU bits of the layer below), pbias unused
hipError_t dg_head_mfma(int C, const void* X, int B, const float* w, const float* bias,
                        const float* posb, const int* labels, float* loss, int* pred,
                        float* logp_out, void* dZ, float* gw_part, float* dzb, int head_relu,
                        float grad_scale, hipStream_t stream);

static hipError_t stack_launch(int epi, const long long* table, int nl, const void* X0, int KP,
                               int B, const dghead::HeadMArgs* head, hipStream_t stream) {
  if (nl <= 0 || nl > MAXL || KP < T * C || KP % 64 != 0 || B <= 0) return hipErrorInvalidValue;
  if (epi != EPI_FWD && epi != EPI_DGRAD) return hipErrorInvalidValue;
  StackArgs a;
  a.fuse_head = 0;
  a.head = dghead::HeadMArgs{};
  a.X0 = (const char*)X0;
  a.nl = nl;
  a.KP = KP;
  a.prof = g_stack_prof;
  if (g_stack_stagger < 0) {
    const char* e = getenv("DG_STACK_STAGGER");
    g_stack_stagger = e ? atoi(e) : 0;
  }
  a.stagger = g_stack_stagger;
  for (int i = 0; i < nl; ++i) {
    a.L[i].A = (const bf16_t*)table[4 * i];
    a.L[i].pbias = (const bf16_t*)table[4 * i + 1];
    a.L[i].Y = (char*)table[4 * i + 2];
    a.L[i].mask = (uint8_t*)table[4 * i + 3];
    if (!a.L[i].A || !a.L[i].Y) return hipErrorInvalidValue;
    if (epi == EPI_FWD && !a.L[i].pbias) return hipErrorInvalidValue;
    if (epi == EPI_DGRAD && !a.L[i].mask) return hipErrorInvalidValue;
  }
  const int nring = g_stack_ring ? g_stack_ring : 2;
  if (head) {
    if (epi != EPI_FWD) return hipErrorInvalidValue;
    if (g_stack_ablate || g_stack_waves == 16) {
      // variants without the fused head: the stack, then the standalone head kernel
      const hipError_t e = stack_launch(epi, table, nl, X0, KP, B, nullptr, stream);
      if (e != hipSuccess) return e;
      const dghead::HeadMArgs& h = *head;
      return dg_head_mfma(C, a.L[nl - 1].Y, B, h.w, h.bias, h.posb, h.labels, h.loss, h.pred,
                          h.logp_out, h.dZ, h.gw_part, h.dzb, h.head_relu, h.grad_scale, stream);
    }
    a.fuse_head = 1;
    a.head = *head;
  }
  if (g_stack_ablate)
    return epi == EPI_FWD ? (nring == 3 ? dispatch_ablate<3>(g_stack_ablate, a, B, stream)
                                        : dispatch_ablate<2>(g_stack_ablate, a, B, stream))
                          : hipErrorInvalidValue;
  if (g_stack_waves == 16)
    return epi == EPI_FWD ? launch_stack<EPI_FWD, 2, 0, false, 16>(a, B, stream)
                          : launch_stack<EPI_DGRAD, 2, 0, false, 16>(a, B, stream);
  if (!g_stack_bpf)
    return epi == EPI_FWD ? launch_stack<EPI_FWD, 2, 0, false>(a, B, stream)
                          : launch_stack<EPI_DGRAD, 2, 0, false>(a, B, stream);
  if (epi == EPI_FWD)
    return nring == 3 ? launch_stack<EPI_FWD, 3, 0>(a, B, stream)
                      : launch_stack<EPI_FWD, 2, 0>(a, B, stream);
  return nring == 3 ? launch_stack<EPI_DGRAD, 3, 0>(a, B, stream)
                    : launch_stack<EPI_DGRAD, 2, 0>(a, B, stream);
}

hipError_t dg_conv_stack(int epi, const long long* table, int nl, const void* X0, int KP, int B,
                         hipStream_t stream) {
  return stack_launch(epi, table, nl, X0, KP, B, nullptr, stream);
}

hipError_t dg_conv_stack_fwd(const long long* table, int nl, const void* X0, int KP, int B,
                             hipStream_t stream) {
  return stack_launch(EPI_FWD, table, nl, X0, KP, B, nullptr, stream);
}

// Forward stack + the 3x3 / 128-channel policy head fused after its last layer (training:
// labels, loss, pred, dZ of the last hidden layer, per-board weight partials, dz for the
// bias reduce — the head_mfma arguments, minus the activation frame).
hipError_t dg_conv_stack_fwd_head(const long long* table, int nl, const void* X0, int KP, int B,
                                  const float* w, const float* bias, const float* posb,
                                  const int* labels, float* loss, int* pred, void* dZ,
                                  float* gw_part, float* dzb, int head_relu, float grad_scale,
                                  hipStream_t stream) {
  const dghead::HeadMArgs h{nullptr, w, bias, posb, labels, loss, pred, nullptr, (char*)dZ,
                            gw_part, dzb, head_relu, grad_scale};
  return stack_launch(EPI_FWD, table, nl, X0, KP, B, &h, stream);
}

}  // extern "C"
