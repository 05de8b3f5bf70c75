// Fused forward of a run of hidden 3x3 layers (C -> C, C = 128, pad 1): the whole
// board-resident forward stack in ONE launch.
//
// Per-layer kernels (conv_board.hip) end every layer with a burst of 23.6 MB of stores
// from all workgroups at once, plus a prologue that re-reads the same activation from HBM;
// ablations (profiles/) put that epilogue/prologue at ~14 of ~32 us per layer, and it
// cannot overlap with anything because every workgroup reaches it at the same time.
//
// Here one workgroup owns one board for ALL layers of the run:
//   * the board's zero-bordered 21x21x128 activation frame lives in LDS (two 64-channel
//     halo images, 112 KB, XOR-swizzled 128-B rows — the conv_board layout);
//   * each layer is 18 K-steps (2 chunks x 9 taps) of v_mfma_f32_16x16x32_bf16 over that
//     image, weight tiles [128 co][64 k] streamed by LDS-DMA (double-buffered, the next
//     layer's first tile prefetched during the current layer's last step);
//   * the epilogue (bias + pos-bias table, ReLU) writes the layer's bf16 output straight
//     back INTO the LDS image (it is the next layer's input), and the global store of that
//     output (activation frame for the backward + 1-bit ReLU mask) is spread over the next
//     layer's first 12 K-steps, underneath its MFMAs.
// Only the first input load and the last layer's stores are exposed.
//
// Reference ops: nn.SpatialZeroPadding + SpatialConvolutionMM + Add + ReLU per layer
// (experiments.lua:137-147).
#include "dg_common.h"

using namespace dg;

namespace {

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
constexpr int WN = 4, MF = 4, NF = 6;     // 2 x 4 waves, 64 co x 96 px per wave

struct StackLayer {
  const bf16_t* A;      // [128][KP] forward weights, k = tap*128 + ci
  const bf16_t* pbias;  // [361][128] bf16 bias + pos-bias
  char* Y;              // output frame [B][21][21][128] bf16
  uint8_t* mask;        // [B][361][16] ReLU bits or null
};
struct StackArgs {
  const char* X0;       // input frame [B][21][21][128] bf16 of the first layer
  int nl, KP;
  StackLayer L[MAXL];
};

__global__ void __launch_bounds__(512) conv_stack_fwd_kernel(StackArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int b = blockIdx.x;
  char* sA0 = smem;
  char* sH = smem + 2 * A_BYTES;  // image c at sH + c * H_BYTES
  const int g_src = (lane & 7) ^ (lane >> 3);

  auto stage_A = [&](int buf, const bf16_t* A, int step) {
    const int c = step / T, t = step - (step / T) * T;
    const int kcol = t * C + c * 64;
    char* dst = sA0 + buf * A_BYTES;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int r = (wave * 2 + i) * 8 + (lane >> 3);
      glds16((const char*)A + ((size_t)r * a.KP + kcol + g_src * 8) * 2,
             (LDS_AS void*)(dst + (wave * 2 + i) * 1024));
    }
  };

  // ---- prologue: the first layer's input frame (both images) + its first weight tile ----
  {
    const char* Xb = a.X0 + (size_t)b * FF * C * 2;
    for (int j = wave; j < 2 * (HROWS / 8); j += 8) {
      const int c = j / (HROWS / 8), jj = j - c * (HROWS / 8);
      int r = jj * 8 + (lane >> 3);
      r = r < FF ? r : FF - 1;
      glds16(Xb + ((size_t)r * C + c * 64 + g_src * 8) * 2,
             (LDS_AS void*)(sH + c * H_BYTES + jj * 1024));
    }
    stage_A(0, a.L[0].A, 0);
  }
  __syncthreads();

  const int lr = lane & 15;
  const int lq = lane >> 4;
  int fp[NF];
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    int p = wn * NF * 16 + j * 16 + lr;
    if (p >= NPTS) p = 0;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    fp[j] = (h + 1) * F + (w + 1);
  }

  // store one 16-B piece (8 channels of one pixel) of the activation held in LDS
  auto copy_out = [&](int u, const StackLayer& Lo) {
    const int p = u >> 4, q = u & 15;
    const int c = q >> 3, g = q & 7;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    const int f = (h + 1) * F + (w + 1);
    const uint4 v = *(const uint4*)(sH + c * H_BYTES + f * 128 + ((g ^ (f & 7)) * 16));
    *(uint4*)(Lo.Y + ((size_t)(b * FF + f) * C + c * 64 + g * 8) * 2) = v;
    if (Lo.mask) {
      auto nz = [](uint32_t x) { return ((x & 0xFFFFu) ? 1u : 0u) | ((x >> 16) ? 2u : 0u); };
      Lo.mask[((size_t)b * NPTS + p) * 16 + q] =
          (uint8_t)(nz(v.x) | (nz(v.y) << 2) | (nz(v.z) << 4) | (nz(v.w) << 6));
    }
  };

  int gs = 0;  // global step counter (A buffer parity)
  for (int l = 0; l < a.nl; ++l) {
    const StackLayer L = a.L[l];
    f32x4 acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int s = 0; s < NSTEP; ++s, ++gs) {
      const int c = s / T, t = s - (s / T) * T;
      if (s + 1 < NSTEP) stage_A((gs + 1) & 1, L.A, s + 1);
      else if (l + 1 < a.nl) stage_A((gs + 1) & 1, a.L[l + 1].A, 0);
      // the previous layer's output (already in the image) goes to HBM under this layer's
      // MFMAs: 512 pieces per step over the first 12 steps
      if (l > 0) {
        const int u = s * 512 + tid;
        if (u < UNITS) copy_out(u, a.L[l - 1]);
      }
      const char* sA = sA0 + (gs & 1) * A_BYTES;
      const char* sHc = sH + c * H_BYTES;
      const int toff = (t / 3 - 1) * F + (t % 3 - 1);
      // one k-half's fragments live at a time (register budget with the copy-out in the
      // loop); the compiler overlaps half 1's reads with half 0's MFMAs
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int g = kk * 4 + lq;
        bf16x8 af[MF], bfr[NF];
#pragma unroll
        for (int i = 0; i < MF; ++i) {
          const int row = wm * 64 + i * 16 + lr;
          af[i] = lds_read_b128((const LDS_AS char*)(sA + row * 128 + ((g ^ (row & 7)) * 16)));
        }
#pragma unroll
        for (int j = 0; j < NF; ++j) {
          const int row = fp[j] + toff;
          bfr[j] = lds_read_b128((const LDS_AS char*)(sHc + row * 128 + ((g ^ (row & 7)) * 16)));
        }
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
          for (int j = 0; j < NF; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      __syncthreads();
    }

    // ---- epilogue: + (bias + pos-bias), ReLU, bf16 -> back into the LDS image ----
    // (every wave is past its last read of the image: barrier above)
#pragma unroll
    for (int j = 0; j < NF; ++j) {
      const int p = wn * NF * 16 + j * 16 + lr;
      if (p >= NPTS) continue;
      const int f = fp[j];
#pragma unroll
      for (int i = 0; i < MF; ++i) {
        const int cl = i * 16 + lq * 4;  // channel within the wave's 64-channel image
        const uint2 u = *(const uint2*)(L.pbias + p * C + wm * 64 + cl);
        f32x4 v = acc[i][j];
        v[0] = fmaxf(v[0] + __uint_as_float(u.x << 16), 0.f);
        v[1] = fmaxf(v[1] + __uint_as_float(u.x & 0xFFFF0000u), 0.f);
        v[2] = fmaxf(v[2] + __uint_as_float(u.y << 16), 0.f);
        v[3] = fmaxf(v[3] + __uint_as_float(u.y & 0xFFFF0000u), 0.f);
        uint2 o;
        o.x = pack_bf16x2(v[0], v[1]);
        o.y = pack_bf16x2(v[2], v[3]);
        const int slot = (cl >> 3) ^ (f & 7);
        *(uint2*)(sH + wm * H_BYTES + f * 128 + slot * 16 + (cl & 4) * 2) = o;
      }
    }
    __syncthreads();
  }
  // last layer's output: exposed copy-out
  for (int u = tid; u < UNITS; u += 512) copy_out(u, a.L[a.nl - 1]);
}

}  // namespace

extern "C" {

// table: nl rows of {A, pbias, Y, mask} (int64 pointers; mask may be 0)
hipError_t dg_conv_stack_fwd(const long long* table, int nl, const void* X0, int KP, int B,
                             hipStream_t stream) {
  if (nl <= 0 || nl > MAXL || KP < T * C || KP % 64 != 0 || B <= 0) return hipErrorInvalidValue;
  StackArgs a;
  a.X0 = (const char*)X0;
  a.nl = nl;
  a.KP = KP;
  for (int i = 0; i < nl; ++i) {
    a.L[i].A = (const bf16_t*)table[4 * i];
    a.L[i].pbias = (const bf16_t*)table[4 * i + 1];
    a.L[i].Y = (char*)table[4 * i + 2];
    a.L[i].mask = (uint8_t*)table[4 * i + 3];
    if (!a.L[i].A || !a.L[i].pbias || !a.L[i].Y) return hipErrorInvalidValue;
  }
  constexpr size_t lds = 2 * (size_t)A_BYTES + 2 * (size_t)H_BYTES;
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)conv_stack_fwd_kernel,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL(conv_stack_fwd_kernel, dim3(B), dim3(512), lds, stream, a);
  return hipGetLastError();
}

}  // extern "C"
