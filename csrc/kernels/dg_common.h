// Common device helpers for the deep_go_amd CDNA4 (gfx950) kernels.
//
// Everything here is written for 64-lane wavefronts, bf16 MFMA (v_mfma_f32_16x16x32_bf16)
// and LDS-DMA staging (global_load_lds_dwordx4).  No CUDA/HIP dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DG_DEV __device__ __forceinline__
#define LDS_AS __attribute__((address_space(3)))

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef uint16_t bf16_t;  // storage type for bf16 in global memory

namespace dg {

constexpr int BOARD = 19;
constexpr int NPTS = 361;

// f32 -> bf16 round-to-nearest-even (NaN kept NaN via the compiler's v_cvt_pk_bf16_f32).
DG_DEV bf16_t f2bf(float f) {
  __bf16 h = (__bf16)f;
  return __builtin_bit_cast(bf16_t, h);
}
DG_DEV float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }

DG_DEV uint32_t pack_bf16x2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// Async 16-byte global->LDS copy.  The LDS destination is (wave-uniform base) + lane*16.
DG_DEV void glds16(const void* gsrc, LDS_AS void* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(gsrc, lds_wave_base, 16, 0, 0);
}

// LDS-DMA issued from inline asm: the compiler's waitcnt pass does not see it, so it neither
// waits for it in front of later LDS reads (it cannot tell transposing-read addresses from
// the DMA destination) nor before barriers.  Kernels using it count their own DMA
// instructions per stage and wait with dma_wait<N>() = s_waitcnt vmcnt(N) (newest stages in
// flight).  lds_wave_base must be wave-uniform (SGPR); each lane lands 16 B at base+lane*16.
DG_DEV void dma16(const void* gsrc, uint32_t lds_wave_base) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off"
               :
               : "s"(lds_wave_base), "v"(gsrc)
               : "memory", "m0");
}
template <int N>
DG_DEV void dma_wait() {
  static_assert(N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

DG_DEV f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

DG_DEV bf16x8 lds_read_b128(const LDS_AS char* p) { return *(const LDS_AS bf16x8*)p; }

// Staggered two-group schedules of the board-resident stacks (conv_stack2 / conv_stack_f8
// STAG): LDS counters instead of workgroup barriers.  A wave
// counts itself in (+1 from one lane) once its LDS accesses are done (lgkmcnt(0)); waiters
// poll with s_sleep between reads.  Both in inline asm: as C++ (a lane-0 branch, a polling
// loop) the control flow inside the rolled K loop costs 100-160 spilled VGPRs.  (An asm
// ds_add / ds_read outstanding ahead of the compiler's own LDS reads only lengthens its
// in-order lgkmcnt waits.)
DG_DEV void grp_signal(LDS_AS unsigned* c) {
  unsigned long long sv;
  asm volatile(
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %1, %2\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(sv) : "v"((unsigned)(size_t)c), "v"(1u) : "memory");
}
DG_DEV void grp_wait(LDS_AS unsigned* c, unsigned target) {
  unsigned v, sc;
  asm volatile(
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_nop 4\n\t"
      "s_cmp_ge_u32 %1, %3\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n"
      "2:"
      : "=&v"(v), "=&s"(sc) : "v"((unsigned)(size_t)c), "s"(target) : "memory", "scc");
}
// The same only when the (wave-uniform, SGPR) step index st equals at: the test is inside the
// asm, so a rolled K loop keeps straight-line code (a C++ branch around the asm there costs
// ~30-40 spilled VGPRs)
DG_DEV void grp_signal_at(LDS_AS unsigned* c, int st, int at) {
  unsigned long long sv;
  asm volatile(
      "s_cmp_eq_u32 %3, %4\n\t"
      "s_cbranch_scc0 3f\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, 1\n\t"
      "ds_add_u32 %1, %2\n\t"
      "s_mov_b64 exec, %0\n"
      "3:"
      : "=&s"(sv) : "v"((unsigned)(size_t)c), "v"(1u), "s"(st), "s"(at) : "memory", "scc");
}
DG_DEV void grp_wait_at(LDS_AS unsigned* c, unsigned target, int st, int at) {
  unsigned v, sc;
  asm volatile(
      "s_cmp_eq_u32 %4, %5\n\t"
      "s_cbranch_scc0 2f\n"
      "1:\n\t"
      "ds_read_b32 %0, %2\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %1, %0\n\t"
      "s_nop 4\n\t"
      "s_cmp_ge_u32 %1, %3\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n"
      "2:"
      : "=&v"(v), "=&s"(sc)
      : "v"((unsigned)(size_t)c), "s"(target), "s"(st), "s"(at)
      : "memory", "scc");
}


// ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies &row q, cols 4p..4p+3;
// lane i receives column i of the 4 rows (row q in element q).
DG_DEV s16x4 lds_read_tr(const LDS_AS char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)p);
}

DG_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
DG_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide max of non-negative v folded into *amax (float bits) with ONE device atomic per
// workgroup, skipped when the stored value is already larger (thousands of same-address
// atomics serialize at the memory side).  s_tmp: >= blockDim/64 floats of LDS.  Every
// thread of the block must call it (contains a barrier).
DG_DEV void block_amax(float v, unsigned* amax, float* s_tmp) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) s_tmp[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float m = s_tmp[0];
    for (int w = 1; w < nw; ++w) m = fmaxf(m, s_tmp[w]);
    const unsigned u = __float_as_uint(m);
    if (u > __hip_atomic_load(amax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMax(amax, u);
  }
}

// ---- deterministic second-pass sums of the weight / bias gradient partials -------------
// Shared by the slab reduce (conv_mfma.hip wgrad_reduce_kernel) and the fused reduce +
// update + refresh (elementwise.hip grad_update_kernel), so the two produce bit-identical
// gradients: a fixed summation order that does not depend on the thread mapping.
//
// sum over split slabs z of src[z * zstride] (four interleaved accumulators, z mod 4, the tail
// into the first, then (s0 + s1) + (s2 + s3)); element-wise identical for the f32x4 form
DG_DEV f32x4 slab_sum4(const float* src, int splits, size_t zstride) {
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0, s2 = s0, s3 = s0;
  int z = 0;
  for (; z + 4 <= splits; z += 4) {
    s0 += *(const f32x4*)(src + (z + 0) * zstride);
    s1 += *(const f32x4*)(src + (z + 1) * zstride);
    s2 += *(const f32x4*)(src + (z + 2) * zstride);
    s3 += *(const f32x4*)(src + (z + 3) * zstride);
  }
  for (; z < splits; ++z) s0 += *(const f32x4*)(src + z * zstride);
  return (s0 + s1) + (s2 + s3);
}
// NU independent slab_sum4's with all their loads interleaved (more loads in flight per
// thread); element-wise the same order as slab_sum4
template <int NU>
DG_DEV void slab_sums4(const float* const (&src)[NU], int splits, size_t zstride,
                       f32x4 (&out)[NU]) {
  f32x4 s[NU][4];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int q = 0; q < 4; ++q) s[u][q] = f32x4{0.f, 0.f, 0.f, 0.f};
  int z = 0;
  for (; z + 4 <= splits; z += 4) {
    f32x4 v[NU][4];
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[u][q] = *(const f32x4*)(src[u] + (z + q) * zstride);
#pragma unroll
    for (int u = 0; u < NU; ++u)
#pragma unroll
      for (int q = 0; q < 4; ++q) s[u][q] += v[u][q];
  }
  for (; z < splits; ++z)
#pragma unroll
    for (int u = 0; u < NU; ++u) s[u][0] += *(const f32x4*)(src[u] + z * zstride);
#pragma unroll
  for (int u = 0; u < NU; ++u) out[u] = (s[u][0] + s[u][1]) + (s[u][2] + s[u][3]);
}
DG_DEV float slab_sum1(const float* src, int splits, size_t zstride) {
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int z = 0;
  for (; z + 4 <= splits; z += 4) {
    s0 += src[(z + 0) * zstride];
    s1 += src[(z + 1) * zstride];
    s2 += src[(z + 2) * zstride];
    s3 += src[(z + 3) * zstride];
  }
  for (; z < splits; ++z) s0 += src[z * zstride];
  return (s0 + s1) + (s2 + s3);
}
// per-position bias gradient: sum over board chunks of part[chunk * np] (even / odd chunks)
DG_DEV float chunk_sum(const float* part, int nchunks, size_t np) {
  float s0 = 0.f, s1 = 0.f;
  int z = 0;
  for (; z + 2 <= nchunks; z += 2) {
    s0 += part[(size_t)z * np];
    s1 += part[(size_t)(z + 1) * np];
  }
  for (; z < nchunks; ++z) s0 += part[(size_t)z * np];
  return s0 + s1;
}
// per-channel bias gradient of channel c: sum of the R = chunks x 19 row partials
// rowpart[r][C], as four partial sums (rows r = q mod 4 below 4 floor(R / 4), in increasing
// r; the tail rows into partial 0) computed by 4 ADJACENT lanes q = lane & 3, combined as
// (p0 + p1) + (p2 + p3) by two xor shuffles — every one of the 4 lanes returns the total.
// All 4 lanes of a quad must call it.
DG_DEV float rows_sum4(const float* rowpart, int R, int C, int c, int q) {
  const int R4 = R & ~3;
  float s = 0.f;
  int r = q;
  for (; r + 60 < R4; r += 64) {   // 16 rows of this lane per iteration, loads first
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = rowpart[(size_t)(r + 4 * k) * C + c];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += v[k];
  }
  for (; r < R4; r += 4) s += rowpart[(size_t)r * C + c];
  if (q == 0)
    for (int t = R4; t < R; ++t) s += rowpart[(size_t)t * C + c];
  s += __shfl_xor(s, 1, 64);
  s += __shfl_xor(s, 2, 64);
  return s;
}

// ---- the fused update's all-or-nothing gate ----------------------------------------------
// A training step whose gradient pass 2 is deferred into grad_update has no reduced gradient
// to check before the parameters change.  So every producer of that pass's inputs (window
// weight-gradient slabs, bias-gradient partials, the head / first-layer reduces) checks what
// it writes (or, for the bias partials, every dZ value it reads) and tags the step when any
// value is non-finite or |v| >= 2^120 (2^100 for dZ): sf[1] = sf[0] + 1, sf[0] being the
// device step counter.  Those bounds keep every sum the deferred pass 2 forms finite (<= 64
// split slabs, <= 16 bias chunks of <= 64 boards, a first-layer weight gradient over 92k
// pixels of 0/1 inputs), so grad_update can skip the WHOLE step on the tag before writing any
// parameter (HipGoNet._stepflag; the reference's pcall around the step, train.lua:106-111).
constexpr float GRAD_BOUND = 0x1p120f;
constexpr float DZ_BOUND = 0x1p100f;
DG_DEV bool grad_out_of_range(float v) { return !(__builtin_fabsf(v) < GRAD_BOUND); }
DG_DEV void flag_bad_step(long long* sf) { sf[1] = sf[0] + 1; }

// Exact floor(n / d) for 0 <= n < 2^22 and 1 <= d <= 4096 via a 64-bit magic
// m = floor(2^32 / d) + 1 (host computes it; checked exhaustively in tests/tools).
DG_DEV uint32_t fastdiv(uint32_t n, uint64_t m) { return (uint32_t)(((uint64_t)n * m) >> 32); }
inline uint64_t fastdiv_magic(uint32_t d) { return (0x100000000ull / d) + 1; }

// Byte offset of board pixel (b, h, w) inside a zero-bordered NHWC frame
// [B][19+2pad][19+2pad][C] of bf16.
DG_DEV uint32_t frame_off(int b, int h, int w, int pad, int C) {
  const int F = BOARD + 2 * pad;
  return (uint32_t)(((b * F + h + pad) * F + (w + pad)) * C) * 2u;
}
DG_DEV uint32_t pixel_frame_off(int n, int pad, int C) {
  const int b = n / NPTS;
  const int p = n - b * NPTS;
  const int h = p / BOARD;
  const int w = p - h * BOARD;
  return frame_off(b, h, w, pad, C);
}

}  // namespace dg
