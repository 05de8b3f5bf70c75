// Memory-bound helper kernels: GPU feature expansion, per-channel / per-position bias
// gradients, fused SGD / RMSProp updates, device-side LR decay and the bf16 weight
// refresh that re-lays the fp32 OHWI master weights into the two MFMA operand layouts.
#include "dg_common.h"
#include "dg_features.h"

using namespace dg;

namespace {

// ------------------------------------------------------------------------------------
// 9 stored uint8 planes -> 37 network planes (padded to CP channels) written straight
// into the first layer's zero-bordered NHWC frame.  Reference: preprocess()
// (dataloader.lua:50-92), which builds float64 planes on 32 CPU threads.
// planes: [B][9][361] uint8, player: [B] (1 black / 2 white), rank: [B] (dan of the
// player to move, 1..9).  One thread per (board, point).
__global__ void expand_features_kernel(const uint8_t* __restrict__ planes,
                                       const uint8_t* __restrict__ player,
                                       const uint8_t* __restrict__ rank, char* __restrict__ out,
                                       int B, int pad, int CP, char* __restrict__ out2,
                                       int CP2) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * NPTS) return;
  const int b = idx / NPTS;
  const int p = idx - b * NPTS;
  const uint8_t* pl = planes + (size_t)b * 9 * NPTS + p;
  float v[48];
  expand_point(pl, player[b], rank[b], v);
  const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
  char* dst = out + frame_off(b, h, w, pad, CP);
  // optional second frame with CP2 (64) channels for the board-tiled first layer; its
  // channels >= CP are never written (zero from allocation)
  char* dst2 = out2 ? out2 + frame_off(b, h, w, pad, CP2) : nullptr;
#pragma unroll
  for (int c = 0; c < 48; c += 8) {
    if (c >= CP) break;
    uint4 o;
    o.x = pack_bf16x2(v[c + 0], v[c + 1]);
    o.y = pack_bf16x2(v[c + 2], v[c + 3]);
    o.z = pack_bf16x2(v[c + 4], v[c + 5]);
    o.w = pack_bf16x2(v[c + 6], v[c + 7]);
    *(uint4*)(dst + c * 2) = o;
    if (dst2) *(uint4*)(dst2 + c * 2) = o;
  }
}

// ------------------------------------------------------------------------------------
// Bias gradients of a conv layer from its pre-activation gradient frame dZ, pass 1:
//   part[chunk][p][c]     = sum_{b in chunk} dZ[b][p][c]
//   rowpart[chunk][h][c]  = sum_{w} part[chunk][h*19+w][c]
// Grid: (board row h) x (chunk of BG_BT boards).  A workgroup streams the 19*C contiguous
// values of row h for each of its boards with independent 16-byte loads (unrolled over
// the chunk) and writes plain coalesced partials — no atomics, deterministic.  Pass 2
// (sum over chunks -> gposb, gbias) runs inside the wgrad slab-reduce launch.
// Reference: nn.Add / conv bias backward (experiments.lua:138,144).
constexpr int BG_BT = 16;   // boards per chunk of a single-layer launch
constexpr int BG_BT_MULTI = 64;  // ... of a multi-layer launch (enough workgroups from the
                            // layers: 4x fewer partials for the slab reduce to read)
constexpr int BG_LD = 16;   // 16-B loads in flight per thread
constexpr int BG_MAXL = 16;
struct BiasLayers {  // blockIdx.z = layer (several same-shape layers in one launch)
  const char* dZ[BG_MAXL];
  float* part[BG_MAXL];
  // optional: dZ is the fp8 backward-data stack's e5m2 copy ([B][FP8_ROWS][C] bytes, the
  // 21x21 frame in rows 0..440) and *s8 its power-of-two scale — the bf16 frame it replaces
  // is exactly e5m2 x s8, so the partials are bit-identical (null: a bf16 frame)
  const float* s8[BG_MAXL];
  long long* sf;   // the fused update's step tag (dg_common.h): a dZ value out of range sets it
};
constexpr int BG_FP8_ROWS = 448;
// LD: 16-B loads in flight per thread.  The multi-layer launch runs beside the window weight
// gradient, whose two workgroups per CU leave 64 VGPRs per SIMD: its variant (LD 2, 256
// threads, 48 VGPRs) fits next to them on every CU instead of only on the 32 CUs that hold
// one window workgroup (the 1024-thread, 110-VGPR version was confined there and outlasted
// the window kernel at d = 256: 12x256 bf16 +1.5%, profiles/r3_bias_partial_small_wg.txt).
template <int LD>
__global__ void __launch_bounds__(LD == BG_LD ? 1024 : 256, LD == BG_LD ? 1 : 8)
bias_grad_partial_kernel(BiasLayers Ls, int B, int C, int pad, int nchunks, int bt) {
  extern __shared__ __attribute__((aligned(16))) float s_row[];  // [19][C]
  const int h = blockIdx.x;
  const int chunk = blockIdx.y;
  const char* __restrict__ dZ = Ls.dZ[blockIdx.z];
  float* __restrict__ part = Ls.part[blockIdx.z];
  const float* s8p = Ls.s8[blockIdx.z];
  const bool f8 = s8p != nullptr;            // uniform per workgroup
  const float s8 = f8 ? *s8p : 1.f;
  const int b0 = chunk * bt;
  const int G = C / 8;
  const int F = BOARD + 2 * pad;
  const int items = BOARD * G;  // (w, g) pairs of the row
  const int tid = threadIdx.x;
  const int esz = f8 ? 1 : 2;
  const size_t board_stride = (size_t)(f8 ? BG_FP8_ROWS : F * F) * C * esz;
  const char* row0 = dZ + ((size_t)((h + pad) * F + pad) * C) * esz;
  float* prow = part + ((size_t)chunk * NPTS + h * BOARD) * C;
  // blockDim covers all 19*C/8 items of the row in ONE pass (the 256-thread version ran a
  // second pass on 48 threads whose load latency the whole workgroup waited for)
  float dzmax = 0.f;   // max |dZ| read, fp8 frames (the step tag; NaN shows in the sums)
  // bf16 frames: the max |bits| of the two halves of every word read (one AND + one packed
  // 16-bit max per word; the float fabs / fmax form doubled the VALU work of a kernel that
  // runs beside the window weight gradient and slowed both at d = 256)
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  u16x2 hmax = {0, 0};
  bool nonfinite = false;
  for (int it = tid; it < items; it += blockDim.x) {
    const int w = it / G, g = it - (it / G) * G;
    const char* src = row0 + ((size_t)w * C + g * 8) * esz;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (f8) {
      for (int jb = 0; jb < bt && b0 + jb < B; jb += LD) {
        uint2 v[LD];
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          const int b = b0 + jb + j;
          v[j] = b < B ? *(const uint2*)(src + (size_t)b * board_stride) : uint2{0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          const int u[2] = {(int)v[j].x, (int)v[j].y};
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const auto lo = __builtin_amdgcn_cvt_pk_f32_bf8(u[e], false);
            const auto hi = __builtin_amdgcn_cvt_pk_f32_bf8(u[e], true);
            acc[4 * e] += lo[0] * s8;
            acc[4 * e + 1] += lo[1] * s8;
            acc[4 * e + 2] += hi[0] * s8;
            acc[4 * e + 3] += hi[1] * s8;
            dzmax = fmaxf(dzmax, fmaxf(fmaxf(fabsf(lo[0]), fabsf(lo[1])),
                                       fmaxf(fabsf(hi[0]), fabsf(hi[1]))) * s8);
          }
        }
      }
    } else {
      for (int jb = 0; jb < bt && b0 + jb < B; jb += LD) {
        uint4 v[LD];
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          const int b = b0 + jb + j;
          v[j] = b < B ? *(const uint4*)(src + (size_t)b * board_stride) : uint4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int j = 0; j < LD; ++j) {
          const uint32_t u[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[2 * e] += __uint_as_float(u[e] << 16);
            acc[2 * e + 1] += __uint_as_float(u[e] & 0xFFFF0000u);
            hmax = __builtin_elementwise_max(hmax,
                                             __builtin_bit_cast(u16x2, u[e] & 0x7FFF7FFFu));
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) nonfinite |= !__builtin_isfinite(acc[e]);
    f32x4* dst = (f32x4*)(prow + w * C + g * 8);
    dst[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    dst[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
    float* sr = s_row + w * C + g * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) sr[e] = acc[e];
  }
  // (bf16 bits of 2^100 = 0x7180; a NaN's or an infinity's |bits| exceed it)
  const unsigned hm = hmax.x > hmax.y ? hmax.x : hmax.y;
  if (Ls.sf && (nonfinite || !(dzmax < DZ_BOUND) || hm >= 0x7180u)) flag_bad_step(Ls.sf);
  __syncthreads();
  float* rowpart = part + (size_t)nchunks * NPTS * C + ((size_t)chunk * BOARD + h) * C;
  for (int c = tid; c < C; c += blockDim.x) {
    float sc = 0.f;
    for (int w = 0; w < BOARD; ++w) sc += s_row[w * C + c];
    rowpart[c] = sc;
  }
}

// ------------------------------------------------------------------------------------
// gradient element i as fp32: the flat fp32 gradient, or its bf16 twin (the data-parallel
// bf16 wire format: the all-reduced bucket is read as it came off the wire)
DG_DEV float grad_at(const float* g, size_t i) { return g[i]; }
DG_DEV float grad_at(const bf16_t* g, size_t i) { return bf2f(g[i]); }
DG_DEV f32x4 grad4_at(const float* g, size_t i4) { return ((const f32x4*)g)[i4]; }
DG_DEV f32x4 grad4_at(const bf16_t* g, size_t i4) {
  const uint2 u = ((const uint2*)g)[i4];
  return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xFFFF0000u),
               __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xFFFF0000u)};
}

// SGD (optimizer.lua:24-27): theta -= lr * g over the flat fp32 master buffer.  lr lives
// on the device (double) so the step can be replayed inside a hipGraph.
template <typename G>
__global__ void sgd_kernel(float* __restrict__ p, const G* __restrict__ g, size_t n,
                           const double* __restrict__ lr, float gscale,
                           const float* __restrict__ gate) {
  // gate (optional, device): 0 skips the update (non-finite loss/gradient policy, graph-
  // friendly).  Return, do not scale by it: 0 * NaN gradient is still NaN.
  if (gate && *gate == 0.f) return;
  const float l = (float)(*lr) * gscale;
  const size_t n4 = n / 4;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    f32x4 pv = ((f32x4*)p)[i];
    const f32x4 gv = grad4_at(g, i);
    pv -= l * gv;
    ((f32x4*)p)[i] = pv;
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] -= l * grad_at(g, i);
}

// RMSProp-style update (the reference's misnamed AdagradOptimizer, optimizer.lua:1-14):
// ms = decay*ms + (1-decay)*g^2 ; theta -= lr * g / sqrt(ms); ms initialised to 1.
template <typename G>
__global__ void rmsprop_kernel(float* __restrict__ p, const G* __restrict__ g,
                               float* __restrict__ ms, size_t n, const double* __restrict__ lr,
                               float decay, float gscale, const float* __restrict__ gate) {
  if (gate && *gate == 0.f) return;
  const float l = (float)(*lr);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const float gi = grad_at(g, i) * gscale;
    const float m = decay * ms[i] + (1.f - decay) * gi * gi;
    ms[i] = m;
    p[i] -= l * gi * rsqrtf(m);
  }
}

__global__ void set_gate_kernel(float* gate) {
  if (threadIdx.x == 0) *gate = 1.f;
}

// gate = isfinite(sum(loss[0..n))) ? 1 : 0 — one workgroup; feeds the optimizer gate.
__global__ void finite_gate_kernel(const float* __restrict__ loss, int n, float* __restrict__ gate,
                                   int* __restrict__ bad_count) {
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  int bad = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) bad |= !isfinite(loss[i]);
  if (bad) atomicOr(&s_bad, 1);
  __syncthreads();
  if (threadIdx.x == 0) {
    *gate = s_bad ? 0.f : 1.f;
    if (s_bad && bad_count) *bad_count += 1;
  }
}

// gate &= all-finite(g[0..n)): run after finite_gate_kernel on the (all-reduced) flat gradient.
// Under data parallelism every rank sees the same reduced gradient, so every rank takes the
// same decision (a rank-local loss check would let one rank's NaN reach ranks that still
// step).  The first lane that finds a bad value flips the gate and counts the step once.
template <typename G>
__global__ void grad_gate_kernel(const G* __restrict__ g, size_t n, float* __restrict__ gate,
                                 int* __restrict__ bad_count) {
  const size_t n4 = n / 4;
  bool bad = false;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4;
       i += (size_t)gridDim.x * blockDim.x) {
    const f32x4 v = grad4_at(g, i);
    bad |= !(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]) && isfinite(v[3]));
  }
  for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    bad |= !isfinite(grad_at(g, i));
  if (bad) {
    const int old = atomicExch((int*)gate, 0);
    if (old != 0 && bad_count) atomicAdd(bad_count, 1);
  }
}

// The whole gate in ONE launch (the loss check and the gradient scan were two, in series on
// the data-parallel step's tail): every block scans its share of the (all-reduced) gradient,
// block 0 also the loss; each block's verdict rides on its ticket (count | bad << 16, one
// device atomic) and the LAST block writes the gate, counts a bad step once and re-zeroes the
// ticket (graph-replayable).
template <typename G>
__global__ void __launch_bounds__(256) gate_all_kernel(const float* __restrict__ loss, int nloss,
                                                       const G* __restrict__ g, size_t n,
                                                       float* __restrict__ gate,
                                                       int* __restrict__ bad_count,
                                                       unsigned* __restrict__ ticket) {
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  bool bad = false;
  if (blockIdx.x == 0 && loss)
    for (int i = threadIdx.x; i < nloss; i += blockDim.x) bad |= !isfinite(loss[i]);
  if (g) {
    const size_t n4 = n / 4;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {   // 8 loads in flight per thread
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = grad4_at(g, i + u * stride);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        bad |= !(isfinite(v[u][0]) && isfinite(v[u][1]) && isfinite(v[u][2]) &&
                 isfinite(v[u][3]));
    }
    for (; i < n4; i += stride) {
      const f32x4 v = grad4_at(g, i);
      bad |= !(isfinite(v[0]) && isfinite(v[1]) && isfinite(v[2]) && isfinite(v[3]));
    }
    for (size_t i = n4 * 4 + blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
      bad |= !isfinite(grad_at(g, i));
  }
  if (bad) s_bad = 1;   // (benign same-value race)
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned old = atomicAdd(ticket, 1u + (s_bad ? 0x10000u : 0u));
    if ((old & 0xFFFFu) == gridDim.x - 1) {
      const bool any = (old >> 16) != 0u || s_bad;
      *gate = any ? 0.f : 1.f;
      if (any && bad_count) *bad_count += 1;
      *ticket = 0u;
    }
  }
}

__global__ void lr_decay_kernel(double* lr, double decay, long long* step) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    *lr = *lr * (1.0 - decay);
    if (step) *step += 1;
  }
}

// ------------------------------------------------------------------------------------
// fp32 OHWI master -> bf16 operand layouts, all layers in one launch (grid.y = layer):
//   fwd  : Wf[co][t*cinp + ci]          (A operand of the forward NT GEMM)
//   dgrad: Wd[ci][(T-1-t)*cout + co]    (A operand of the dgrad NT GEMM, flipped taps)
struct WRefreshLayer {
  const float* w;
  bf16_t* wf;
  bf16_t* wd;          // may be null (first layer / head)
  uint8_t* wf8;        // e4m3 forward operand (fp8 layers) or null; same [co][t*cinp+ci], kpf
  const float* s_w;    // its quantization scale (device)
  unsigned* amax_w;    // |w| max observed here (float bits) -> next step's s_w: one slot per
                       // workgroup (blockIdx.x < REFRESH_PARTS), reduced by fp8_update_scales
  const float* bias;   // [cout]            } pbias[p][co] = bf16(bias[co] + posb[p][co]):
  const float* posb;   // [361][cout]       } the forward epilogue's single bias table
  bf16_t* pbias;       // [361][cout] or null
  uint2* pbias_frag;   // the same table in the board-resident stack's accumulator-fragment
                       // order (cout == 128): [24 px frags][2 co halves][4][64 lanes] x 4 bf16
  uint4* wf_frag;      // conv_stack2 / conv_layer2 A operands (3x3, C -> C, C = 128 | 256),
  uint4* wd_frag;      //   MFMA fragment order [h C/128][step 9 C/64][wm 2][kk 2][i 4][lane 64]
                       //   x 8 bf16 (forward / dgrad)
  uint4* wf8_frag;     // conv_stack_f8 A operands (e4m3, quantized with s_w like wf8):
                       //   [h][tap 9][c][wm 2][i 4][half 2][lane 64] x 16 B (requires wf8)
  uint4* wd8_frag;     // the same for the backward-data operand (flipped taps, transposed)
  // (wf / wd / wf8 may be null: the per-step refresh skips the plain copies no launch of the
  // step reads — the stacks read the fragment-ordered ones; s_w != null marks an fp8 layer)
  int cout, cin, taps, cinp, kpf, kpd;
};
constexpr int MAX_REFRESH = 48;
constexpr int REFRESH_PARTS = 512;   // max workgroups per layer (= amax_w slots per layer)
struct WRefreshArgs {
  int n;
  WRefreshLayer L[MAX_REFRESH];
};

// Per-element part of a 64 x 64 (co, ci) tile's refresh at tap t: the plain bf16 forward
// operand, the plain e4m3 copy, the |w| max (fp8 layers).
DG_DEV void refresh_elem(const WRefreshLayer& L, int co, int ci, int t, float v, float inv8,
                         float& wmax) {
  if (L.wf) L.wf[(size_t)co * L.kpf + t * L.cinp + ci] = f2bf(v);
  if (L.s_w) {   // fp8 layer: |w| max for the next scale; the plain e4m3 copy if kept
    if (L.wf8) {
      const float q = fmaxf(fminf(v * inv8, 448.f), -448.f);
      L.wf8[(size_t)co * L.kpf + t * L.cinp + ci] =
          (uint8_t)(__builtin_amdgcn_cvt_pk_fp8_f32(q, 0.f, 0, false) & 0xFF);
    }
    wmax = fmaxf(wmax, fabsf(v));
  }
}

DG_DEV bool refresh_needs_tile(const WRefreshLayer& L) {
  return L.wd || L.wf_frag || L.wd_frag || L.wf8_frag || L.wd8_frag;
}

// conv_stack_f8's K-step of (tap t, 128-channel chunk c, 64-channel half kh) and the first of
// the two lane groups holding it: C = 128 (nc = 1) runs half-major steps — unit n = 9 kh + t
// is step n / 2, lane groups 2 (n % 2), +1 (conv_stack_f8.hip read_B); C = 256 steps are
// (tap, chunk) with the half in lane groups 2 kh, +1
DG_DEV void f8_step_of(int nc, int t, int c, int kh, int& st, int& lg) {
  if (nc == 1) {
    const int n = 9 * kh + t;
    st = n >> 1;
    lg = 2 * (n & 1);
  } else {
    st = t * nc + c;
    lg = 2 * kh;
  }
}

// The whole-tile operand copies of tile (t, cot, cit) from tileS[co - 64 cot][ci - 64 cit]
// (fp32 weights, written and made visible by the caller): the transposed / flipped dgrad
// operand and the MFMA fragment orders of the stacks.  Ends with a barrier.
DG_DEV void refresh_tile_copies(const WRefreshLayer& L, int t, int cot, int cit,
                                float (*tileS)[65], float inv8) {
    if (L.wd) {
      for (int e = threadIdx.x; e < 64 * 64; e += 256) {
        const int rr = e >> 6, cc = e & 63;
        const int ci = cit * 64 + rr, co = cot * 64 + cc;
        if (co < L.cout && ci < L.cin)
          L.wd[(size_t)ci * L.kpd + (L.taps - 1 - t) * L.cout + co] = f2bf(tileS[cc][rr]);
      }
    }
    if (L.wf_frag && L.taps != 9) {
      // the first layer fused in front of the forward stack (conv_stack2.hip l1 mode) or
      // on conv_l1_frag (conv_l1.hip): [co][K = taps*cinp (linear, padded to 1024)] in the
      // stack's fragment order [h][s][wm][kk][i][lane] x 8 bf16 (h = 128-channel output
      // pass); the 16-B unit of row co and 8-channel chunk kc = t*gpt + c8 sits at s = kc/8,
      // kk = (kc/4)&1, lane group kc&3 (chunks past the last tap stay zero: the buffer is
      // zero-initialised and never written there)
      const int gpt = L.cinp / 8;
      for (int u = threadIdx.x; u < 64 * gpt; u += 256) {
        const int rr = u / gpt, c8 = u - (u / gpt) * gpt;
        const int kc = t * gpt + c8;
        const int lane = (kc & 3) * 16 + (rr & 15);
        uint32_t f[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          f[e] = pack_bf16x2(tileS[rr][c8 * 8 + 2 * e], tileS[rr][c8 * 8 + 2 * e + 1]);
        L.wf_frag[(((((size_t)(cot >> 1) * 16 + (kc >> 3)) * 2 + (cot & 1)) * 2 +
                    ((kc >> 2) & 1)) * 4 + (rr >> 4)) * 64 + lane] = uint4{f[0], f[1], f[2], f[3]};
      }
    } else if (L.wf_frag || L.wd_frag) {
      // this tile is exactly one 8 KB (step, co-half) chunk of each fragment layout:
      //   forward: rows co (wm = cot), k = ci of chunk cit at tap t -> step cit * 9 + t
      //   dgrad  : rows ci (wm = cit), k = co of chunk cot at flipped tap 8 - t
      // 16-B unit u = (kk * 4 + i) * 64 + lane holds rows i*16 + (lane & 15), k = kk*32 +
      // (lane >> 4)*8 .. +7: one coalesced 16-B store per thread and unit
      for (int u = threadIdx.x; u < 512; u += 256) {
        const int kk = u >> 8, i = (u >> 6) & 3, ln = u & 63;
        const int r = i * 16 + (ln & 15), k0 = kk * 32 + (ln >> 4) * 8;
        uint32_t f[4], d[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          f[e] = pack_bf16x2(tileS[r][k0 + 2 * e], tileS[r][k0 + 2 * e + 1]);
          d[e] = pack_bf16x2(tileS[k0 + 2 * e][r], tileS[k0 + 2 * e + 1][r]);
        }
        // (C = 256: [h = co half][36 steps] — h = cot / 2 (forward) / cit / 2 (dgrad rows))
        const int nst = (L.cin / 64) * 9;
        if (L.wf_frag)
          L.wf_frag[(((size_t)(cot >> 1) * nst + cit * 9 + t) * 2 + (cot & 1)) * 512 + u] =
              uint4{f[0], f[1], f[2], f[3]};
        if (L.wd_frag)
          L.wd_frag[(((size_t)(cit >> 1) * nst + cot * 9 + (8 - t)) * 2 + (cit & 1)) * 512 + u] =
              uint4{d[0], d[1], d[2], d[3]};
      }
    }
    if (L.wf8_frag) {
      // this tile = rows co of output pass h = cot / 2, co-half wm = cot % 2; k = ci of
      // 128-channel chunk c = cit / 2, lane groups 2 (cit % 2), +1; at tap t.  Layout
      // [h][t][c][wm 2][i 4][half 2][lane 64] x 16 B (C = 128: h = c = 0); unit (i, half,
      // lane group, row) = 16 e4m3 bytes ci = 32 lq + 16 half + e
      const int u = threadIdx.x;  // 256 units, one per thread
      const int lr = u & 15, lql = (u >> 4) & 1, hf = (u >> 5) & 1, i = u >> 6;
      const int r = i * 16 + lr, c0 = 32 * lql + 16 * hf;
      uint32_t q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v4[k] = fmaxf(fminf(tileS[r][c0 + 4 * e + k] * inv8, 448.f), -448.f);
        int pkd = __builtin_amdgcn_cvt_pk_fp8_f32(v4[0], v4[1], 0, false);
        pkd = __builtin_amdgcn_cvt_pk_fp8_f32(v4[2], v4[3], pkd, true);
        q[e] = (uint32_t)pkd;
      }
      const int nc = L.cout / 128, h = cot >> 1, wm = cot & 1, c = cit >> 1;
      int st, lg;
      f8_step_of(nc, t, c, cit & 1, st, lg);
      const int lane = (lg + lql) * 16 + lr;
      L.wf8_frag[(((((size_t)h * 9 * nc + st) * 2 + wm) * 4 + i) * 2 + hf) * 64 + lane] =
          uint4{q[0], q[1], q[2], q[3]};
    }
    if (L.wd8_frag) {
      // dgrad operand A_d[ci][8 - t][co] = W[co][t][ci]: rows ci (pass h = cit / 2, co-half
      // wm = cit % 2), k = co (chunk c = cot / 2, lane groups 2 (cot % 2), +1) at tap 8 - t
      const int u = threadIdx.x;
      const int lr = u & 15, lql = (u >> 4) & 1, hf = (u >> 5) & 1, i = u >> 6;
      const int r = i * 16 + lr, c0 = 32 * lql + 16 * hf;
      uint32_t q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v4[k] = fmaxf(fminf(tileS[c0 + 4 * e + k][r] * inv8, 448.f), -448.f);
        int pkd = __builtin_amdgcn_cvt_pk_fp8_f32(v4[0], v4[1], 0, false);
        pkd = __builtin_amdgcn_cvt_pk_fp8_f32(v4[2], v4[3], pkd, true);
        q[e] = (uint32_t)pkd;
      }
      const int nc = L.cout / 128, h = cit >> 1, wm = cit & 1, c = cot >> 1;
      int st, lg;
      f8_step_of(nc, 8 - t, c, cot & 1, st, lg);
      const int lane = (lg + lql) * 16 + lr;
      L.wd8_frag[(((((size_t)h * 9 * nc + st) * 2 + wm) * 4 + i) * 2 + hf) * 64 + lane] =
          uint4{q[0], q[1], q[2], q[3]};
    }
    __syncthreads();
}

// this block's |w| max into its amax slot (fp8 layers; uniform per block, a plain store)
DG_DEV void refresh_amax(const WRefreshLayer& L, float wmax, float* s_amax) {
  if (L.s_w && L.amax_w) {
    wmax = wave_max(wmax);
    if ((threadIdx.x & 63) == 0) s_amax[threadIdx.x >> 6] = wmax;
    __syncthreads();
    if (threadIdx.x == 0)
      L.amax_w[blockIdx.x] =
          __float_as_uint(fmaxf(fmaxf(s_amax[0], s_amax[1]), fmaxf(s_amax[2], s_amax[3])));
  }
}

// pbias_frag unit of pixel q (0..383; pixels past 360 repeat 360) and channels c..c+3:
// element (((h * 24 + jg) * 2 + wm) * 4 + i) * 64 + lane, pixel jg*16 + (lane & 15),
// channels 128h + wm*64 + i*16 + (lane >> 4)*4 .. +3 — the stacks' accumulator-fragment
// order (one coalesced 512-B load per epilogue fragment)
DG_DEV size_t pbias_frag_index(int q, int c) {
  const int h = c >> 7, wm = (c >> 6) & 1, i = (c >> 4) & 3, lg = (c >> 2) & 3;
  return ((((size_t)h * 24 + (q >> 4)) * 2 + wm) * 4 + i) * 64 + lg * 16 + (q & 15);
}

// Tiled: one block per (layer, tap, 64 co x 64 ci tile); wf rows are written along ci and
// the flipped-tap transpose wd along co through a padded LDS tile, so every global store
// is a coalesced 128-B row piece (the per-element version scattered 2-byte dgrad stores
// and ran at ~12 us for 2.1M weights).  Block (0, 0) also applies the per-step learning
// rate decay lr *= (1 - decay) (the reference's SGD, optimizer.lua:25-26) when lr != 0:
// this kernel runs after the update kernel that reads lr, and nothing here reads it.
__global__ void __launch_bounds__(256)
weight_refresh_kernel(WRefreshArgs a, double* lr, double decay, long long* step) {
  if (lr && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    *lr = *lr * (1.0 - decay);
    if (step) *step += 1;
  }
  const WRefreshLayer L = a.L[blockIdx.y];
  const int nct = (L.cout + 63) / 64, nit = (L.cin + 63) / 64;
  const int tiles = L.taps * nct * nit;
  __shared__ float tileS[64][65];
  __shared__ float s_amax[4];
  float wmax = 0.f;
  const float inv8 = L.s_w ? 1.f / *L.s_w : 0.f;
  for (int tix = blockIdx.x; tix < tiles; tix += gridDim.x) {
    const int t = tix / (nct * nit);
    const int r = tix - t * nct * nit;
    const int cot = r / nit, cit = r - cot * nit;
    for (int e = threadIdx.x; e < 64 * 64; e += 256) {
      const int rr = e >> 6, cc = e & 63;
      const int co = cot * 64 + rr, ci = cit * 64 + cc;
      float v = 0.f;
      if (co < L.cout && ci < L.cin) {
        v = L.w[((size_t)co * L.taps + t) * L.cin + ci];
        refresh_elem(L, co, ci, t, v, inv8, wmax);
      }
      tileS[rr][cc] = v;
    }
    if (refresh_needs_tile(L)) {
      __syncthreads();
      refresh_tile_copies(L, t, cot, cit, tileS, inv8);
    }
  }
  refresh_amax(L, wmax, s_amax);
  if (L.pbias) {
    const int n = NPTS * L.cout;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256)
      L.pbias[e] = f2bf(L.bias[e % L.cout] + L.posb[e]);
  }
  if (L.pbias_frag) {
    const int ne = (L.cout / 128) * 24 * 2 * 4 * 64;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < ne; e += gridDim.x * 256) {
      const int lane = e & 63, i = (e >> 6) & 3, wm = (e >> 8) & 1, jg = (e >> 9) % 24,
                h = e / (24 * 512);
      int p = jg * 16 + (lane & 15);
      p = p < NPTS ? p : NPTS - 1;
      const int c = 128 * h + wm * 64 + i * 16 + (lane >> 4) * 4;
      const float* pb = L.posb + (size_t)p * L.cout + c;
      L.pbias_frag[e] = uint2{pack_bf16x2(L.bias[c] + pb[0], L.bias[c + 1] + pb[1]),
                              pack_bf16x2(L.bias[c + 2] + pb[2], L.bias[c + 3] + pb[3])};
    }
  }
}

// ------------------------------------------------------------------------------------
// The end of a training step in ONE launch: gradient second pass + optimizer + operand
// refresh + LR decay.  Replaces (slab reduce, bias pass 2, head-less SGD / RMSProp, weight
// refresh) — three launches, their idle gaps and the fp32 gradient round trip between them.
//
// Per conv layer l (grid.y = l) the gradient comes either from the weight-gradient kernels'
// split-K slabs and the bias partials (single-GPU training: nothing needs the reduced
// gradient before the update) or from the flat gradient (data parallel: the all-reduced
// buckets, fp32 or the bf16 wire twin).  The weight part runs on the weight_refresh tiling
// (64 co x 64 ci at one tap per tile): sum the slabs (the same fixed order as
// wgrad_reduce_kernel: bit-identical gradients), write the fp32 gradient, update the fp32
// master weight, and write the tile's operand copies from the updated values.  The bias
// part runs in its OWN blocks (blockIdx.x >= tblocks, beside the tile blocks rather than after
// their tiles — each block's chain of dependent memory round trips is the launch's limiter):
// a bias block recomputes the new per-channel bias of its 64-channel block (64 sums of R row
// partials), updates its share of the per-position biases, then writes the forward
// epilogue's bias tables from the new values.  Readers of an old value and the writer of its
// new value must not race: the per-channel biases and the learning rate are written by the
// LAST block to finish (atomic tickets taken after the block's reads; the counters are reset
// by that block, so the launch is graph-replayable).  The grid's ticket is a 3-level tree
// (16-block groups -> rows -> grid): device-scope atomics on ONE address serialize, and a
// flat grid ticket (1872 increments at 12x256) cost more than the rest of the launch.
// grid.y = n: the plain range (the head's parameters, whose gradient head_reduce already
// wrote).
//
// Non-finite gradient entries are not applied (the parameter keeps its value) and flag the
// step (bad_steps += 1 once); gate (device, optional) = 0 skips every update (a non-finite
// loss); the LR decays either way, as with the separate kernels.
// Reference: SGD step + LR decay (optimizer.lua:24-27); AdagradOptimizer (:1-14).
struct GUSrc {
  const float* slab;    // [splits][Mpad][KP], k = t * cinp + ci; null: the flat gradient
  const float* bpart;   // [bchunks][361][C] partials + [bchunks][19][C] row partials; or null
  int splits, Mpad, KP, bchunks;
  long long w_off, b_off, pos_off;   // element offsets into the flat P / G / MS
};
constexpr int MAX_GU = 20;
// bias work in channel blocks of GU_BCH (or all C when C is smaller): C <= 256 -> at most 4
// blocks per layer, one ticket each
constexpr int GU_BCH = 64;
DG_DEV int gu_bch(int C) { return C < GU_BCH ? C : GU_BCH; }
constexpr int GU_NB = 16;        // bias blocks per 64-channel block (of the widest layer)
constexpr int GU_TG = 16;        // blocks per first-level ticket group
constexpr int GU_MAXG = 64;      // groups per row (grid.x <= 1024)
// ticket layout (uint32): per (layer, channel block) | per row | per (row, group) | grid
constexpr int GU_T_ROW = 4 * MAX_GU;
constexpr int GU_T_GRP = GU_T_ROW + MAX_GU + 1;
constexpr int GU_T_GRID = GU_T_GRP + (MAX_GU + 1) * GU_MAXG;
constexpr int GU_T_PEND = GU_T_GRID + 1;   // a non-final launch's non-finite flag
constexpr int GU_TICKETS = GU_T_PEND + 1;
struct GUArgs {
  int n;
  int tblocks;         // blocks [0, tblocks) of a row: weight tiles; the rest: biases
  WRefreshLayer L[MAX_GU];
  GUSrc S[MAX_GU];
  long long plain_off, plain_n;
  float* P;
  float* G;            // fp32 gradient: read (no slab) or written (slab)
  const bf16_t* G16;   // bf16 wire twin to read instead of G (data parallel), or null
  float* MS;           // RMSProp mean square (same flat layout), or null: SGD
  float rms_decay, gscale;
  const float* gate;
  const double* lr;
  double decay;
  long long* step;
  unsigned* tickets;   // [GU_TICKETS] zeroed (the tree counters carry the non-finite flag
                       // << 16)
  int write_grads;     // slab mode: also write the reduced fp32 gradient (tests / tools)
  int* bad_steps;
  // the step tag the gradient producers set (dg_common.h; null: none): when it equals
  // *step + 1 NO parameter of this launch changes (all-or-nothing with the producers'
  // bounds; the per-entry non-finite skip below is only a last line)
  const long long* gflag;
  // 1: the step's last (or only) update launch — decays the LR, counts the step, consumes a
  // pending non-finite flag; 0: an earlier part (e.g. the hidden layers, issued as soon as
  // their gradients exist) — leaves the LR alone and parks its non-finite flag
  int final;
};

// one parameter's update; ms (RMSProp only) is updated in place
DG_DEV float gu_update(float p, float g, bool rms, float& ms, float l, float rms_decay,
                       float gscale, bool apply, unsigned& bad) {
  if (!isfinite(g)) {
    bad = 1u;
    return p;
  }
  if (!apply) return p;
  if (rms) {
    const float gi = g * gscale;
    const float m = rms_decay * ms + (1.f - rms_decay) * gi * gi;
    ms = m;
    return p - l * gi * rsqrtf(m);
  }
  return p - l * g;
}
// the same on flat element o (P, MS in global memory)
DG_DEV float gu_update_at(const GUArgs& a, long long o, float g, float l, bool apply,
                          unsigned& bad) {
  const bool rms = a.MS != nullptr;
  float ms = rms ? a.MS[o] : 0.f;
  const float v = gu_update(a.P[o], g, rms, ms, l, a.rms_decay, a.gscale, apply, bad);
  if (rms) a.MS[o] = ms;
  return v;
}

__global__ void __launch_bounds__(256) grad_update_kernel(GUArgs a) {
  __shared__ float tileS[64][65];
  __shared__ float s_amax[4];
  __shared__ float s_b[256];       // the layer's new per-channel bias,
  __shared__ float s_gb[256];      // its gradient
  __shared__ float s_ms[256];      // and mean square (RMSProp)
  __shared__ unsigned s_flag[2];
  const int ly = blockIdx.y;
  const int tid = threadIdx.x;
  const bool gate_ok = !(a.gate && *a.gate == 0.f);
  const bool tagged = a.gflag && a.step && *a.gflag == *a.step + 1;
  const bool apply = gate_ok && !tagged;
  // SGD: l = lr * gscale (as sgd_kernel); RMSProp: l = lr, gscale inside
  const float l = a.MS ? (float)(*a.lr) : (float)(*a.lr) * a.gscale;
  unsigned bad = 0u;
  if (tid == 0) s_flag[0] = 0u;
  __syncthreads();
  if (ly == a.n) {
    // the head: plain update from the flat gradient
    for (long long i = blockIdx.x * 256LL + tid; i < a.plain_n; i += gridDim.x * 256LL) {
      const long long o = a.plain_off + i;
      const float g = a.G16 ? bf2f(a.G16[o]) : a.G[o];
      a.P[o] = gu_update_at(a, o, g, l, apply, bad);
    }
  } else {
    const WRefreshLayer L = a.L[ly];
    const GUSrc S = a.S[ly];
    float* Pw = a.P + S.w_off;
    float* Gw = a.G + S.w_off;
    float* MSw = a.MS ? a.MS + S.w_off : nullptr;
    const int nct = (L.cout + 63) / 64, nit = (L.cin + 63) / 64;
    const int tiles = L.taps * nct * nit;
    float wmax = 0.f;
    const float inv8 = L.s_w ? 1.f / *L.s_w : 0.f;
    const size_t zstride = (size_t)S.Mpad * S.KP;
    const bool vec = S.slab && (L.cin & 3) == 0 && (L.cinp & 3) == 0 && (S.KP & 3) == 0;
    // the flat (all-reduced, data-parallel) gradient: 4 consecutive ci per thread too (the
    // per-element form below loaded one bf16 per lane: +8 us on the DP step at 12x128)
    const bool vecf = !S.slab && (L.cin & 3) == 0 && (S.w_off & 3) == 0;
    const bool tile_block = (int)blockIdx.x < a.tblocks;
    for (int tix = blockIdx.x; tile_block && tix < tiles; tix += a.tblocks) {
      const int t = tix / (nct * nit);
      const int r = tix - t * nct * nit;
      const int cot = r / nit, cit = r - cot * nit;
      if (vec) {
        // 4 consecutive ci per thread and unit, the tile's 4 units per thread summed together
        // (16 16-B slab loads in flight per thread; slab_sums4 = slab_sum4's order per element)
        const float* src[4];
        bool ok[4];
        f32x4 pp[4];   // the weights, loaded beside the slabs
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + 256 * u;
          const int rr = e4 >> 4, cc = (e4 & 15) * 4;
          const int co = cot * 64 + rr, ci = cit * 64 + cc;
          ok[u] = co < L.cout && ci < L.cin;
          src[u] = S.slab + (ok[u] ? (size_t)co * S.KP + t * L.cinp + ci : 0);
          const size_t o = ok[u] ? ((size_t)co * L.taps + t) * L.cin + ci : 0;
          pp[u] = *(const f32x4*)(Pw + o);
        }
        f32x4 gs[4];
        slab_sums4<4>(src, S.splits, zstride, gs);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + 256 * u;
          const int rr = e4 >> 4, cc = (e4 & 15) * 4;
          const int co = cot * 64 + rr, ci = cit * 64 + cc;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (ok[u]) {
            const f32x4 g4 = gs[u];
            const size_t o = ((size_t)co * L.taps + t) * L.cin + ci;
            if (a.write_grads) *(f32x4*)(Gw + o) = g4;
            const f32x4 p4 = pp[u];
            f32x4 m4 = {0.f, 0.f, 0.f, 0.f};
            if (MSw) m4 = *(const f32x4*)(MSw + o);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              float m = m4[k];
              v[k] = gu_update(p4[k], g4[k], MSw != nullptr, m, l, a.rms_decay, a.gscale, apply,
                               bad);
              m4[k] = m;
              refresh_elem(L, co, ci + k, t, v[k], inv8, wmax);
            }
            *(f32x4*)(Pw + o) = v;
            if (MSw) *(f32x4*)(MSw + o) = m4;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) tileS[rr][cc + k] = v[k];
        }
      } else if (vecf) {
        // the same 4-ci units over the flat gradient (G or its bf16 twin G16)
        f32x4 gs[4], pp[4];
        bool ok[4];
        size_t os[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + 256 * u;
          const int rr = e4 >> 4, cc = (e4 & 15) * 4;
          const int co = cot * 64 + rr, ci = cit * 64 + cc;
          ok[u] = co < L.cout && ci < L.cin;
          os[u] = ok[u] ? ((size_t)co * L.taps + t) * L.cin + ci : 0;
          gs[u] = a.G16 ? grad4_at(a.G16 + S.w_off, os[u] / 4) : *(const f32x4*)(Gw + os[u]);
          pp[u] = *(const f32x4*)(Pw + os[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int e4 = tid + 256 * u;
          const int rr = e4 >> 4, cc = (e4 & 15) * 4;
          const int co = cot * 64 + rr, ci = cit * 64 + cc;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (ok[u]) {
            f32x4 m4 = {0.f, 0.f, 0.f, 0.f};
            if (MSw) m4 = *(const f32x4*)(MSw + os[u]);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              float m = m4[k];
              v[k] = gu_update(pp[u][k], gs[u][k], MSw != nullptr, m, l, a.rms_decay, a.gscale,
                               apply, bad);
              m4[k] = m;
              refresh_elem(L, co, ci + k, t, v[k], inv8, wmax);
            }
            *(f32x4*)(Pw + os[u]) = v;
            if (MSw) *(f32x4*)(MSw + os[u]) = m4;
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) tileS[rr][cc + k] = v[k];
        }
      } else {
        for (int e = tid; e < 64 * 64; e += 256) {
          const int rr = e >> 6, cc = e & 63;
          const int co = cot * 64 + rr, ci = cit * 64 + cc;
          float v = 0.f;
          if (co < L.cout && ci < L.cin) {
            const size_t o = ((size_t)co * L.taps + t) * L.cin + ci;
            float g;
            if (S.slab) {
              g = slab_sum1(S.slab + (size_t)co * S.KP + t * L.cinp + ci, S.splits, zstride);
              if (a.write_grads) Gw[o] = g;
            } else {
              g = a.G16 ? bf2f(a.G16[S.w_off + o]) : Gw[o];
            }
            v = gu_update_at(a, S.w_off + o, g, l, apply, bad);
            Pw[o] = v;
            refresh_elem(L, co, ci, t, v, inv8, wmax);
          }
          tileS[rr][cc] = v;
        }
      }
      __syncthreads();    // tileS complete (also orders the next tile's writes after reads)
      if (refresh_needs_tile(L)) refresh_tile_copies(L, t, cot, cit, tileS, inv8);
    }
    if (tile_block) refresh_amax(L, wmax, s_amax);   // (slot blockIdx.x < tblocks <= 512)
    // ---- biases (blocks tblocks..), in channel blocks of 64: bias block (cb, pb) = channels
    // 64 cb .. +63 over position range pb.  Each recomputes the NEW per-channel bias of its 64
    // channels only (64 sums of R row partials), updates its positions' per-position biases
    // and writes those entries of the bias tables.
    const int C = L.cout;
    const int bch = gu_bch(C);
    const int ncb = C / bch;
    const int nbb = (int)gridDim.x - a.tblocks;
    const int npb = nbb / ncb;
    const int bidx = (int)blockIdx.x - a.tblocks;
    const int cb = bidx % ncb, pb = bidx / ncb;
    if (!tile_block && pb < npb) {
      const int c0 = cb * bch;
      const int R = S.bchunks * BOARD;
      const float* rowpart = S.bpart ? S.bpart + (size_t)S.bchunks * NPTS * C : nullptr;
      if (tid < 4 * bch) {            // one lane quad per channel (rows_sum4)
        const int cl = tid >> 2, c = c0 + cl;
        float g;
        if (S.bpart) {
          g = rows_sum4(rowpart, R, C, c, tid & 3);
        } else {
          const long long o = S.b_off + c;
          g = a.G16 ? bf2f(a.G16[o]) : a.G[o];
        }
        if ((tid & 3) == 0) {
          float ms_v = a.MS ? a.MS[S.b_off + c] : 0.f;
          s_b[cl] = gu_update(a.P[S.b_off + c], g, a.MS != nullptr, ms_v, l, a.rms_decay,
                              a.gscale, apply, bad);
          // (the per-channel bias, its gradient and mean square are written by the last
          // block of this channel block below: the others still read the old values here)
          s_gb[cl] = g;
          s_ms[cl] = ms_v;
        }
      }
      __syncthreads();
      const size_t np = (size_t)NPTS * C;
      const int p0 = pb * NPTS / npb, p1 = (pb + 1) * NPTS / npb;
      for (int it = tid; it < (p1 - p0) * (bch / 4); it += 256) {
        const int p = p0 + it / (bch / 4), cl = (it % (bch / 4)) * 4, c = c0 + cl;
        const size_t j = (size_t)p * C + c;
        f32x4 g4;
        if (S.bpart) {
#pragma unroll
          for (int k = 0; k < 4; ++k) g4[k] = chunk_sum(S.bpart + j + k, S.bchunks, np);
          if (a.write_grads) *(f32x4*)(a.G + S.pos_off + j) = g4;
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k)
            g4[k] = a.G16 ? bf2f(a.G16[S.pos_off + j + k]) : a.G[S.pos_off + j + k];
        }
        float nb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float v = gu_update_at(a, S.pos_off + j + k, g4[k], l, apply, bad);
          a.P[S.pos_off + j + k] = v;
          nb[k] = s_b[cl + k] + v;
          if (L.pbias) L.pbias[j + k] = f2bf(nb[k]);
        }
        if (L.pbias_frag) {
          const uint2 u = uint2{pack_bf16x2(nb[0], nb[1]), pack_bf16x2(nb[2], nb[3])};
          L.pbias_frag[pbias_frag_index(p, c)] = u;
          if (p == NPTS - 1)
            for (int q = NPTS; q < 24 * 16; ++q) L.pbias_frag[pbias_frag_index(q, c)] = u;
        }
      }
    }
  }
  // ---- tickets: the last block of each (layer, channel block) writes its per-channel biases;
  // the grid's last block decays the LR, counts a step with a non-finite gradient entry and
  // resets the flag.  No fences: every block's reads of an old value (lr, the per-channel
  // biases) have returned before its ticket is taken (their values were consumed before the
  // barrier), and the writers act only after seeing the final ticket; the new values are read
  // by later launches.  The grid ticket carries the non-finite flag in its high half.
  if (bad) s_flag[0] = 1u;     // (benign same-value race)
  __syncthreads();
  int cbw = -1;   // the channel block this block closes (last of its position blocks)
  if (ly < a.n && (int)blockIdx.x >= a.tblocks) {
    const int ncb = a.L[ly].cout / gu_bch(a.L[ly].cout);
    const int npb = ((int)gridDim.x - a.tblocks) / ncb;
    const int bidx = (int)blockIdx.x - a.tblocks;
    const int cb = bidx % ncb, pb = bidx / ncb;
    if (pb < npb) {
      if (tid == 0)
        s_flag[1] = atomicAdd(&a.tickets[4 * ly + cb], 1u) == (unsigned)npb - 1 ? 1u : 0u;
      __syncthreads();
      if (s_flag[1]) cbw = cb;
    }
  }
  if (cbw >= 0) {
    const GUSrc S = a.S[ly];
    const int bch = gu_bch(a.L[ly].cout);
    if (tid < bch) {
      const int c = cbw * bch + tid;
      a.P[S.b_off + c] = s_b[tid];
      if (S.bpart && a.write_grads) a.G[S.b_off + c] = s_gb[tid];
      if (a.MS) a.MS[S.b_off + c] = s_ms[tid];
    }
    if (tid == 0) a.tickets[4 * ly + cbw] = 0u;
  }
  if (tid == 0) {
    // 3-level ticket tree: group of GU_TG blocks -> row -> grid; the last arrival at each
    // level resets its counter and moves up, carrying the non-finite flag in the high half
    unsigned* T = a.tickets;
    const unsigned g = blockIdx.x / GU_TG;
    const unsigned ng = (gridDim.x + GU_TG - 1) / GU_TG;
    const unsigned gsize = min((unsigned)GU_TG, gridDim.x - g * GU_TG);
    unsigned flag = s_flag[0] ? 0x10000u : 0u;
    unsigned* tg = T + GU_T_GRP + ly * GU_MAXG + g;
    unsigned old = atomicAdd(tg, 1u + flag);
    if ((old & 0xFFFFu) == gsize - 1) {
      *tg = 0u;
      flag = ((old >> 16) != 0u || flag) ? 0x10000u : 0u;
      old = atomicAdd(T + GU_T_ROW + ly, 1u + flag);
      if ((old & 0xFFFFu) == ng - 1) {
        T[GU_T_ROW + ly] = 0u;
        flag = ((old >> 16) != 0u || flag) ? 0x10000u : 0u;
        old = atomicAdd(T + GU_T_GRID, 1u + flag);
        if ((old & 0xFFFFu) == gridDim.y - 1) {
          const bool flagged = (old >> 16) != 0u || flag;
          if (a.final) {
            double* lrw = const_cast<double*>(a.lr);
            *lrw = *lrw * (1.0 - a.decay);
            if (a.step) *a.step += 1;
            // (a non-finite loss was counted by the gate kernel; a tagged step here)
            const bool any = flagged || tagged || T[GU_T_PEND] != 0u;
            if (any && a.bad_steps && gate_ok) *a.bad_steps += 1;
            T[GU_T_PEND] = 0u;
          } else if (flagged) {
            T[GU_T_PEND] = 1u;
          }
          T[GU_T_GRID] = 0u;
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// Stand-in for a ring all-reduce on ONE GPU (bench.py --force-dp --comm proxy; the real
// collective needs peers): a small grid (RCCL drives a ring with a few channel workgroups)
// streams 2(n-1)/n x the bucket's bytes through HBM (read + write back, values unchanged),
// paced by s_memrealtime (100 MHz) so it lasts as long as the wire transfer would at the
// given link rate.  Its kernel trace shows whether such a comm-stream kernel co-schedules
// beside the step's compute launches (tools/overlap_report.py).
__global__ void __launch_bounds__(256) comm_proxy_kernel(float4* __restrict__ buf, long long n4,
                                                         long long moves,
                                                         long long dur_ticks) {
  const long long per = (moves + gridDim.x - 1) / gridDim.x;
  const long long lo = (long long)blockIdx.x * per;
  const long long hi = lo + per < moves ? lo + per : moves;
  if (lo >= hi) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (long long base = lo; base < hi; base += blockDim.x) {
    if (dur_ticks > 0) {
      const unsigned long long due =
          t0 + (unsigned long long)((double)(base - lo) / (double)(hi - lo) * (double)dur_ticks);
      while (__builtin_amdgcn_s_memrealtime() < due) __builtin_amdgcn_s_sleep(4);
    }
    const long long i = base + threadIdx.x;
    if (i < hi) {
      const long long j = i % n4;
      float4 v = buf[j];
      asm volatile("" : "+v"(v.x));
      buf[j] = v;
    }
  }
}
}  // namespace

extern "C" {

hipError_t dg_expand_features(const uint8_t* planes, const uint8_t* player, const uint8_t* rank,
                              void* out, int B, int pad, int CP, void* out2, int CP2,
                              hipStream_t s) {
  if (CP % 8 != 0 || CP < 40 || CP > 48) return hipErrorInvalidValue;
  if (out2 && (CP2 % 8 != 0 || CP2 < CP)) return hipErrorInvalidValue;
  const int n = B * NPTS;
  hipLaunchKernelGGL(expand_features_kernel, dim3((n + 255) / 256), dim3(256), 0, s, planes,
                     player, rank, (char*)out, B, pad, CP, (char*)out2, CP2);
  return hipGetLastError();
}

// part must hold nchunks*(361 + 19)*C floats, nchunks = ceil(B / 16)
hipError_t dg_bias_grad_partial(const void* dZ, int B, int C, int pad, float* part,
                                hipStream_t s) {
  if (C % 8 != 0 || C > 2048) return hipErrorInvalidValue;
  const int nchunks = (B + BG_BT - 1) / BG_BT;
  int threads = (BOARD * (C / 8) + 63) / 64 * 64;  // one item per thread (19*C/8)
  if (threads > 1024) threads = 1024;
  if (threads < 64) threads = 64;
  BiasLayers Ls{};
  Ls.dZ[0] = (const char*)dZ;
  Ls.part[0] = part;
  hipLaunchKernelGGL(bias_grad_partial_kernel<BG_LD>, dim3(BOARD, nchunks, 1), dim3(threads),
                     (size_t)BOARD * C * sizeof(float), s, Ls, B, C, pad, nchunks, BG_BT);
  return hipGetLastError();
}

// Pass 1 for nl same-shape layers in one launch: table = nl rows of {dZ frame, part, s8}
// (s8: 0 = bf16 frame, else the e5m2 copy's scale pointer; pad must be 1 then);
// chunks of BG_BT_MULTI boards (dg_bias_chunks_multi).
hipError_t dg_bias_grad_partial_multi(const long long* table, int nl, int B, int C, int pad,
                                      long long* sf, hipStream_t s) {
  if (C % 8 != 0 || C > 2048 || nl <= 0 || nl > BG_MAXL) return hipErrorInvalidValue;
  const int nchunks = (B + BG_BT_MULTI - 1) / BG_BT_MULTI;
  int threads = (BOARD * (C / 8) + 63) / 64 * 64;
  if (threads > 256) threads = 256;
  if (threads < 64) threads = 64;
  BiasLayers Ls{};
  for (int i = 0; i < nl; ++i) {
    Ls.dZ[i] = (const char*)table[3 * i];
    Ls.part[i] = (float*)table[3 * i + 1];
    Ls.s8[i] = (const float*)table[3 * i + 2];
    if (Ls.s8[i] && pad != 1) return hipErrorInvalidValue;
  }
  Ls.sf = sf;
  hipLaunchKernelGGL(bias_grad_partial_kernel<2>, dim3(BOARD, nchunks, nl), dim3(threads),
                     (size_t)BOARD * C * sizeof(float), s, Ls, B, C, pad, nchunks, BG_BT_MULTI);
  return hipGetLastError();
}
int dg_bias_chunks(int B) { return (B + BG_BT - 1) / BG_BT; }
int dg_bias_chunks_multi(int B) { return (B + BG_BT_MULTI - 1) / BG_BT_MULTI; }

// g16 (optional): read the bf16 twin gradient instead of g (data-parallel bf16 wire)
hipError_t dg_sgd(float* p, const float* g, size_t n, const double* lr, float gscale,
                  const float* gate, const void* g16, hipStream_t s) {
  int blocks = (int)((n / 4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  if (g16)
    hipLaunchKernelGGL(sgd_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, p,
                       (const bf16_t*)g16, n, lr, gscale, gate);
  else
    hipLaunchKernelGGL(sgd_kernel<float>, dim3(blocks), dim3(256), 0, s, p, g, n, lr, gscale,
                       gate);
  return hipGetLastError();
}

hipError_t dg_rmsprop(float* p, const float* g, float* ms, size_t n, const double* lr,
                      float decay, float gscale, const float* gate, const void* g16,
                      hipStream_t s) {
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (g16)
    hipLaunchKernelGGL(rmsprop_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, p,
                       (const bf16_t*)g16, ms, n, lr, decay, gscale, gate);
  else
    hipLaunchKernelGGL(rmsprop_kernel<float>, dim3(blocks), dim3(256), 0, s, p, g, ms, n, lr,
                       decay, gscale, gate);
  return hipGetLastError();
}

// loss (optional, rank-local) and grads (optional, flat, all-reduced; or its bf16 twin
// grads16) -> gate in {0, 1}
hipError_t dg_finite_gate(const float* loss, int n, const float* grads, size_t ng, float* gate,
                          int* bad_count, const void* grads16, hipStream_t s) {
  if (loss) {
    hipLaunchKernelGGL(finite_gate_kernel, dim3(1), dim3(256), 0, s, loss, n, gate, bad_count);
  } else {
    hipLaunchKernelGGL(set_gate_kernel, dim3(1), dim3(64), 0, s, gate);
  }
  if ((grads || grads16) && ng) {
    int blocks = (int)((ng / 4 + 255) / 256);
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    if (grads16)
      hipLaunchKernelGGL(grad_gate_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s,
                         (const bf16_t*)grads16, ng, gate, bad_count);
    else
      hipLaunchKernelGGL(grad_gate_kernel<float>, dim3(blocks), dim3(256), 0, s, grads, ng,
                         gate, bad_count);
  }
  return hipGetLastError();
}

// gate = finite(loss) && finite(grads | grads16) in one launch (gate_all_kernel); ticket: one
// zeroed word the launch leaves zeroed
hipError_t dg_finite_gate1(const float* loss, int n, const float* grads, const void* grads16,
                           size_t ng, float* gate, int* bad_count, unsigned* ticket,
                           hipStream_t s) {
  if (!gate || !ticket) return hipErrorInvalidValue;
  // (<= 256 blocks: the tickets serialize on one address, ~11 ns each — 1024 blocks cost
  // 15 us at 2.1M gradients, more than the scan; 128 blocks of 4 loads in flight per lane
  // were latency-bound at 7.2M: 12.7 us)
  int blocks = 1;
  if ((grads || grads16) && ng) {
    blocks = (int)((ng / 4 + 2047) / 2048);
    if (blocks > 256) blocks = 256;
    if (blocks < 1) blocks = 1;
  }
  if (grads16)
    hipLaunchKernelGGL(gate_all_kernel<bf16_t>, dim3(blocks), dim3(256), 0, s, loss, n,
                       (const bf16_t*)grads16, ng, gate, bad_count, ticket);
  else
    hipLaunchKernelGGL(gate_all_kernel<float>, dim3(blocks), dim3(256), 0, s, loss, n,
                       grads, grads ? ng : (size_t)0, gate, bad_count, ticket);
  return hipGetLastError();
}

hipError_t dg_lr_decay(double* lr, double decay, long long* step, hipStream_t s) {
  hipLaunchKernelGGL(lr_decay_kernel, dim3(1), dim3(64), 0, s, lr, decay, step);
  return hipGetLastError();
}

// layers: n entries of 20 int64 words
//   {w, wf, wd, cout, cin, taps, cinp, kpf, kpd, pbias_frag, wf8, s_w, amax_w, bias, posb,
//    pbias, wf_frag, wd_frag, wf8_frag, wd8_frag}  (pbias_frag / *_frag: stack-order tables,
//    or 0)
// lr (optional): fused per-step decay lr *= (1 - decay), step += 1 (see the kernel).
static hipError_t parse_refresh_row(const long long* t, WRefreshLayer& L) {
  L.w = (const float*)t[0];
  L.wf = (bf16_t*)t[1];
  L.wd = (bf16_t*)t[2];
  L.cout = (int)t[3];
  L.cin = (int)t[4];
  L.taps = (int)t[5];
  L.cinp = (int)t[6];
  L.kpf = (int)t[7];
  L.kpd = (int)t[8];
  L.wf8 = (uint8_t*)t[10];
  L.s_w = (const float*)t[11];
  L.amax_w = (unsigned*)t[12];
  L.bias = (const float*)t[13];
  L.posb = (const float*)t[14];
  L.pbias = (bf16_t*)t[15];
  L.pbias_frag = (uint2*)t[9];
  if (L.pbias_frag && L.cout != 128 && L.cout != 256) return hipErrorInvalidValue;
  L.wf_frag = (uint4*)t[16];
  L.wd_frag = (uint4*)t[17];
  if (L.wf8 && !L.s_w) return hipErrorInvalidValue;
  if (L.wf_frag && L.taps != 9 &&   // the fused-first-layer layout (l1 mode)
      (L.wd_frag || (L.cout != 128 && L.cout != 256) || L.cin > 64 || L.cinp % 8 != 0 ||
       L.taps * L.cinp > 1024))
    return hipErrorInvalidValue;
  L.wf8_frag = (uint4*)t[18];
  L.wd8_frag = (uint4*)t[19];
  if ((L.wf8_frag || L.wd8_frag) &&
      (!L.s_w || L.taps != 9 || L.cout != L.cin || (L.cout != 128 && L.cout != 256)))
    return hipErrorInvalidValue;
  if (L.wd_frag && L.taps != 9) return hipErrorInvalidValue;
  if ((L.wf_frag || L.wd_frag) && L.taps == 9 &&
      (L.cout != L.cin || (L.cout != 128 && L.cout != 256)))
    return hipErrorInvalidValue;
  return hipSuccess;
}
static int refresh_tiles(const WRefreshLayer& L) {
  return L.taps * ((L.cout + 63) / 64) * ((L.cin + 63) / 64);
}

hipError_t dg_weight_refresh(const long long* table, int n, double* lr, double decay,
                             long long* step, hipStream_t s) {
  if (n <= 0 || n > MAX_REFRESH) return hipErrorInvalidValue;
  WRefreshArgs a;
  a.n = n;
  int maxtotal = 1;
  for (int i = 0; i < n; ++i) {
    const hipError_t e = parse_refresh_row(table + 20 * i, a.L[i]);
    if (e != hipSuccess) return e;
    const int tiles = refresh_tiles(a.L[i]);
    if (tiles > maxtotal) maxtotal = tiles;
  }
  const int blocks = maxtotal < REFRESH_PARTS ? maxtotal : REFRESH_PARTS;
  hipLaunchKernelGGL(weight_refresh_kernel, dim3(blocks, n), dim3(256), 0, s, a, lr, decay, step);
  return hipGetLastError();
}

// The fused gradient pass 2 + optimizer + refresh (grad_update_kernel).  table: n rows of
// GU_COLS int64 = the 20 weight_refresh columns, then {slab, bpart, splits, Mpad, KP,
// bchunks, w_off, b_off, pos_off} (slab / bpart 0: the layer's gradient is read from G / G16).
// plain_off / plain_n: a flat range updated from G only (the head).  tickets:
// dg_grad_update_tickets() zeroed uint32 (left zeroed).  write_grads: with slabs, also store
// the reduced gradient in G.  Tile blocks per row = dg_weight_refresh's block count (the fp8
// |w| max slots), plus GU_NB bias blocks per 64-channel block of the widest layer.
constexpr int GU_COLS = 29;
int dg_grad_update_cols() { return GU_COLS; }
int dg_grad_update_tickets() { return GU_TICKETS; }
hipError_t dg_grad_update(const long long* table, int n, long long plain_off, long long plain_n,
                          float* P, float* G, const void* G16, float* MS, float rms_decay,
                          float gscale, const float* gate, double* lr, double decay,
                          long long* step, unsigned* tickets, int* bad_steps, int write_grads,
                          int final, const long long* gflag, hipStream_t s) {
  if (n <= 0 || n > MAX_GU || !P || !G || !lr || !tickets || plain_n < 0)
    return hipErrorInvalidValue;
  GUArgs a;
  a.n = n;
  int maxtotal = 1, maxncb = 1;
  for (int i = 0; i < n; ++i) {
    const long long* t = table + GU_COLS * i;
    WRefreshLayer& L = a.L[i];
    const hipError_t e = parse_refresh_row(t, L);
    if (e != hipSuccess) return e;
    if (L.cout > 256 || L.cout % 4 != 0 || (L.cout > GU_BCH && L.cout % GU_BCH != 0))
      return hipErrorInvalidValue;
    GUSrc& S = a.S[i];
    S.slab = (const float*)t[20];
    S.bpart = (const float*)t[21];
    S.splits = (int)t[22];
    S.Mpad = (int)t[23];
    S.KP = (int)t[24];
    S.bchunks = (int)t[25];
    S.w_off = t[26];
    S.b_off = t[27];
    S.pos_off = t[28];
    if (S.slab && (S.splits <= 0 || S.Mpad < L.cout || S.KP < L.taps * L.cinp))
      return hipErrorInvalidValue;
    if (S.bpart && S.bchunks <= 0) return hipErrorInvalidValue;
    if (L.w != P + S.w_off || L.bias != P + S.b_off || L.posb != P + S.pos_off)
      return hipErrorInvalidValue;   // the refresh row must describe the same parameters
    const int tiles = refresh_tiles(L);
    if (tiles > maxtotal) maxtotal = tiles;
    const int ncb = L.cout > GU_BCH ? L.cout / GU_BCH : 1;
    if (ncb > maxncb) maxncb = ncb;
  }
  a.plain_off = plain_off;
  a.plain_n = plain_n;
  a.P = P;
  a.G = G;
  a.G16 = (const bf16_t*)G16;
  a.MS = MS;
  a.rms_decay = rms_decay;
  a.gscale = gscale;
  a.gate = gate;
  a.lr = lr;
  a.decay = decay;
  a.step = step;
  a.tickets = tickets;
  a.bad_steps = bad_steps;
  a.write_grads = write_grads;
  a.final = final;
  a.gflag = gflag;
  a.tblocks = maxtotal < REFRESH_PARTS ? maxtotal : REFRESH_PARTS;
  const int blocks = a.tblocks + GU_NB * maxncb;
  if (blocks > GU_TG * GU_MAXG) return hipErrorInvalidValue;   // the ticket tree's groups
  hipLaunchKernelGGL(grad_update_kernel, dim3(blocks, n + 1), dim3(256), 0, s, a);
  return hipGetLastError();
}

// nbytes of a bucket (multiple of 16), world = the ring size it stands in for, gbps = link
// rate (GB/s; 0 = unpaced), blocks = channel workgroups
hipError_t dg_comm_proxy(void* buf, long long nbytes, int world, double gbps, int blocks,
                         hipStream_t s) {
  if (!buf || nbytes < 16 || nbytes % 16 != 0 || world < 2 || blocks < 1 || blocks > 1024)
    return hipErrorInvalidValue;
  const long long n4 = nbytes / 16;
  const long long moves = (long long)((double)n4 * 2.0 * (world - 1) / world);
  const double wire = (double)nbytes * 2.0 * (world - 1) / world;
  const long long ticks = gbps > 0 ? (long long)(wire / (gbps * 1e9) * 1e8) : 0;
  hipLaunchKernelGGL(comm_proxy_kernel, dim3(blocks), dim3(256), 0, s, (float4*)buf, n4,
                     moves, ticks);
  return hipGetLastError();
}

}  // extern "C"
