// Fused policy head: the last (c_out = 1) conv of the stack, its per-channel and untied
// per-position biases, the head ReLU, LogSoftMax over 361 points, mean ClassNLL, top-1
// argmax, and the whole backward of that block, one workgroup per board.
//
// Reference: getBasicModel's last iteration + Reshape(361) + LogSoftMax
// (experiments.lua:135-151), nn.ClassNLLCriterion (experiments.lua:45), Tensor:max(2) /
// ne / sum for accuracy (train.lua:29,36).  The reference runs these as ~8 separate
// cunn kernels; here they are a single pass over the board held on-chip.
//
// M = 1 makes MFMA pointless (GEMV-shaped), so the dot products run on the VALU.  The
// board's zero-bordered activation frame is staged into LDS in 128-channel chunks with
// wide independent loads (one HBM pass per chunk); the forward dots, the input gradient
// and the weight-gradient partials all read it from LDS.  Lane mapping: 16 lanes cover
// the 16 8-channel groups of one pixel (256 contiguous bytes -> conflict-free
// ds_read_b128), 4 pixels per wave.
#include <stdlib.h>

#include "dg_common.h"

using namespace dg;

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2v;

namespace {

constexpr int HT = 512;      // threads per board (8 waves: 2 per SIMD)
constexpr int CCH = 128;     // channels staged per chunk (64-ch chunks / 2 boards per CU
                             // measured 79 vs 58 us: the backward re-stages every chunk)
constexpr int GC = CCH / 8;  // 8-channel groups per chunk (16)

struct HeadArgs {
  const char* X;        // last hidden activation frame [B][F][F][C] bf16
  const float* w;       // head weights OHWI [1][KW][KW][C] fp32 (master)
  const float* bias;    // [1]
  const float* posb;    // [361]
  const int* labels;    // [B] (0..360) ; may be null in eval
  float* loss;          // [B]  -log p(label)
  int* pred;            // [B]  argmax
  float* logp_out;      // [B][361] optional (null = skip)
  char* dZ;             // gradient frame of the last hidden layer (null = eval only)
  float* gw_part;       // [B][KW*KW*C] per-board weight-grad partials (plain stores)
  float* gbias;         // unused (head_reduce computes it)
  float* dzb;           // [B][361] per-board d loss / d z (plain stores)
  int B;
  int C;
  int x_pad;
  int dz_pad;
  int head_relu;
  float grad_scale;     // 1 / global batch (mean NLL)
};

DG_DEV float dot2(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, a),
                                         __builtin_bit_cast(bf16x2v, b), c, false);
}

DG_DEV void unpack8(const uint4 v, float* f) {
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xFFFF0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xFFFF0000u);
  f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xFFFF0000u);
  f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xFFFF0000u);
}

template <int KW>
__global__ void __launch_bounds__(HT) head_kernel(HeadArgs a) {
  constexpr int R = (KW - 1) / 2;
  constexpr int T = KW * KW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int C = a.C;
  const int F = BOARD + 2 * a.x_pad;
  const int FF = F * F;
  const int cc = C < CCH ? C : CCH;         // channels per chunk
  const int gcc = cc / 8;                   // groups per chunk
  const int nchunk = C / cc;
  // LDS carve (16-B aligned pieces)
  char* s_x = smem;                                   // [FF][cc] bf16
  // s_x is padded to whole 1-KiB DMA wave-instructions (64 pieces of 16 B): the tail
  // instruction writes all 64 lanes' destinations.
  const int xbytes = ((FF * gcc + 63) / 64) * 64 * 16;
  float* s_w = (float*)(smem + xbytes);               // [T][C]
  float* s_z = s_w + T * C;                           // [384]
  float* s_dz = s_z + 384;                            // [384]
  float* s_gw = s_dz + 384;                           // [T][cc] dw partial (chunk)
  float* s_red = s_gw + T * CCH;                      // [HT]
  int* s_redi = (int*)(s_red + HT);                   // [HT]

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const char* Xb = a.X + (size_t)b * FF * C * 2;

  for (int i = tid; i < T * C; i += HT) s_w[i] = a.w[i];
  for (int p = tid; p < 384; p += HT) s_z[p] = 0.f;

  auto stage_chunk = [&](int ch) {
    // LDS-DMA: piece i (frame pixel f = i / gcc, group g) lands at byte 16*i of s_x, which is
    // exactly the lane-linear destination of global_load_lds_dwordx4 (base + lane*16).
    const int pieces = FF * gcc;
    for (int i0 = wave * 64; i0 < pieces; i0 += HT) {
      int i = i0 + lane;
      if (i >= pieces) i = pieces - 1;  // duplicate last piece: same bytes, same address
      const int f = i / gcc, g = i - (i / gcc) * gcc;
      glds16(Xb + ((size_t)f * C + ch * cc + g * 8) * 2, (LDS_AS void*)(s_x + i0 * 16));
    }
    __builtin_amdgcn_s_waitcnt(0);  // (vmcnt=0) this wave's DMA landed; barrier follows
  };

  // lane -> (pixel slot, group): 16 lanes per pixel when gcc == 16
  const int lg = lane % gcc;                 // group within chunk
  const int lpix = lane / gcc;               // pixel slot within wave
  const int ppw = 64 / gcc;                  // pixels per wave-iteration
  const int lanes_used = ppw * gcc;

  // ---------------- forward: z[p] = sum_{t,c} w[t][c] X[p+off(t)][c] ----------------
  // weights of this lane's channel group live in registers as packed bf16 pairs;
  // v_dot2_f32_bf16 consumes the staged bf16 activations without unpacking.
  for (int ch = 0; ch < nchunk; ++ch) {
    __syncthreads();
    stage_chunk(ch);
    __syncthreads();
    uint32_t wp[T][4];
#pragma unroll
    for (int t = 0; t < T; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float* wt = s_w + t * C + ch * cc + lg * 8 + 2 * e;
        wp[t][e] = pack_bf16x2(wt[0], wt[1]);
      }
    for (int p0 = wave * ppw; p0 < NPTS; p0 += (HT / 64) * ppw) {
      const int p = p0 + lpix;
      float acc = 0.f;
      if (p < NPTS && lane < lanes_used) {
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
        // four independent accumulation chains (one serial chain of 4T dot2 was latency
        // bound at 2 waves per SIMD)
        float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const int f = (h + a.x_pad + t / KW - R) * F + (w + a.x_pad + t % KW - R);
          const uint4 xv = *(const uint4*)(s_x + (f * cc + lg * 8) * 2);
          a0 = dot2(xv.x, wp[t][0], a0);
          a1 = dot2(xv.y, wp[t][1], a1);
          a2 = dot2(xv.z, wp[t][2], a2);
          a3 = dot2(xv.w, wp[t][3], a3);
        }
        acc = (a0 + a1) + (a2 + a3);
      }
      // reduce over the gcc lanes of this pixel
      for (int o = gcc / 2; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
      if (p < NPTS && lg == 0 && lane < lanes_used) s_z[p] += acc;
    }
  }
  __syncthreads();
  for (int p = tid; p < NPTS; p += HT) s_z[p] += a.bias[0] + a.posb[p];
  __syncthreads();

  // ---------------- log-softmax over 361 logits (logit = relu(z) if head_relu) --------
  float m = -INFINITY;
  int am = 0;
  for (int p = tid; p < NPTS; p += HT) {
    const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
    if (l > m) { m = l; am = p; }
  }
  // (max, lowest argmax) over the workgroup: wave shuffles, then the 8 wave results
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oi = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oi < am)) { m = om; am = oi; }
  }
  if (lane == 0) { s_red[wave] = m; s_redi[wave] = am; }
  __syncthreads();
  float mx = s_red[0];
  int amax = s_redi[0];
#pragma unroll
  for (int w8 = 1; w8 < HT / 64; ++w8) {
    const float o = s_red[w8];
    const int oi = s_redi[w8];
    if (o > mx || (o == mx && oi < amax)) { mx = o; amax = oi; }
  }
  float se = 0.f;
  for (int p = tid; p < NPTS; p += HT) {
    const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
    se += __expf(l - mx);
  }
  se = wave_sum(se);
  __syncthreads();  // everyone has read s_red / s_redi
  if (lane == 0) s_red[wave] = se;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int w8 = 0; w8 < HT / 64; ++w8) tot += s_red[w8];
  const float lse = mx + __logf(tot);
  const int y = a.labels ? a.labels[b] : -1;
  if (tid == 0) {
    if (a.pred) a.pred[b] = amax;
    if (a.loss && y >= 0) {
      const float ly = a.head_relu ? fmaxf(s_z[y], 0.f) : s_z[y];
      a.loss[b] = lse - ly;
    }
  }
  if (a.logp_out) {
    for (int p = tid; p < NPTS; p += HT) {
      const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
      a.logp_out[(size_t)b * NPTS + p] = l - lse;
    }
  }
  if (a.dZ == nullptr) return;

  // ---------------- backward: dz = (softmax - onehot) * scale * relu'(z) --------------
  for (int p = tid; p < 384; p += HT) {
    float d = 0.f;
    if (p < NPTS) {
      const float z = s_z[p];
      const float l = a.head_relu ? fmaxf(z, 0.f) : z;
      d = (__expf(l - lse) - (p == y ? 1.f : 0.f)) * a.grad_scale;
      if (a.head_relu && !(z > 0.f)) d = 0.f;
      a.dzb[(size_t)b * NPTS + p] = d;
    }
    s_dz[p] = d;
  }

  const int Fd = BOARD + 2 * a.dz_pad;
  char* dZb = a.dZ + (size_t)b * Fd * Fd * C * 2;
  // chunk order: the last staged chunk is still in LDS; walk chunks backwards
  for (int ci = nchunk - 1; ci >= 0; --ci) {
    __syncthreads();
    if (ci != nchunk - 1) stage_chunk(ci);
    for (int i = tid; i < T * CCH; i += HT) s_gw[i] = 0.f;
    __syncthreads();
    // ---- dX[q][c] = sum_t w[t][c] dz[q - off(t)], masked by X[q][c] > 0 ----
    {
      const int g = tid % gcc;  // HT is a multiple of gcc: fixed group per thread
      float wr[T][8];
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) wr[t][e] = s_w[t * C + ci * cc + g * 8 + e];
      for (int idx = tid; idx < NPTS * gcc; idx += HT) {
        const int q = idx / gcc;
        const int h = q / BOARD, w = q - (q / BOARD) * BOARD;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const int ph = h - (t / KW - R), pw = w - (t % KW - R);
          const bool in = ph >= 0 && ph < BOARD && pw >= 0 && pw < BOARD;
          const float d = in ? s_dz[ph * BOARD + pw] : 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] += d * wr[t][e];
        }
        float xm[8];
        unpack8(*(const uint4*)(s_x + (((h + a.x_pad) * F + (w + a.x_pad)) * cc + g * 8) * 2), xm);
        uint4 o;
        o.x = pack_bf16x2(xm[0] > 0.f ? v[0] : 0.f, xm[1] > 0.f ? v[1] : 0.f);
        o.y = pack_bf16x2(xm[2] > 0.f ? v[2] : 0.f, xm[3] > 0.f ? v[3] : 0.f);
        o.z = pack_bf16x2(xm[4] > 0.f ? v[4] : 0.f, xm[5] > 0.f ? v[5] : 0.f);
        o.w = pack_bf16x2(xm[6] > 0.f ? v[6] : 0.f, xm[7] > 0.f ? v[7] : 0.f);
        *(uint4*)(dZb + ((size_t)((h + a.dz_pad) * Fd + (w + a.dz_pad)) * C + ci * cc + g * 8) * 2) = o;
      }
    }
    // ---- dw[t][c] += sum_p dz[p] X[p + off(t)][c]: lanes (group, pixel slice) ----
    {
      const int g = tid % gcc;
      const int slice = tid / gcc;
      const int nslice = HT / gcc;
      float v[T][8];
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) v[t][e] = 0.f;
      for (int p = slice; p < NPTS; p += nslice) {
        const float d = s_dz[p];
        const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
#pragma unroll
        for (int t = 0; t < T; ++t) {
          const int f = (h + a.x_pad + t / KW - R) * F + (w + a.x_pad + t % KW - R);
          float xv[8];
          unpack8(*(const uint4*)(s_x + (f * cc + g * 8) * 2), xv);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[t][e] += d * xv[e];
        }
      }
      // lanes l, l+gcc, l+2gcc.. of a wave share g: fold them with shuffles first
#pragma unroll
      for (int t = 0; t < T; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = v[t][e];
          for (int o = gcc; o < 64; o <<= 1) x += __shfl_xor(x, o, 64);
          v[t][e] = x;
        }
      // the 8 waves' sums added in wave order (an LDS atomicAdd made the head's weight
      // gradient depend on wave arrival order: runs were not bit-reproducible)
      for (int w8 = 0; w8 < HT / 64; ++w8) {
        if (wave == w8 && lane < gcc) {
#pragma unroll
          for (int t = 0; t < T; ++t)
#pragma unroll
            for (int e = 0; e < 8; ++e) s_gw[t * CCH + g * 8 + e] += v[t][e];
        }
        __syncthreads();
      }
    }
    __syncthreads();
    for (int i = tid; i < T * cc; i += HT) {
      const int t = i / cc, c = i - (i / cc) * cc;
      a.gw_part[(size_t)b * T * C + t * C + ci * cc + c] = s_gw[t * CCH + c];
    }
  }
}

// Deterministic batch reduction of the head's per-board partials (plain stores: the
// step needs no gradient zeroing):
//   gw[j]    = sum_b gw_part[b][j]        (j < n = KW*KW*C)
//   gposb[p] = sum_b dzb[b][p]
//   gbias    = sum_b sum_p dzb[b][p]      (one dedicated workgroup)
// Workgroup = 64 outputs x 16 board groups (1024 threads): each thread issues all loads of
// its board group (<= 16 boards for B = 256) before summing; the 16 group sums are combined
// in LDS in a fixed order.
constexpr int HR_G = 16;
__global__ void __launch_bounds__(1024)
head_reduce_kernel(const float* __restrict__ dzb, const float* __restrict__ gw_part, int B, int n,
                   float* __restrict__ gw, float* __restrict__ gbias, float* __restrict__ gposb,
                   bf16_t* gw16, bf16_t* gbias16, bf16_t* gposb16, long long* sf) {
  // (sf: the fused update's step tag, dg_common.h — set when an output is out of range)
  // (gw16 / gbias16 / gposb16: optional bf16 twins for the data-parallel bf16 wire format)
  __shared__ float s_red[HR_G][64];
  const int nout = n + NPTS;
  const int tid = threadIdx.x;
  if ((int)blockIdx.x * 64 >= nout) {  // last workgroup: gbias
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    const int tot = B * NPTS;
    int e = tid;
    for (; e + 3072 < tot; e += 4096) {
      a0 += dzb[e];
      a1 += dzb[e + 1024];
      a2 += dzb[e + 2048];
      a3 += dzb[e + 3072];
    }
    for (; e < tot; e += 1024) a0 += dzb[e];
    const float v = wave_sum((a0 + a1) + (a2 + a3));
    if ((tid & 63) == 0) s_red[0][tid >> 6] = v;
    __syncthreads();
    if (tid == 0) {
      float t = 0.f;
      for (int w = 0; w < 16; ++w) t += s_red[0][w];
      *gbias = t;
      if (gbias16) *gbias16 = f2bf(t);
      if (sf && grad_out_of_range(t)) flag_bad_step(sf);
    }
    return;
  }
  const int o = blockIdx.x * 64 + (tid & 63);
  const int grp = tid >> 6;
  const bool is_w = o < n;
  const float* src = is_w ? gw_part + o : dzb + (o - n);
  const size_t stride = is_w ? (size_t)n : (size_t)NPTS;
  const int per = (B + HR_G - 1) / HR_G;
  const int b0 = grp * per, b1 = min(B, b0 + per);
  float acc = 0.f;
  if (o < nout) {
    int b = b0;
    for (; b + 16 <= b1; b += 16) {
      float v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = src[(size_t)(b + k) * stride];
#pragma unroll
      for (int k = 0; k < 16; ++k) acc += v[k];
    }
    for (; b < b1; ++b) acc += src[(size_t)b * stride];
  }
  s_red[grp][tid & 63] = acc;
  __syncthreads();
  if (grp == 0 && o < nout) {
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < HR_G; ++g) v += s_red[g][tid];
    if (is_w) {
      gw[o] = v;
      if (gw16) gw16[o] = f2bf(v);
    } else {
      gposb[o - n] = v;
      if (gposb16) gposb16[o - n] = f2bf(v);
    }
    if (sf && grad_out_of_range(v)) flag_bad_step(sf);
  }
}

}  // namespace

extern "C" hipError_t dg_head_reduce(const float* dzb, const float* gw_part, int B, int n,
                                     float* gw, float* gbias, float* gposb, void* gw16,
                                     void* gbias16, void* gposb16, long long* sf,
                                     hipStream_t stream) {
  const int blocks = (n + NPTS + 63) / 64 + 1;  // + the gbias workgroup
  hipLaunchKernelGGL(head_reduce_kernel, dim3(blocks), dim3(1024), 0, stream, dzb, gw_part, B, n,
                     gw, gbias, gposb, (bf16_t*)gw16, (bf16_t*)gbias16, (bf16_t*)gposb16, sf);
  return hipGetLastError();
}

template <typename K>
static void allow_lds_once(K kernel, size_t bytes) {
  static size_t done = 0;  // one per instantiation; raise when a larger frame appears
  if (bytes > done) {
    (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    done = bytes;
  }
}

extern "C" hipError_t dg_head_mfma(int C, const void* X, int B, const float* w, const float* bias,
                                   const float* posb, const int* labels, float* loss, int* pred,
                                   float* logp_out, void* dZ, float* gw_part, float* dzb,
                                   int head_relu, float grad_scale, hipStream_t stream);

extern "C" hipError_t dg_head(int kw, const void* X, int x_pad, int C, int B, const float* w,
                              const float* bias, const float* posb, const int* labels,
                              float* loss, int* pred, float* logp_out, void* dZ, int dz_pad,
                              float* gw_part, float* unused, float* dzb, int head_relu,
                              float grad_scale, hipStream_t stream) {
  if (C % 8 != 0 || B <= 0) return hipErrorInvalidValue;
  // 3x3 head over a 128/256-channel pad-1 frame: the MFMA kernel (head_mfma.hip)
  if (kw == 3 && (C == 128 || C == 256) && x_pad == 1 && (!dZ || dz_pad == 1))
    return dg_head_mfma(C, X, B, w, bias, posb, labels, loss, pred, logp_out, dZ, gw_part, dzb,
                        head_relu, grad_scale, stream);
  if (C > CCH && C % CCH != 0) return hipErrorInvalidValue;
  if (C < CCH && (64 % (C / 8)) != 0) return hipErrorInvalidValue;  // lanes per pixel
  HeadArgs a{(const char*)X, w, bias, posb, labels, loss, pred, logp_out, (char*)dZ, gw_part,
             unused, dzb, B, C, x_pad, dz_pad, head_relu, grad_scale};
  const int F = 19 + 2 * x_pad;
  const int cc = C < CCH ? C : CCH;
  const size_t lds = (size_t)((F * F * (cc / 8) + 63) / 64) * 64 * 16 +
                     (size_t)(kw * kw * C + 384 + 384 + kw * kw * CCH + HT) * 4 + HT * 4;
  switch (kw) {
    case 1:
      allow_lds_once(head_kernel<1>, lds);
      hipLaunchKernelGGL(head_kernel<1>, dim3(B), dim3(HT), lds, stream, a);
      break;
    case 3:
      allow_lds_once(head_kernel<3>, lds);
      hipLaunchKernelGGL(head_kernel<3>, dim3(B), dim3(HT), lds, stream, a);
      break;
    case 5:
      allow_lds_once(head_kernel<5>, lds);
      hipLaunchKernelGGL(head_kernel<5>, dim3(B), dim3(HT), lds, stream, a);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
