// Fused policy head: the last (c_out = 1) conv of the stack, its per-channel and untied
// per-position biases, the head ReLU, LogSoftMax over 361 points, mean ClassNLL, top-1
// argmax, and the whole backward of that block, one workgroup per board.
//
// Reference: getBasicModel's last iteration + Reshape(361) + LogSoftMax
// (experiments.lua:135-151), nn.ClassNLLCriterion (experiments.lua:45), Tensor:max(2) /
// ne / sum for accuracy (train.lua:29,36).  The reference runs these as ~8 separate
// cunn kernels; here they are a single pass over the board held on-chip.
//
// M = 1 makes MFMA pointless (GEMV-shaped), so the dot products run on the VALU with
// 16-byte vector loads; the 361 logits / probabilities stay in LDS.
#include "dg_common.h"

using namespace dg;

namespace {

constexpr int HT = 256;  // threads per board

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
  float* gw;            // grad of head weights [KW*KW*C] (atomic accumulate)
  float* gbias;         // [1] (atomic)
  float* gposb;         // [361] (atomic)
  int B;
  int C;
  int x_pad;
  int dz_pad;
  int head_relu;
  float grad_scale;     // 1 / global batch (mean NLL)
};

template <int KW>
__global__ void __launch_bounds__(HT) head_kernel(HeadArgs a) {
  constexpr int R = (KW - 1) / 2;
  constexpr int T = KW * KW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* s_w = (float*)smem;                 // [T*C]
  float* s_z = s_w + T * a.C;                // [361] pre-activation
  float* s_dz = s_z + 384;                   // [361] d loss / d z
  float* s_red = s_dz + 384;                 // [HT] scratch
  int* s_redi = (int*)(s_red + HT);          // [HT]

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int C = a.C;
  const int G = C / 8;                       // 8-channel groups
  const int F = BOARD + 2 * a.x_pad;

  for (int i = tid; i < T * C; i += HT) s_w[i] = a.w[i];
  __syncthreads();

  // ---- forward: z[p] = sum_{t,c} w[t][c] * X[p + off(t)][c] ----
  const char* Xb = a.X + (size_t)b * F * F * C * 2;
  for (int p = wave; p < NPTS; p += HT / 64) {
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    float acc = 0.f;
    for (int idx = lane; idx < T * G; idx += 64) {
      const int t = idx / G, g = idx - (idx / G) * G;
      const int hh = h + t / KW - R + a.x_pad, ww = w + t % KW - R + a.x_pad;
      const uint4 v = *(const uint4*)(Xb + ((hh * F + ww) * C + g * 8) * 2);
      const float* wt = s_w + t * C + g * 8;
      const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc += wt[2 * e] * __uint_as_float(u[e] << 16);
        acc += wt[2 * e + 1] * __uint_as_float(u[e] & 0xFFFF0000u);
      }
    }
    acc = wave_sum(acc);
    if (lane == 0) s_z[p] = acc + a.bias[0] + a.posb[p];
  }
  __syncthreads();

  // ---- log-softmax over 361 logits (logit = relu(z) if head_relu) ----
  float m = -INFINITY;
  int am = 0;
  for (int p = tid; p < NPTS; p += HT) {
    const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
    if (l > m) { m = l; am = p; }
  }
  s_red[tid] = m;
  s_redi[tid] = am;
  __syncthreads();
  for (int s = HT / 2; s > 0; s >>= 1) {
    if (tid < s) {
      const float o = s_red[tid + s];
      const int oi = s_redi[tid + s];
      if (o > s_red[tid] || (o == s_red[tid] && oi < s_redi[tid])) {
        s_red[tid] = o;
        s_redi[tid] = oi;
      }
    }
    __syncthreads();
  }
  const float mx = s_red[0];
  const int amax = s_redi[0];
  __syncthreads();
  float se = 0.f;
  for (int p = tid; p < NPTS; p += HT) {
    const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
    se += __expf(l - mx);
  }
  s_red[tid] = se;
  __syncthreads();
  for (int s = HT / 2; s > 0; s >>= 1) {
    if (tid < s) s_red[tid] += s_red[tid + s];
    __syncthreads();
  }
  const float lse = mx + __logf(s_red[0]);
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

  // ---- backward: dlogit = (softmax - onehot) * scale ; dz = dlogit * relu'(z) ----
  float dsum = 0.f;
  for (int p = tid; p < NPTS; p += HT) {
    const float z = s_z[p];
    const float l = a.head_relu ? fmaxf(z, 0.f) : z;
    float d = __expf(l - lse) - (p == y ? 1.f : 0.f);
    d *= a.grad_scale;
    if (a.head_relu && !(z > 0.f)) d = 0.f;
    s_dz[p] = d;
    dsum += d;
    atomicAdd(a.gposb + p, d);
  }
  dsum = wave_sum(dsum);
  if (lane == 0) atomicAdd(a.gbias, dsum);
  __syncthreads();

  // ---- dX[q][c] = sum_t w[t][c] * dz[q - off(t)], masked by X[q][c] > 0 ----
  char* dZb = a.dZ + (size_t)b * (BOARD + 2 * a.dz_pad) * (BOARD + 2 * a.dz_pad) * C * 2;
  const int Fd = BOARD + 2 * a.dz_pad;
  for (int idx = tid; idx < NPTS * G; idx += HT) {
    const int q = idx / G, g = idx - (idx / G) * G;
    const int h = q / BOARD, w = q - (q / BOARD) * BOARD;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const int ph = h - (t / KW - R), pw = w - (t % KW - R);
      if (ph < 0 || ph >= BOARD || pw < 0 || pw >= BOARD) continue;
      const float d = s_dz[ph * BOARD + pw];
      const float* wt = s_w + t * C + g * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] += d * wt[e];
    }
    const uint4 xm = *(const uint4*)(Xb + (((h + a.x_pad) * F + (w + a.x_pad)) * C + g * 8) * 2);
    const uint32_t u[4] = {xm.x, xm.y, xm.z, xm.w};
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = __uint_as_float(u[e] << 16) > 0.f ? v[2 * e] : 0.f;
      const float hi = __uint_as_float(u[e] & 0xFFFF0000u) > 0.f ? v[2 * e + 1] : 0.f;
      o[e] = pack_bf16x2(lo, hi);
    }
    *(uint4*)(dZb + (((h + a.dz_pad) * Fd + (w + a.dz_pad)) * C + g * 8) * 2) =
        uint4{o[0], o[1], o[2], o[3]};
  }

  // ---- dw[t][c] += sum_p dz[p] * X[p + off(t)][c] ----
  for (int idx = tid; idx < T * G; idx += HT) {
    const int t = idx / G, g = idx - (idx / G) * G;
    const int dh = t / KW - R, dw = t % KW - R;
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < NPTS; ++p) {
      const float d = s_dz[p];
      if (d == 0.f) continue;
      const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
      const uint4 xv = *(const uint4*)(Xb + (((h + dh + a.x_pad) * F + (w + dw + a.x_pad)) * C + g * 8) * 2);
      const uint32_t u[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] += d * __uint_as_float(u[e] << 16);
        v[2 * e + 1] += d * __uint_as_float(u[e] & 0xFFFF0000u);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) atomicAdd(a.gw + t * C + g * 8 + e, v[e]);
  }
}

}  // namespace

extern "C" hipError_t dg_head(int kw, const void* X, int x_pad, int C, int B, const float* w,
                              const float* bias, const float* posb, const int* labels,
                              float* loss, int* pred, float* logp_out, void* dZ, int dz_pad,
                              float* gw, float* gbias, float* gposb, int head_relu,
                              float grad_scale, hipStream_t stream) {
  if (C % 8 != 0 || B <= 0) return hipErrorInvalidValue;
  HeadArgs a{(const char*)X, w, bias, posb, labels, loss, pred, logp_out, (char*)dZ, gw, gbias,
             gposb, B, C, x_pad, dz_pad, head_relu, grad_scale};
  const size_t lds = (size_t)(kw * kw * C + 384 + 384 + HT) * 4 + HT * 4;
  switch (kw) {
    case 1: hipLaunchKernelGGL(head_kernel<1>, dim3(B), dim3(HT), lds, stream, a); break;
    case 3: hipLaunchKernelGGL(head_kernel<3>, dim3(B), dim3(HT), lds, stream, a); break;
    case 5: hipLaunchKernelGGL(head_kernel<5>, dim3(B), dim3(HT), lds, stream, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
