// Policy-head device body shared by head_mfma.hip (standalone kernel) and conv_stack.hip
// (fused after the forward stack's last layer, on the board image already in LDS).
// See head_mfma.hip for the algorithm.  Requires 512 threads (8 waves) and the conv_stack
// image layout (two 64-channel images of HROWS 128-B rows, slot g ^ ((x + 3y) & 7)).
#pragma once
#include <math.h>

#include "dg_common.h"

namespace dghead {

using namespace dg;

constexpr int F = 21;
constexpr int FF = F * F;          // 441
constexpr int HROWS = 448;
constexpr int HB = HROWS * 128;    // one 64-channel image
constexpr int T = 9;
constexpr int DZM = 32;            // margin of the frame-shaped dz array (taps reach +-22)
constexpr int DZN = DZM + HROWS + DZM;
constexpr int HT = 512;

struct HeadMArgs {
  const char* X;        // last hidden activation frame [B][21][21][128] bf16
  const float* w;       // head weights OHWI [1][3][3][128] fp32 (master)
  const float* bias;    // [1]
  const float* posb;    // [361]
  const int* labels;    // [B] or null
  float* loss;          // [B]
  int* pred;            // [B]
  float* logp_out;      // [B][361] or null
  char* dZ;             // gradient frame [B][21][21][128] bf16 (null = eval only)
  float* gw_part;       // [B][9*128]
  float* dzb;           // [B][361]
  int head_relu;
  float grad_scale;
};

DG_DEV int fsig(int f) { return ((f % F) + 3 * (f / F)) & 7; }
DG_DEV int toff_of(int t) { return (t / 3 - 1) * F + (t % 3 - 1); }

// x -> (hi, lo) bf16 pair, x ~= hi + lo
DG_DEV void split_bf(float x, uint16_t& hi, uint16_t& lo) {
  hi = f2bf(x);
  lo = f2bf(x - bf2f(hi));
}
DG_DEV bf16x8 pack8(const uint16_t* v) {
  s16x8 s;
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = (short)v[e];
  return __builtin_bit_cast(bf16x8, s);
}

// scratch: T*C*6 + 384*4 + DZN*4 + 32*4 bytes of LDS (16-B aligned)
constexpr size_t scratch_bytes(int C) { return (size_t)T * C * 6 + 384 * 4 + DZN * 4 + 32 * 4; }

// The head for board b: weights into scratch, forward z, log-softmax / NLL / argmax, and the
// backward (per-board weight-gradient partials, dz, input gradient into a.dZ).  The caller
// has staged channel half 0 of the board image into sX (and synchronised or not: a barrier
// follows the weight staging here); stage(hf) re-stages half hf (C = 256 only).
template <int C, typename StageFn>
DG_DEV void head_body(const HeadMArgs& a, int b, char* sX, char* scratch, StageFn&& stage) {
  static_assert(C == 128 || C == 256, "channels");
  constexpr int NH = C / 128;
  uint16_t* s_wb = (uint16_t*)scratch;                  // [T*C] bf16 weights
  float* s_w = (float*)(s_wb + T * C);                  // [T*C] fp32 weights
  float* s_z = s_w + T * C;                             // [384]
  float* s_dzf = s_z + 384;                             // [DZN] frame-shaped dz
  float* s_red = s_dzf + DZN;                           // [16]
  int* s_redi = (int*)(s_red + 16);                     // [16]
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int lr = lane & 15;
  const int lq = lane >> 4;
  for (int i = tid; i < T * C; i += HT) {
    const float v = a.w[i];
    s_w[i] = v;
    s_wb[i] = f2bf(v);
  }
  for (int i = tid; i < 384; i += HT) s_z[i] = 0.f;
  for (int i = tid; i < DZN; i += HT) s_dzf[i] = 0.f;
  __syncthreads();

  // pixels of this wave: 3 fragments of 16 (N = 384 >= 361)
  int fp[3], fs[3], pp3[3];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    int p = wave * 48 + jj * 16 + lr;
    pp3[jj] = p;
    if (p >= NPTS) p = 0;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    fp[jj] = (h + 1) * F + (w + 1);
    fs[jj] = (w + 1) + 3 * (h + 1);
  }

  // ---- forward: z = w . im2col(X) ----
  {
    f32x4 acc[3];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) acc[jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < 2 * T * NH; ++s) {
      const int hs = s / (2 * T), s2 = s - hs * (2 * T);
      if (NH > 1 && s2 == 0 && hs > 0) {
        __syncthreads();  // every wave is past its reads of half hs-1
        stage(hs);
        __syncthreads();
      }
      const int c = s2 / T, t = s2 - (s2 / T) * T;
      const char* sXc = sX + c * HB;
      const int toff = toff_of(t);
      const int tsig = (t % 3 - 1) + 3 * (t / 3 - 1);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int g = kk * 4 + lq;
        bf16x8 af = bf16x8{};
        if (lr == 0)  // A row 0 = the weights, rows 1..15 zero
          af = *(const bf16x8*)(s_wb + t * C + hs * 128 + c * 64 + g * 8);
#pragma unroll
        for (int jj = 0; jj < 3; ++jj) {
          const int row = fp[jj] + toff;
          const bf16x8 bfr = lds_read_b128(
              (const LDS_AS char*)(sXc + row * 128 + ((g ^ ((fs[jj] + tsig) & 7)) * 16)));
          acc[jj] = mfma16(af, bfr, acc[jj]);
        }
      }
    }
    // D row 0 (lanes lq == 0, element 0) = z of pixel lr
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
      if (lq == 0 && pp3[jj] < NPTS) s_z[pp3[jj]] = acc[jj][0] + a.bias[0] + a.posb[pp3[jj]];
  }
  __syncthreads();

  // ---- log-softmax over 361 logits (logit = relu(z) if head_relu), argmax, NLL ----
  float m = -INFINITY;
  int am = 0;
  for (int p = tid; p < NPTS; p += HT) {
    const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
    if (l > m) { m = l; am = p; }
  }
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
  __syncthreads();
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
  if (a.logp_out)
    for (int p = tid; p < NPTS; p += HT) {
      const float l = a.head_relu ? fmaxf(s_z[p], 0.f) : s_z[p];
      a.logp_out[(size_t)b * NPTS + p] = l - lse;
    }
  if (a.dZ == nullptr) return;

  // ---- dz = (softmax - onehot) * scale * relu'(z), frame-shaped in LDS ----
  for (int p = tid; p < NPTS; p += HT) {
    const float z = s_z[p];
    const float l = a.head_relu ? fmaxf(z, 0.f) : z;
    float d = (__expf(l - lse) - (p == y ? 1.f : 0.f)) * a.grad_scale;
    if (a.head_relu && !(z > 0.f)) d = 0.f;
    a.dzb[(size_t)b * NPTS + p] = d;
    const int h = p / BOARD, w = p - (p / BOARD) * BOARD;
    s_dzf[DZM + (h + 1) * F + (w + 1)] = d;
  }
  __syncthreads();

  for (int hb = NH - 1; hb >= 0; --hb) {
  if (hb != NH - 1) {
    __syncthreads();  // every wave is past its reads of the resident half
    stage(hb);
    __syncthreads();
  }
  // ---- weight-gradient partial: dW[t][c] = sum_f dz[f - off t] X[f][c] ----
  {
    const int ch0 = wave * 16;                  // this wave's 16 channels (N fragment)
    const int img = ch0 / 64, cw = ch0 % 64;
    const char* sXi = sX + img * HB;
    const int li = lane & 15, q = li >> 2, pq = li & 3;
    const int toffA = lr < T ? toff_of(lr) : 0;
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int ks = 0; ks < HROWS / 32; ++ks) {
      // A (taps x rows): row t = lr, k = f = ks*32 + lq*8 + e
      uint16_t ah[8], al[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int f = ks * 32 + lq * 8 + e;
        const float v = lr < T ? s_dzf[DZM + f - toffA] : 0.f;
        split_bf(v, ah[e], al[e]);
      }
      // B (rows x channels): transposing reads, lane supplies row (8 lq + 4 half + q),
      // channels cw + 4 pq .. +3
      s16x4 tb[2];
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int row = ks * 32 + 8 * lq + 4 * half + q;
        const int slot = (cw + 4 * pq) / 8;
        tb[half] = lds_read_tr((const LDS_AS char*)(sXi + row * 128 +
                                                   ((slot ^ fsig(row)) * 16) + (pq & 1) * 8));
      }
      const s16x8 bv = {tb[0][0], tb[0][1], tb[0][2], tb[0][3],
                        tb[1][0], tb[1][1], tb[1][2], tb[1][3]};
      const bf16x8 bfr = __builtin_bit_cast(bf16x8, bv);
      acc = mfma16(pack8(ah), bfr, acc);
      acc = mfma16(pack8(al), bfr, acc);
    }
    // D rows = taps (lq*4 + r), column = channel ch0 + lr
    float* gp = a.gw_part + (size_t)b * T * C;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int t = lq * 4 + r;
      if (t < T) gp[t * C + hb * 128 + ch0 + lr] = acc[r];
    }
  }

  // ---- input gradient: dX[c][q] = sum_t w[t][c] dz[q - off t], gated by X[q][c] > 0 ----
  {
    // B fragments (taps x pixels) of this wave's 3 pixel fragments, hi + lo
    bf16x8 bh[3], bl[3];
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      uint16_t vh[8], vl[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int t = lq * 8 + e;
        const float v = t < T ? s_dzf[DZM + fp[jj] - toff_of(t)] : 0.f;
        split_bf(v, vh[e], vl[e]);
      }
      bh[jj] = pack8(vh);
      bl[jj] = pack8(vl);
    }
    char* dZb = a.dZ + (size_t)b * FF * C * 2;
    for (int mi = 0; mi < 8; ++mi) {
      // A fragment (channels x taps): row c = mi*16 + lr, k = taps lq*8 + e
      uint16_t wh[8], wl[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int t = lq * 8 + e;
        const float v = t < T ? s_w[t * C + hb * 128 + mi * 16 + lr] : 0.f;
        split_bf(v, wh[e], wl[e]);
      }
      const bf16x8 ah = pack8(wh), al = pack8(wl);
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
        acc = mfma16(ah, bh[jj], acc);
        acc = mfma16(ah, bl[jj], acc);
        acc = mfma16(al, bh[jj], acc);
        if (pp3[jj] >= NPTS) continue;
        // lane: channels c .. c+3 (rows lq*4 + r of the fragment) of pixel fp[jj]
        const int c = mi * 16 + lq * 4;  // channel within the resident half
        const int ci = c & 63;
        const uint2 xm = *(const uint2*)(sX + (c / 64) * HB + fp[jj] * 128 +
                                         (((ci >> 3) ^ (fs[jj] & 7)) * 16) + (ci & 4) * 2);
        auto pos = [](uint32_t h16) { return h16 != 0u && !(h16 & 0x8000u); };
        const float v0 = pos(xm.x & 0xFFFFu) ? acc[0] : 0.f;
        const float v1 = pos(xm.x >> 16) ? acc[1] : 0.f;
        const float v2 = pos(xm.y & 0xFFFFu) ? acc[2] : 0.f;
        const float v3 = pos(xm.y >> 16) ? acc[3] : 0.f;
        uint2 o;
        o.x = pack_bf16x2(v0, v1);
        o.y = pack_bf16x2(v2, v3);
        *(uint2*)(dZb + ((size_t)fp[jj] * C + hb * 128 + c) * 2) = o;
      }
    }
  }
  }  // halves
}

// The head for board b on the activation frame a.X in global memory (the standalone
// head_mfma kernel, and the forward launches at d = 256 that run it after their last layer:
// conv_layer2_multi / conv_stack_f8, whose 256-channel image does not stay in LDS): channel
// half hf staged by LDS-DMA into the two-image layout at smem, scratch after it (2 HB +
// scratch_bytes(C) of LDS).  The caller has retired its own stores to a.X (vmcnt(0)) and
// synchronised the workgroup.
template <int C>
DG_DEV void head_from_frame(const HeadMArgs& a, int b, char* smem) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const char* Xb = a.X + (size_t)b * FF * C * 2;
  auto stage = [&](int hf) {
    for (int j = wave; j < 2 * (HROWS / 8); j += HT / 64) {
      const int c = j / (HROWS / 8), jj = j - c * (HROWS / 8);
      const int rl = jj * 8 + (lane >> 3);
      const int r = rl < FF ? rl : FF - 1;  // rows 441.. duplicate the (zero) border row 440
      const int g = (lane & 7) ^ fsig(rl);
      glds16(Xb + ((size_t)r * C + hf * 128 + c * 64 + g * 8) * 2,
             (LDS_AS void*)(smem + c * HB + jj * 1024));
    }
  };
  stage(0);
  head_body<C>(a, b, smem, smem + 2 * HB, stage);
}
constexpr size_t frame_head_lds(int C) { return 2 * (size_t)HB + scratch_bytes(C); }

}  // namespace dghead
