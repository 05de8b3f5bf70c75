// Policy head on the matrix cores: the c_out = 1 3x3 conv over 128 channels, biases, head
// ReLU, LogSoftMax / NLL / argmax, and the whole backward of the block (input gradient with
// the ReLU gate of the layer below, per-board weight-gradient partials, dz for the bias
// reduce) — one workgroup (8 waves) per board, every GEMM-shaped part on
// v_mfma_f32_16x16x32_bf16:
//
//   forward  z[p]      = sum_{t,c} w[t][c] X[p + off t][c]   M = 16 (row 0 = w), N = 384 px,
//                                                           K = 1152 (B from the LDS image)
//   weights  dW[t][c]  = sum_f dz[f - off t] X[f][c]         M = 16 (9 taps), N = 128 ch,
//                                                           K = 448 frame rows (B: transposing
//                                                           ds_read_b64_tr_b16 of the image)
//   input    dX[c][q]  = sum_t w[t][c] dz[q - off t]         M = 128 ch, N = 384 px, K = 32
//                                                           (9 taps), gated by X[q][c] > 0
//
// dz and (for dX) the fp32 master weights enter as hi + lo bf16 pairs (x = hi + lo, each
// product term summed in fp32), which keeps the backward at ~16 significant bits — the
// VALU version (head.hip) used fp32 FMAs there.  The board's 21x21x128 activation frame
// is staged once into LDS by LDS-DMA with the conv_stack image layout (two 64-channel
// images, 128-B rows, 16-B slot g ^ ((x + 3y) & 7)).
//
// Replaces head.hip's VALU dot/FMA loops for the 3x3 / 128-channel head (58 -> see
// profiles/).  Reference: getBasicModel's last layer + Reshape + LogSoftMax
// (experiments.lua:135-151), ClassNLLCriterion (:45), max/ne/sum accuracy (train.lua:29,36).
#include "head_body.h"

using namespace dg;
using namespace dghead;

namespace {

// C = 128: the board's two 64-channel images are resident for the whole kernel.
// C = 256: the image pair holds one 128-channel half at a time — forward over half 0 then
// half 1 (z accumulates in registers), the backward on half 1 (still resident), then half 0
// re-staged: 3 image loads instead of 2, all GEMMs unchanged.
template <int C>
__global__ void __launch_bounds__(HT) head_mfma_kernel(HeadMArgs a) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  head_from_frame<C>(a, blockIdx.x, smem);
}

}  // namespace

template <int C>
static hipError_t launch(int B, const HeadMArgs& a, hipStream_t stream) {
  constexpr size_t lds = frame_head_lds(C);
  static_assert(lds <= 160 * 1024, "LDS");
  static bool done = false;
  if (!done) {
    (void)hipFuncSetAttribute((const void*)head_mfma_kernel<C>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    done = true;
  }
  hipLaunchKernelGGL(head_mfma_kernel<C>, dim3(B), dim3(HT), lds, stream, a);
  return hipGetLastError();
}

// 3x3 head over a 128- or 256-channel pad-1 frame (the 12-layer configs); see dg_head.
extern "C" hipError_t dg_head_mfma(int C, const void* X, int B, const float* w, const float* bias,
                                   const float* posb, const int* labels, float* loss, int* pred,
                                   float* logp_out, void* dZ, float* gw_part, float* dzb,
                                   int head_relu, float grad_scale, hipStream_t stream) {
  if (B <= 0) return hipErrorInvalidValue;
  HeadMArgs a{(const char*)X, w, bias, posb, labels, loss, pred, logp_out, (char*)dZ, gw_part,
              dzb, head_relu, grad_scale};
  return C == 256 ? launch<256>(B, a, stream) : launch<128>(B, a, stream);
}
