// pybind11 bindings for the deep_go_amd HIP kernels (module `_dghip`).
//
// Tensors cross the boundary as raw device addresses (tensor.data_ptr()) and the HIP
// stream as its handle (torch.cuda.current_stream().cuda_stream): the Python layer
// (deep_go_amd/ops) owns allocation, shape checks and stream choice, and every launcher
// here validates the shape invariants it relies on before touching the GPU.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace py = pybind11;

extern "C" {
hipError_t dg_comm_proxy(void* buf, long long nbytes, int world, double gbps, int blocks,
                         hipStream_t s);
hipError_t dg_conv_nt_ex(int epi, int kw, int bm, int bn, const void* A, int KP, int M,
                         int Mpad, const void* X, int x_pad, int x_C, int Npix, void* Y,
                         int y_pad, const float* bias, const float* posb, const void* aux,
                         int aux_pad, void* mask, hipStream_t stream);
hipError_t dg_conv_nt(int epi, int kw, int bm, int bn, const void* A, int KP, int M, int Mpad,
                      const void* X, int x_pad, int x_C, int Npix, void* Y, int y_pad,
                      const float* bias, const float* posb, const void* aux, int aux_pad,
                      hipStream_t stream);
hipError_t dg_conv_board(int epi, int kw, int bm, const void* A, int KP, int M, int Mpad,
                         const void* X, int x_pad, int x_C, int B, void* Y, int y_pad,
                         const float* bias, const float* posb, const void* aux, int aux_pad,
                         hipStream_t stream);
void dg_conv_board_set_ablate(int mode);
void dg_conv_stack2_set_mode(int on);
void dg_conv_stack2_set_sched(int stag, int prio, int delay);
void dg_conv_stack_f8_set_mode(int m);
void dg_conv_stack_f8_set_sched(int stag, int delay);
void dg_conv_stack_f8_set_debug(unsigned long long* dbg);
hipError_t dg_conv_stack_f8(int C, int epi, const long long* table, int nl, const void* X0,
                            const float* s_x0, unsigned* amax_x0, int B, const long long* y8,
                            const long long* sr_step, hipStream_t stream);
hipError_t dg_conv_wgrad_win8(const long long* table, int nl, int M, int Mpad, int Cx, int B,
                              int KP, int splits, long long* sf, hipStream_t stream);
int dg_conv_wgrad_win8_splits(int nl, int M, int Cx, int B, int num_cus);
void dg_conv_wgrad_win8_set_ablate(int mode);
hipError_t dg_conv_stack_f8_fwd_head(int C, const long long* table, int nl, const void* X0,
                                     const float* s_x0, unsigned* amax_x0, int B, const float* w,
                                     const float* bias, const float* posb, const int* labels,
                                     float* loss, int* pred, void* dZ, float* gw_part,
                                     float* dzb, int head_relu, float grad_scale,
                                     const long long* y8, hipStream_t stream);
hipError_t dg_conv_stack2(int epi, const long long* table, int nl, const void* X0, int l1, int B,
                          hipStream_t stream);
hipError_t dg_conv_stack2_fwd_head(const long long* table, int nl, const void* X0, int l1, int B,
                                   const float* w, const float* bias, const float* posb,
                                   const int* labels, float* loss, int* pred, void* dZ,
                                   float* gw_part, float* dzb, int head_relu, float grad_scale,
                                   hipStream_t stream);
hipError_t dg_conv_stack2_fwd_head_x(const long long* table, int nl, void* X0, int B,
                                     const void* planes, const void* player, const void* rank,
                                     const float* w, const float* bias, const float* posb,
                                     const int* labels, float* loss, int* pred, void* dZ,
                                     float* gw_part, float* dzb, int head_relu, float grad_scale,
                                     hipStream_t stream);
hipError_t dg_conv_board_ex(int epi, int kw, int bm, const void* A, int KP, int M, int Mpad,
                            const void* X, int x_pad, int x_C, int B, void* Y, int y_pad,
                            const float* bias, const float* posb, const void* pbias,
                            const void* aux, int aux_pad, void* mask, hipStream_t stream);
void dg_conv_wgrad_set_ablate(int mode);
void dg_conv_wgrad5_set_ns(int ns);
int dg_conv_wgrad_wgs_per_cu();
int dg_conv_wgrad_ktile(int KP);
int dg_conv_wgrad_wgs_per_cu_for(int KP);
hipError_t dg_conv_wgrad_multi(int kw, const long long* table, int nl, int dz_pad, int M,
                               int Mpad, int x_pad, int x_C, int B, int KP, int splits,
                               hipStream_t stream);
int dg_conv_l1_ok(int kw, int x_pad, int x_C, int Mpad, int KP);
int dg_conv_l1_frag_ok(int kw, int x_pad, int x_C, int M, int y_pad);
hipError_t dg_conv_l1_frag(const void* A, const void* pbias, void* X, int B, int M,
                           void* Y, void* mask, const void* planes, const void* player,
                           const void* rank, hipStream_t stream);
hipError_t dg_conv_l1(int kw, const void* A, int KP, int M, int Mpad, const void* X, int x_pad,
                      int x_C, int B, void* Y, int y_pad, const float* bias, const float* posb,
                      void* mask, const void* pbias, hipStream_t stream);
void dg_conv_wgrad_win_set_ablate(int mode);
int dg_conv_wgrad_win_splits(int nl, int M, int Cx, int B, int num_cus);
hipError_t dg_conv_layer2(int epi, const void* A, const void* pbias, const void* X, void* Y,
                          void* mask, int C, int B, hipStream_t stream);
hipError_t dg_conv_layer2_multi_head(const long long* table, int nl, int B, const float* w,
                                     const float* bias, const float* posb, const int* labels,
                                     float* loss, int* pred, void* dZ, float* gw_part,
                                     float* dzb, int head_relu, float grad_scale,
                                     hipStream_t stream);
hipError_t dg_conv_layer2_multi(int epi, const long long* table, int nl, int C, int B,
                                hipStream_t stream);
hipError_t dg_conv_wgrad_win(const long long* table, int nl, int M, int Mpad, int Cx, int B,
                             int KP, int splits, long long* sf, hipStream_t stream);
hipError_t dg_conv_board_fp8(int kw, int bm, const void* A8, int KP, int M, int Mpad,
                             const void* X8, int x_pad, int x_C, int B, void* Y, void* Y8,
                             int y_pad, const float* bias, const float* posb, const float* s_x,
                             const float* s_w, const float* s_y, unsigned* amax_y, void* mask,
                             hipStream_t stream);
hipError_t dg_fp8_update_scales(int n, float* scales, unsigned* amax_w, int nparts_w, unsigned* amax_y, float w_margin,
                               float g_headroom, int* sat, float* gscales, unsigned* gamax,
                               float* ghist, hipStream_t s);
hipError_t dg_weight_fp8(const float* w, void* wf8, int cout, int cin, int taps, int cinp, int kp,
                         const float* s_w, hipStream_t s);
hipError_t dg_frame_to_fp8(const void* src, void* dst, size_t n, const float* scale,
                           unsigned* amax, hipStream_t s);
hipError_t dg_conv_wgrad(int kw, const void* dZ, int dz_pad, int M, int Mpad, const void* X,
                         int x_pad, int x_C, int B, int KP, int splits, float* slab,
                         hipStream_t stream);
hipError_t dg_wgrad_reduce_multi(const long long* table, int nl, int cols, hipStream_t stream);
hipError_t dg_bias_grad_partial_multi(const long long* table, int nl, int B, int C, int pad,
                                      long long* sf, hipStream_t s);
hipError_t dg_wgrad_reduce(const float* slab, float* out, int splits, int M, int Mpad, int KP,
                           int taps, int cin, int cinp, const float* bpart, int bchunks,
                           float* gposb, float* gbias, void* out16, void* gposb16,
                           void* gbias16, long long* sf, hipStream_t stream);
hipError_t dg_head_reduce(const float* dzb, const float* gw_part, int B, int n, float* gw,
                          float* gbias, float* gposb, void* gw16, void* gbias16, void* gposb16,
                          long long* sf, hipStream_t stream);
hipError_t dg_head(int kw, const void* X, int x_pad, int C, int B, const float* w,
                   const float* bias, const float* posb, const int* labels, float* loss,
                   int* pred, float* logp_out, void* dZ, int dz_pad, float* gw_part,
                   float* unused, float* dzb, int head_relu, float grad_scale,
                   hipStream_t stream);
hipError_t dg_expand_features(const uint8_t* planes, const uint8_t* player, const uint8_t* rank,
                              void* out, int B, int pad, int CP, void* out2, int CP2,
                              hipStream_t s);
hipError_t dg_bias_grad_partial(const void* dZ, int B, int C, int pad, float* part,
                                hipStream_t s);
int dg_bias_chunks(int B);
int dg_bias_chunks_multi(int B);
hipError_t dg_sgd(float* p, const float* g, size_t n, const double* lr, float gscale,
                  const float* gate, const void* g16, hipStream_t s);
hipError_t dg_rmsprop(float* p, const float* g, float* ms, size_t n, const double* lr,
                      float decay, float gscale, const float* gate, const void* g16,
                      hipStream_t s);
hipError_t dg_finite_gate(const float* loss, int n, const float* grads, size_t ng, float* gate,
                          int* bad_count, const void* grads16, hipStream_t s);
hipError_t dg_lr_decay(double* lr, double decay, long long* step, hipStream_t s);
hipError_t dg_finite_gate1(const float* loss, int n, const float* grads, const void* grads16,
                           size_t ng, float* gate, int* bad_count, unsigned* ticket,
                           hipStream_t s);
hipError_t dg_weight_refresh(const long long* table, int n, double* lr, double decay,
                             long long* step, hipStream_t s);
int dg_grad_update_tickets();
int dg_grad_update_cols();
hipError_t dg_grad_update(const long long* table, int n, long long plain_off, long long plain_n,
                          float* P, float* G, const void* G16, float* MS, float rms_decay,
                          float gscale, const float* gate, double* lr, double decay,
                          long long* step, unsigned* tickets, int* bad_steps, int write_grads, int final,
                          const long long* gflag, hipStream_t s);
}

namespace {

template <typename T>
T* P(uintptr_t v) {
  return reinterpret_cast<T*>(v);
}
hipStream_t S(uintptr_t v) { return reinterpret_cast<hipStream_t>(v); }

void check(hipError_t e, const char* what) {
  if (e != hipSuccess)
    throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

PYBIND11_MODULE(_dghip, m) {
  m.doc() = "deep_go_amd CDNA4 (gfx950) HIP kernels";
  m.attr("EPI_LINEAR") = 0;
  m.attr("EPI_FWD") = 1;
  m.attr("EPI_DGRAD") = 2;

  m.def("conv_nt",
        [](int epi, int kw, int bm, int bn, uintptr_t A, int KP, int M, int Mpad, uintptr_t X,
           int x_pad, int x_C, int Npix, uintptr_t Y, int y_pad, uintptr_t bias, uintptr_t posb,
           uintptr_t aux, int aux_pad, uintptr_t stream) {
          check(dg_conv_nt(epi, kw, bm, bn, P<void>(A), KP, M, Mpad, P<void>(X), x_pad, x_C,
                           Npix, P<void>(Y), y_pad, P<float>(bias), P<float>(posb), P<void>(aux),
                           aux_pad, S(stream)),
                "conv_nt");
        });
  m.def("conv_board",
        [](int epi, int kw, int bm, uintptr_t A, int KP, int M, int Mpad, uintptr_t X, int x_pad,
           int x_C, int B, uintptr_t Y, int y_pad, uintptr_t bias, uintptr_t posb, uintptr_t aux,
           int aux_pad, uintptr_t stream) {
          check(dg_conv_board(epi, kw, bm, P<void>(A), KP, M, Mpad, P<void>(X), x_pad, x_C, B,
                              P<void>(Y), y_pad, P<float>(bias), P<float>(posb), P<void>(aux),
                              aux_pad, S(stream)),
                "conv_board");
        });
  m.def("conv_nt_ex",
        [](int epi, int kw, int bm, int bn, uintptr_t A, int KP, int M, int Mpad, uintptr_t X,
           int x_pad, int x_C, int Npix, uintptr_t Y, int y_pad, uintptr_t bias, uintptr_t posb,
           uintptr_t aux, int aux_pad, uintptr_t mask, uintptr_t stream) {
          check(dg_conv_nt_ex(epi, kw, bm, bn, P<void>(A), KP, M, Mpad, P<void>(X), x_pad, x_C,
                              Npix, P<void>(Y), y_pad, P<float>(bias), P<float>(posb),
                              P<void>(aux), aux_pad, P<void>(mask), S(stream)),
                "conv_nt_ex");
        },
        "conv_nt + optional ReLU bitmask output (EPI_FWD)");
  m.def("conv_board_ex",
        [](int epi, int kw, int bm, uintptr_t A, int KP, int M, int Mpad, uintptr_t X, int x_pad,
           int x_C, int B, uintptr_t Y, int y_pad, uintptr_t bias, uintptr_t posb,
           uintptr_t pbias, uintptr_t aux, int aux_pad, uintptr_t mask, uintptr_t stream) {
          check(dg_conv_board_ex(epi, kw, bm, P<void>(A), KP, M, Mpad, P<void>(X), x_pad, x_C,
                                 B, P<void>(Y), y_pad, P<float>(bias), P<float>(posb),
                                 P<void>(pbias), P<void>(aux), aux_pad, P<void>(mask),
                                 S(stream)),
                "conv_board_ex");
        },
        "conv_board + optional bf16 bias table (fwd) and ReLU bitmask (fwd writes, dgrad reads)");
  // conv_stack2.hip: weights streamed into VGPRs (fragment-ordered), no per-K-step barrier.
  // l1 = 1: table row 0 is the network's first layer (5x5 over the 23x23x40 input frame X0)
  m.def("conv_stack2_fwd", [](uintptr_t table, int nl, uintptr_t X0, int l1, int B,
                              uintptr_t stream) {
    check(dg_conv_stack2(1, P<long long>(table), nl, P<void>(X0), l1, B, S(stream)),
          "conv_stack2_fwd");
  }, "conv_stack2 forward: table rows {A_frag, pbias_frag, Y, mask}; l1: row 0 = first layer");
  m.def("conv_stack2_fwd_head", [](uintptr_t table, int nl, uintptr_t X0, int l1, int B,
                                   uintptr_t w, uintptr_t bias, uintptr_t posb, uintptr_t labels,
                                   uintptr_t loss, uintptr_t pred, uintptr_t dZ, uintptr_t gw_part,
                                   uintptr_t dzb, int head_relu, float grad_scale,
                                   uintptr_t stream) {
    check(dg_conv_stack2_fwd_head(P<long long>(table), nl, P<void>(X0), l1, B, P<float>(w),
                                  P<float>(bias), P<float>(posb), P<int>(labels), P<float>(loss),
                                  P<int>(pred), P<void>(dZ), P<float>(gw_part), P<float>(dzb),
                                  head_relu, grad_scale, S(stream)),
          "conv_stack2_fwd_head");
  }, "conv_stack2 forward + the fused 3x3/128 policy head");
  m.def("conv_stack2_fwd_head_x", [](uintptr_t table, int nl, uintptr_t X0, int B,
                                     uintptr_t planes, uintptr_t player, uintptr_t rank,
                                     uintptr_t w, uintptr_t bias, uintptr_t posb, uintptr_t labels,
                                     uintptr_t loss, uintptr_t pred, uintptr_t dZ,
                                     uintptr_t gw_part, uintptr_t dzb, int head_relu,
                                     float grad_scale, uintptr_t stream) {
    check(dg_conv_stack2_fwd_head_x(P<long long>(table), nl, P<void>(X0), B, P<void>(planes),
                                    P<void>(player), P<void>(rank), P<float>(w), P<float>(bias),
                                    P<float>(posb), P<int>(labels), P<float>(loss), P<int>(pred),
                                    P<void>(dZ), P<float>(gw_part), P<float>(dzb), head_relu,
                                    grad_scale, S(stream)),
          "conv_stack2_fwd_head_x");
  }, "conv_stack2 forward (l1) with the feature expansion fused into its prologue + the head");
  // conv_stack_f8.hip: the fp8 (e4m3, MX MFMA) forward stack of the hidden 128 -> 128 layers
  m.def("conv_stack_f8", [](int C, int epi, uintptr_t table, int nl, uintptr_t X0,
                            uintptr_t s_x0, uintptr_t amax_x0, int B, uintptr_t stream) {
    check(dg_conv_stack_f8(C, epi, P<long long>(table), nl, P<void>(X0), P<float>(s_x0),
                           P<unsigned>(amax_x0), B, nullptr, nullptr, S(stream)),
          "conv_stack_f8");
  }, "fp8 layer stack (C = 128 | 256; epi 1 forward e4m3, 2 backward-data e5m2): table rows "
     "{A8_frag, pbias_frag, Y, mask, s_in, s_w, s_out, amax_out}; X0 quantized with *s_x0");
  m.def("conv_stack_f8_y8", [](int C, int epi, uintptr_t table, int nl, uintptr_t X0,
                               uintptr_t s_x0, uintptr_t amax_x0, int B, uintptr_t y8,
                               uintptr_t stream) {
    check(dg_conv_stack_f8(C, epi, P<long long>(table), nl, P<void>(X0), P<float>(s_x0),
                           P<unsigned>(amax_x0), B, P<long long>(y8), nullptr, S(stream)),
          "conv_stack_f8_y8");
  }, "conv_stack_f8 + fp8 copy-out: y8 = nl + 1 int64 {X8_0, Y8 of each layer} (448-row "
     "frames; the last layer's 0)");
  m.def("conv_stack_f8_dgrad", [](int C, uintptr_t table, int nl, uintptr_t X0,
                                  uintptr_t s_x0, uintptr_t amax_x0, int B, uintptr_t y8,
                                  uintptr_t sr_step, uintptr_t stream) {
    check(dg_conv_stack_f8(C, 2, P<long long>(table), nl, P<void>(X0), P<float>(s_x0),
                           P<unsigned>(amax_x0), B, P<long long>(y8), P<long long>(sr_step),
                           S(stream)),
          "conv_stack_f8_dgrad");
  }, "the e5m2 backward-data stack (conv_stack_f8 epi 2) with optional fp8 copies (y8, 0: "
     "none) and stochastic rounding seeded by the int64 device step counter sr_step (0: "
     "round to nearest even)");
  m.def("conv_wgrad_win8_set_ablate", [](int mode) { dg_conv_wgrad_win8_set_ablate(mode); },
        "conv_wgrad_win8 timing ablation (tools/kbench_win8.py; 0 = production): 1 no MFMA, "
        "2 no LDS reads, 4 no LDS-DMA, 8 no slab store, 16 no barrier (sums of these)");
  m.def("conv_wgrad_win8", [](uintptr_t table, int nl, int M, int Mpad, int Cx, int B, int KP,
                              int splits, uintptr_t sf, uintptr_t stream) {
    check(dg_conv_wgrad_win8(P<long long>(table), nl, M, Mpad, Cx, B, KP, splits,
                             P<long long>(sf), S(stream)),
          "conv_wgrad_win8");
  }, "MX-fp8 sliding-window weight gradients: table rows {dZ8 (e5m2), X8 (e4m3), slab, s_dz, "
     "s_x} (448-row fp8 frames)");
  m.def("conv_wgrad_win8_splits", [](int nl, int M, int Cx, int B, int num_cus) {
    return dg_conv_wgrad_win8_splits(nl, M, Cx, B, num_cus);
  });
  m.def("conv_stack_f8_fwd_head", [](int C, uintptr_t table, int nl, uintptr_t X0,
                                     uintptr_t s_x0, uintptr_t amax_x0, int B, uintptr_t w,
                                     uintptr_t bias, uintptr_t posb, uintptr_t labels,
                                     uintptr_t loss, uintptr_t pred, uintptr_t dZ,
                                     uintptr_t gw_part, uintptr_t dzb, int head_relu,
                                     float grad_scale, uintptr_t stream) {
    check(dg_conv_stack_f8_fwd_head(C, P<long long>(table), nl, P<void>(X0), P<float>(s_x0),
                                    P<unsigned>(amax_x0), B, P<float>(w), P<float>(bias),
                                    P<float>(posb), P<int>(labels), P<float>(loss), P<int>(pred),
                                    P<void>(dZ), P<float>(gw_part), P<float>(dzb), head_relu,
                                    grad_scale, nullptr, S(stream)),
          "conv_stack_f8_fwd_head");
  }, "fp8 forward stack + the fused 3x3 policy head (C = 128 | 256)");
  m.def("conv_stack_f8_fwd_head_y8", [](int C, uintptr_t table, int nl, uintptr_t X0,
                                     uintptr_t s_x0, uintptr_t amax_x0, int B, uintptr_t w,
                                     uintptr_t bias, uintptr_t posb, uintptr_t labels,
                                     uintptr_t loss, uintptr_t pred, uintptr_t dZ,
                                     uintptr_t gw_part, uintptr_t dzb, int head_relu,
                                     float grad_scale, uintptr_t y8, uintptr_t stream) {
    check(dg_conv_stack_f8_fwd_head(C, P<long long>(table), nl, P<void>(X0), P<float>(s_x0),
                                    P<unsigned>(amax_x0), B, P<float>(w), P<float>(bias),
                                    P<float>(posb), P<int>(labels), P<float>(loss), P<int>(pred),
                                    P<void>(dZ), P<float>(gw_part), P<float>(dzb), head_relu,
                                    grad_scale, P<long long>(y8), S(stream)),
          "conv_stack_f8_fwd_head_y8");
  }, "conv_stack_f8_fwd_head + fp8 copy-out (y8 as conv_stack_f8_y8)");
  m.def("conv_stack_f8_set_mode", [](int m) { dg_conv_stack_f8_set_mode(m); },
        "conv_stack_f8 timing-ablation mode (0 = production)");
  m.def("conv_stack_f8_set_debug", [](uintptr_t dbg) {
    dg_conv_stack_f8_set_debug(P<unsigned long long>(dbg));
  }, "conv_stack_f8 diagnostics: s_memtime phase stamps of boards 0..7 into dbg "
     "([8][8 waves][24 layers][8] uint64; 0 = off; C = 128 production variants)");
  m.def("conv_stack_f8_set_sched", [](int stag, int delay) {
    dg_conv_stack_f8_set_sched(stag, delay);
  }, "conv_stack_f8 (C = 128) schedule: staggered two-group on / off (overrides "
     "DG_STACK_F8_STAG; 0 off, 1 both stacks, 2 backward-data only), co-half-1 start delay");
  m.def("conv_stack2_set_mode", [](int on) { dg_conv_stack2_set_mode(on); },
        "conv_stack2 timing-ablation mode (tools/kbench_stack.py; 0 = production)");
  m.def("conv_stack2_set_sched", [](int stag, int prio, int delay) {
    dg_conv_stack2_set_sched(stag, prio, delay);
  }, "conv_stack2 schedule: staggered two-group on / off (overrides DG_STACK2_STAG), co-half-0 "
     "MFMA priority 0..2, co-half-1 start delay");
  m.def("conv_stack2", [](int epi, uintptr_t table, int nl, uintptr_t X0, int l1, int B,
                          uintptr_t stream) {
    check(dg_conv_stack2(epi, P<long long>(table), nl, P<void>(X0), l1, B, S(stream)),
          "conv_stack2");
  }, "conv_stack2: EPI_FWD forward or EPI_DGRAD backward-data chain (fragment-ordered A)");
  m.def("conv_wgrad", [](int kw, uintptr_t dZ, int dz_pad, int M, int Mpad, uintptr_t X,
                         int x_pad, int x_C, int B, int KP, int splits, uintptr_t slab,
                         uintptr_t stream) {
    check(dg_conv_wgrad(kw, P<void>(dZ), dz_pad, M, Mpad, P<void>(X), x_pad, x_C, B, KP,
                        splits, P<float>(slab), S(stream)),
          "conv_wgrad");
  });
  m.def("conv_board_fp8", [](int kw, int bm, uintptr_t A8, int KP, int M, int Mpad, uintptr_t X8,
                             int x_pad, int x_C, int B, uintptr_t Y, uintptr_t Y8, int y_pad,
                             uintptr_t bias, uintptr_t posb, uintptr_t s_x, uintptr_t s_w,
                             uintptr_t s_y, uintptr_t amax_y, uintptr_t mask, uintptr_t stream) {
    check(dg_conv_board_fp8(kw, bm, P<void>(A8), KP, M, Mpad, P<void>(X8), x_pad, x_C, B,
                            P<void>(Y), P<void>(Y8), y_pad, P<float>(bias), P<float>(posb),
                            P<float>(s_x), P<float>(s_w), P<float>(s_y), P<unsigned>(amax_y),
                            P<void>(mask), S(stream)),
          "conv_board_fp8");
  });
  m.def("fp8_update_scales", [](int n, uintptr_t scales, uintptr_t amax_w, int nparts_w,
                                uintptr_t amax_y, float w_margin, float g_headroom,
                                uintptr_t sat, uintptr_t gscales, uintptr_t gamax,
                                uintptr_t ghist, uintptr_t stream) {
    check(dg_fp8_update_scales(n, P<float>(scales), P<unsigned>(amax_w), nparts_w,
                               P<unsigned>(amax_y), w_margin, g_headroom, P<int>(sat),
                               P<float>(gscales), P<unsigned>(gamax), P<float>(ghist),
                               S(stream)),
          "fp8_update_scales");
  });
  m.def("weight_fp8", [](uintptr_t w, uintptr_t wf8, int cout, int cin, int taps, int cinp,
                         int kp, uintptr_t s_w, uintptr_t stream) {
    check(dg_weight_fp8(P<float>(w), P<void>(wf8), cout, cin, taps, cinp, kp, P<float>(s_w),
                        S(stream)),
          "weight_fp8");
  });
  m.def("frame_to_fp8", [](uintptr_t src, uintptr_t dst, size_t n, uintptr_t scale,
                           uintptr_t amax, uintptr_t stream) {
    check(dg_frame_to_fp8(P<void>(src), P<void>(dst), n, P<float>(scale), P<unsigned>(amax),
                          S(stream)),
          "frame_to_fp8");
  });
  m.def("wgrad_reduce_multi", [](uintptr_t table, int nl, uintptr_t stream) {
    check(dg_wgrad_reduce_multi(P<long long>(table), nl, 13, S(stream)), "wgrad_reduce_multi");
  }, "slab reduce + bias pass 2 of nl layers: table rows {slab, out, bpart, gposb, gbias, "
     "splits, M, Mpad, KP, taps, cin, cinp, bchunks}");
  m.def("wgrad_reduce_multi_w", [](uintptr_t table, int nl, uintptr_t stream) {
    check(dg_wgrad_reduce_multi(P<long long>(table), nl, 16, S(stream)), "wgrad_reduce_multi_w");
  }, "wgrad_reduce_multi writing bf16 twins too: rows + {out16, gposb16, gbias16}");
  m.def("bias_grad_partial_multi", [](uintptr_t table, int nl, int B, int C, int pad,
                                      uintptr_t sf, uintptr_t stream) {
    check(dg_bias_grad_partial_multi(P<long long>(table), nl, B, C, pad, P<long long>(sf),
                                     S(stream)),
          "bias_grad_partial_multi");
  });
  m.def("wgrad_reduce", [](uintptr_t slab, uintptr_t out, int splits, int M, int Mpad, int KP,
                           int taps, int cin, int cinp, uintptr_t bpart, int bchunks,
                           uintptr_t gposb, uintptr_t gbias, uintptr_t sf, uintptr_t stream) {
    check(dg_wgrad_reduce(P<float>(slab), P<float>(out), splits, M, Mpad, KP, taps, cin, cinp,
                          P<float>(bpart), bchunks, P<float>(gposb), P<float>(gbias), nullptr,
                          nullptr, nullptr, P<long long>(sf), S(stream)),
          "wgrad_reduce");
  });
  m.def("wgrad_reduce_w", [](uintptr_t slab, uintptr_t out, int splits, int M, int Mpad, int KP,
                             int taps, int cin, int cinp, uintptr_t bpart, int bchunks,
                             uintptr_t gposb, uintptr_t gbias, uintptr_t out16,
                             uintptr_t gposb16, uintptr_t gbias16, uintptr_t sf,
                             uintptr_t stream) {
    check(dg_wgrad_reduce(P<float>(slab), P<float>(out), splits, M, Mpad, KP, taps, cin, cinp,
                          P<float>(bpart), bchunks, P<float>(gposb), P<float>(gbias),
                          P<void>(out16), P<void>(gposb16), P<void>(gbias16), P<long long>(sf),
                          S(stream)),
          "wgrad_reduce_w");
  }, "wgrad_reduce writing bf16 twins of the weight / position-bias / bias gradients too");
  m.def("head_reduce", [](uintptr_t dzb, uintptr_t gw_part, int B, int n, uintptr_t gw,
                          uintptr_t gbias, uintptr_t gposb, uintptr_t sf, uintptr_t stream) {
    check(dg_head_reduce(P<float>(dzb), P<float>(gw_part), B, n, P<float>(gw), P<float>(gbias),
                         P<float>(gposb), nullptr, nullptr, nullptr, P<long long>(sf), S(stream)),
          "head_reduce");
  });
  m.def("head_reduce_w", [](uintptr_t dzb, uintptr_t gw_part, int B, int n, uintptr_t gw,
                            uintptr_t gbias, uintptr_t gposb, uintptr_t gw16, uintptr_t gbias16,
                            uintptr_t gposb16, uintptr_t sf, uintptr_t stream) {
    check(dg_head_reduce(P<float>(dzb), P<float>(gw_part), B, n, P<float>(gw), P<float>(gbias),
                         P<float>(gposb), P<void>(gw16), P<void>(gbias16), P<void>(gposb16),
                         P<long long>(sf), S(stream)),
          "head_reduce_w");
  }, "head_reduce writing bf16 twins too");
  m.def("head", [](int kw, uintptr_t X, int x_pad, int C, int B, uintptr_t w, uintptr_t bias,
                   uintptr_t posb, uintptr_t labels, uintptr_t loss, uintptr_t pred,
                   uintptr_t logp, uintptr_t dZ, int dz_pad, uintptr_t gw, uintptr_t gbias,
                   uintptr_t gposb, int head_relu, float grad_scale, uintptr_t stream) {
    check(dg_head(kw, P<void>(X), x_pad, C, B, P<float>(w), P<float>(bias), P<float>(posb),
                  P<int>(labels), P<float>(loss), P<int>(pred), P<float>(logp), P<void>(dZ),
                  dz_pad, P<float>(gw), P<float>(gbias), P<float>(gposb), head_relu, grad_scale,
                  S(stream)),
          "head");
  });
  m.def("expand_features", [](uintptr_t planes, uintptr_t player, uintptr_t rank, uintptr_t out,
                              int B, int pad, int CP, uintptr_t stream) {
    check(dg_expand_features(P<uint8_t>(planes), P<uint8_t>(player), P<uint8_t>(rank),
                             P<void>(out), B, pad, CP, nullptr, 0, S(stream)),
          "expand_features");
  });
  m.def("bias_grad_partial", [](uintptr_t dZ, int B, int C, int pad, uintptr_t part,
                                uintptr_t stream) {
    check(dg_bias_grad_partial(P<void>(dZ), B, C, pad, P<float>(part), S(stream)),
          "bias_grad_partial");
  });
  m.def("comm_proxy", [](uintptr_t buf, long long nbytes, int world, double gbps, int blocks,
                         uintptr_t stream) {
    check(dg_comm_proxy(P<void>(buf), nbytes, world, gbps, blocks, S(stream)), "comm_proxy");
  });
  m.def("bias_chunks", [](int B) { return dg_bias_chunks(B); });
  m.def("bias_chunks_multi", [](int B) { return dg_bias_chunks_multi(B); });
  m.def("sgd", [](uintptr_t p, uintptr_t g, size_t n, uintptr_t lr, float gscale,
                  uintptr_t gate, uintptr_t stream) {
    check(dg_sgd(P<float>(p), P<float>(g), n, P<double>(lr), gscale, P<float>(gate), nullptr,
                 S(stream)),
          "sgd");
  });
  m.def("sgd_bf16", [](uintptr_t p, uintptr_t g16, size_t n, uintptr_t lr, float gscale,
                       uintptr_t gate, uintptr_t stream) {
    check(dg_sgd(P<float>(p), nullptr, n, P<double>(lr), gscale, P<float>(gate), P<void>(g16),
                 S(stream)),
          "sgd_bf16");
  }, "SGD reading the bf16 (wire-format) gradient");
  m.def("rmsprop", [](uintptr_t p, uintptr_t g, uintptr_t ms, size_t n, uintptr_t lr,
                      float decay, float gscale, uintptr_t gate, uintptr_t stream) {
    check(dg_rmsprop(P<float>(p), P<float>(g), P<float>(ms), n, P<double>(lr), decay, gscale,
                     P<float>(gate), nullptr, S(stream)),
          "rmsprop");
  });
  m.def("rmsprop_bf16", [](uintptr_t p, uintptr_t g16, uintptr_t ms, size_t n, uintptr_t lr,
                           float decay, float gscale, uintptr_t gate, uintptr_t stream) {
    check(dg_rmsprop(P<float>(p), nullptr, P<float>(ms), n, P<double>(lr), decay, gscale,
                     P<float>(gate), P<void>(g16), S(stream)),
          "rmsprop_bf16");
  }, "RMSProp reading the bf16 (wire-format) gradient");
  // loss (or 0) rank-local; grads (or 0) the flat (all-reduced) gradient: gate = all finite
  m.def("finite_gate", [](uintptr_t loss, int n, uintptr_t grads, size_t ng, uintptr_t gate,
                          uintptr_t bad, uintptr_t stream) {
    check(dg_finite_gate(P<float>(loss), n, P<float>(grads), ng, P<float>(gate), P<int>(bad),
                         nullptr, S(stream)),
          "finite_gate");
  });
  m.def("finite_gate_bf16", [](uintptr_t loss, int n, uintptr_t grads16, size_t ng,
                               uintptr_t gate, uintptr_t bad, uintptr_t stream) {
    check(dg_finite_gate(P<float>(loss), n, nullptr, ng, P<float>(gate), P<int>(bad),
                         P<void>(grads16), S(stream)),
          "finite_gate_bf16");
  }, "finite_gate over the bf16 (wire-format) gradient");
  m.def("finite_gate1", [](uintptr_t loss, int n, uintptr_t grads, uintptr_t grads16, size_t ng,
                           uintptr_t gate, uintptr_t bad, uintptr_t ticket, uintptr_t stream) {
    check(dg_finite_gate1(P<float>(loss), n, P<float>(grads), P<void>(grads16), ng,
                          P<float>(gate), P<int>(bad), P<unsigned>(ticket), S(stream)),
          "finite_gate1");
  }, "loss + gradient finite gate in one launch (fp32 grads or the bf16 twin grads16)");
  m.def("lr_decay", [](uintptr_t lr, double decay, uintptr_t step, uintptr_t stream) {
    check(dg_lr_decay(P<double>(lr), decay, P<long long>(step), S(stream)), "lr_decay");
  });
  m.def("weight_refresh", [](uintptr_t table, int n, uintptr_t stream) {
    check(dg_weight_refresh(P<long long>(table), n, nullptr, 0.0, nullptr, S(stream)),
          "weight_refresh");
  });
  m.def("weight_refresh_decay", [](uintptr_t table, int n, uintptr_t lr, double decay,
                                   uintptr_t step, uintptr_t stream) {
    check(dg_weight_refresh(P<long long>(table), n, P<double>(lr), decay, P<long long>(step),
                            S(stream)),
          "weight_refresh_decay");
  });
  m.def("grad_update_cols", []() { return dg_grad_update_cols(); });
  m.def("grad_update", [](uintptr_t table, int n, long long plain_off, long long plain_n,
                          uintptr_t p, uintptr_t g, uintptr_t g16, uintptr_t ms, float rms_decay,
                          float gscale, uintptr_t gate, uintptr_t lr, double decay,
                          uintptr_t step, uintptr_t tickets, uintptr_t bad, int write_grads,
                          int final, uintptr_t gflag, uintptr_t stream) {
    check(dg_grad_update(P<long long>(table), n, plain_off, plain_n, P<float>(p), P<float>(g),
                         P<void>(g16), P<float>(ms), rms_decay, gscale, P<float>(gate),
                         P<double>(lr), decay, P<long long>(step), P<unsigned>(tickets),
                         P<int>(bad), write_grads, final, P<long long>(gflag), S(stream)),
          "grad_update");
  }, "fused gradient pass 2 (slabs / bias partials, or the flat gradient) + SGD / RMSProp + "
     "operand refresh + LR decay (elementwise.hip grad_update_kernel)");
  m.def("grad_update_tickets", []() { return dg_grad_update_tickets(); },
        "uint32 ticket counters grad_update needs (zeroed once; the kernel leaves them zeroed)");
  m.def("conv_board_set_ablate", [](int mode) { dg_conv_board_set_ablate(mode); },
        "diagnostics: 1 skip MFMA, 2 skip LDS fragment reads, 4 skip DMA");
  m.def("conv_wgrad_set_ablate", [](int mode) { dg_conv_wgrad_set_ablate(mode); });
  m.def("conv_wgrad5_set_ns", [](int ns) { dg_conv_wgrad5_set_ns(ns); },
        "5x5 weight gradient: 0 = conv_wgrad_kernel, 4 | 5 = conv_wgrad_pipe_kernel stages");
  m.def("conv_wgrad_wgs_per_cu", []() { return dg_conv_wgrad_wgs_per_cu(); });
  m.def("conv_wgrad_multi", [](int kw, uintptr_t table, int nl, int dz_pad, int M, int Mpad,
                               int x_pad, int x_C, int B, int KP, int splits, uintptr_t stream) {
    check(dg_conv_wgrad_multi(kw, P<long long>(table), nl, dz_pad, M, Mpad, x_pad, x_C, B, KP,
                              splits, S(stream)),
          "conv_wgrad_multi");
  }, "weight gradients of several same-shape layers in one three-slice launch");
  m.def("conv_l1", [](int kw, uintptr_t A, int KP, int M, int Mpad, uintptr_t X, int x_pad,
                      int x_C, int B, uintptr_t Y, int y_pad, uintptr_t bias, uintptr_t posb,
                      uintptr_t mask, uintptr_t pbias, uintptr_t stream) {
    check(dg_conv_l1(kw, P<void>(A), KP, M, Mpad, P<void>(X), x_pad, x_C, B, P<void>(Y), y_pad,
                     P<float>(bias), P<float>(posb), P<void>(mask), P<void>(pbias), S(stream)),
          "conv_l1");
  }, "board-resident first-layer forward (conv_l1.hip): bias + position bias (fp32, or the "
     "bf16 pbias table when given) + ReLU");
  m.def("conv_l1_ok", [](int kw, int x_pad, int x_C, int Mpad, int KP) {
    return dg_conv_l1_ok(kw, x_pad, x_C, Mpad, KP);
  });
  m.def("conv_l1_frag", [](uintptr_t A, uintptr_t pbias, uintptr_t X, int B, int M, uintptr_t Y,
                           uintptr_t mask, uintptr_t planes, uintptr_t player, uintptr_t rank,
                           uintptr_t stream) {
    check(dg_conv_l1_frag(P<void>(A), P<void>(pbias), P<void>(X), B, M, P<void>(Y), P<void>(mask),
                          P<void>(planes), P<void>(player), P<void>(rank), S(stream)),
          "conv_l1_frag");
  }, "5x5 / 40-channel first layer, one board per workgroup, fragment-ordered weights "
     "(conv_l1.hip conv_l1_frag_kernel); planes/player/rank non-zero: the feature expansion "
     "fused in (X written)");
  m.def("conv_l1_frag_ok", [](int kw, int x_pad, int x_C, int M, int y_pad) {
    return dg_conv_l1_frag_ok(kw, x_pad, x_C, M, y_pad);
  });
  m.def("conv_layer2", [](int epi, uintptr_t A, uintptr_t pbias, uintptr_t X, uintptr_t Y,
                         uintptr_t mask, int C, int B, uintptr_t stream) {
    check(dg_conv_layer2(epi, P<void>(A), P<void>(pbias), P<void>(X), P<void>(Y), P<void>(mask),
                         C, B, S(stream)),
          "conv_layer2");
  }, "one hidden 3x3 C -> C layer (C = 256 | 128) on conv_stack2's K loop: epi 1 forward "
     "(fragment weights, pbias_frag, mask written), 2 backward-data (mask of the layer below)");
  m.def("conv_layer2_multi_head", [](uintptr_t table, int nl, int B, uintptr_t w,
                                     uintptr_t bias, uintptr_t posb, uintptr_t labels,
                                     uintptr_t loss, uintptr_t pred, uintptr_t dZ,
                                     uintptr_t gw_part, uintptr_t dzb, int head_relu,
                                     float grad_scale, uintptr_t stream) {
    check(dg_conv_layer2_multi_head(P<long long>(table), nl, B, P<float>(w), P<float>(bias),
                                    P<float>(posb), P<int>(labels), P<float>(loss),
                                    P<int>(pred), P<void>(dZ), P<float>(gw_part),
                                    P<float>(dzb), head_relu, grad_scale, S(stream)),
          "conv_layer2_multi_head");
  }, "d = 256 forward run + the fused 3x3/256 policy head on its last output");
  m.def("conv_layer2_multi", [](int epi, uintptr_t table, int nl, int C, int B,
                               uintptr_t stream) {
    check(dg_conv_layer2_multi(epi, P<long long>(table), nl, C, B, S(stream)),
          "conv_layer2_multi");
  }, "a run of nl conv_layer2 layers in one launch (one workgroup per board, the layers "
     "chained through the board's own L2-resident output); table rows {A, pbias, X, Y, mask}");
  m.def("conv_wgrad_win", [](uintptr_t table, int nl, int M, int Mpad, int Cx, int B, int KP,
                             int splits, uintptr_t sf, uintptr_t stream) {
    check(dg_conv_wgrad_win(P<long long>(table), nl, M, Mpad, Cx, B, KP, splits,
                            P<long long>(sf), S(stream)),
          "conv_wgrad_win");
  }, "sliding-window 3x3 weight gradients (frame-linear K, 9 taps per staged X window)");
  m.def("conv_wgrad_win_splits", [](int nl, int M, int Cx, int B, int num_cus) {
    return dg_conv_wgrad_win_splits(nl, M, Cx, B, num_cus);
  });
  m.def("conv_wgrad_win_set_ablate", [](int mode) { dg_conv_wgrad_win_set_ablate(mode); });
  m.def("conv_wgrad_ktile", [](int KP) { return dg_conv_wgrad_ktile(KP); });
  m.def("conv_wgrad_wgs_per_cu_for", [](int KP) { return dg_conv_wgrad_wgs_per_cu_for(KP); });
  m.def("device_sync", []() { check(hipDeviceSynchronize(), "hipDeviceSynchronize"); });
  m.def("last_error", []() { return std::string(hipGetErrorString(hipGetLastError())); });
}
