// MFMA throughput calibration: each wave issues N independent-accumulator 16x16x32 bf16
// MFMAs.  Reports the per-SIMD cycles per MFMA from wall time and the device clock.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void __launch_bounds__(512) k(float* out, int iters, float seed) {
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) { a[i] = (__bf16)(seed * (threadIdx.x + i)); b[i] = (__bf16)(seed - i); }
  f32x4 c[8] = {};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c[j], 0, 0, 0);
  }
  float s = 0;
  for (int j = 0; j < 8; ++j) s += c[j][0] + c[j][1] + c[j][2] + c[j][3];
  if (s == 1234.5f) out[0] = s;
}
int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("name=%s CUs=%d clock_khz=%d maxSharedPerBlock=%zu sharedPerMP=%zu\n", p.gcnArchName,
         p.multiProcessorCount, clk, p.sharedMemPerBlock, p.maxSharedMemoryPerMultiProcessor);
  float* out;
  hipMalloc(&out, 4);
  const int iters = 2000;
  for (int blocks : {p.multiProcessorCount, 256, 512, 1024}) {
    for (int threads : {256, 512}) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      k<<<blocks, threads>>>(out, 10, 1.f);
      hipEventRecord(e0);
      k<<<blocks, threads>>>(out, iters, 1.f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double mfma = (double)blocks * threads / 64 * iters * 8;
      double tflops = mfma * 16384 / (ms * 1e-3) / 1e12;
      printf("blocks=%d threads=%d ms=%.3f TFLOPs=%.1f\n", blocks, threads, ms, tflops);
    }
  }
  return 0;
}
