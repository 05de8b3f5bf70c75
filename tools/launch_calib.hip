// Launch / dispatch overhead calibration: empty kernels with different dynamic LDS sizes,
// back-to-back stream launches vs one hipGraph of the same launches.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(512) empty_k(int* out, int n) {
  extern __shared__ int sm[];
  if (n < 0) { sm[threadIdx.x] = n; __syncthreads(); out[0] = sm[0]; }
}
__global__ void __launch_bounds__(512) barrier_k(int* out, int n) {
  extern __shared__ int sm[];
  for (int i = 0; i < n; ++i) __syncthreads();
  if (n < 0) out[0] = sm[0];
}
int main() {
  int* out;
  (void)hipMalloc(&out, 4);
  hipStream_t s;
  (void)hipStreamCreate(&s);
  for (int lds : {0, 16384, 65536, 147456}) {
    (void)hipFuncSetAttribute((const void*)empty_k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    (void)hipFuncSetAttribute((const void*)barrier_k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    for (int blocks : {256, 512}) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      const int N = 50;
      for (int i = 0; i < 5; ++i) empty_k<<<blocks, 512, lds, s>>>(out, 1);
      (void)hipEventRecord(e0, s);
      for (int i = 0; i < N; ++i) empty_k<<<blocks, 512, lds, s>>>(out, 1);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float ms; (void)hipEventElapsedTime(&ms, e0, e1);
      // graph of N launches
      hipGraph_t g; hipGraphExec_t ge;
      (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
      for (int i = 0; i < N; ++i) empty_k<<<blocks, 512, lds, s>>>(out, 1);
      (void)hipStreamEndCapture(s, &g);
      (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      (void)hipGraphLaunch(ge, s);
      (void)hipStreamSynchronize(s);
      (void)hipEventRecord(e0, s);
      (void)hipGraphLaunch(ge, s);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float msg; (void)hipEventElapsedTime(&msg, e0, e1);
      // barrier-only kernel: 18 barriers
      (void)hipEventRecord(e0, s);
      for (int i = 0; i < N; ++i) barrier_k<<<blocks, 512, lds, s>>>(out, 18);
      (void)hipEventRecord(e1, s);
      (void)hipEventSynchronize(e1);
      float msb; (void)hipEventElapsedTime(&msb, e0, e1);
      printf("lds=%6d blocks=%d  stream: %.2f us/launch   graph: %.2f us/launch   18-barrier kernel: %.2f us\n",
             lds, blocks, ms * 1000 / N, msg * 1000 / N, msb * 1000 / N);
    }
  }
  return 0;
}
