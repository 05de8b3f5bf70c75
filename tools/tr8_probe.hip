// Probe the lane mapping of ds_read_b64_tr_b8 (gfx950): every lane supplies the address
// base + 8 * lane of a 512-byte LDS region whose bytes encode their own offset (two passes:
// offset & 0xff, offset >> 8); each lane prints which source byte offsets it received.
// Run on the box: hipcc --offload-arch=gfx950 -O2 tools/tr8_probe.hip -o /tmp/tr8 && /tmp/tr8
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef __attribute__((ext_vector_type(2))) int i32x2;

__global__ void probe(unsigned char* out, int hi) {
  __shared__ __attribute__((aligned(16))) unsigned char s[512];
  for (int i = threadIdx.x; i < 512; i += 64) s[i] = hi ? (unsigned char)(i >> 8) : (unsigned char)i;
  __syncthreads();
  const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
      (__attribute__((address_space(3))) i32x2*)(s + threadIdx.x * 8));
  *(i32x2*)(out + threadIdx.x * 8) = v;
}

int main() {
  unsigned char *d, lo[512], hi[512];
  hipMalloc(&d, 512);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 0);
  hipMemcpy(lo, d, 512, hipMemcpyDeviceToHost);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, 1);
  hipMemcpy(hi, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int j = 0; j < 8; ++j) printf(" %3d", lo[l * 8 + j] | (hi[l * 8 + j] << 8));
    printf("\n");
  }
  return 0;
}
