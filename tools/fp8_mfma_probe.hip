// Probe the operand lane layout of v_mfma_scale_f32_16x16x128_f8f6f4 (fp8 e4m3, unit
// block scales) with exact small-integer data, against candidate maps.  Run on the box:
//   hipcc --offload-arch=gfx950 -O2 tools/fp8_mfma_probe.hip -o tools/fp8_mfma_probe
//   ./tools/fp8_mfma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// e4m3fn encoding of small non-negative integers 0..8
static uint8_t enc(int v) {
  static const uint8_t t[9] = {0x00, 0x38, 0x40, 0x44, 0x48, 0x4A, 0x4C, 0x4E, 0x50};
  return t[v];
}

__global__ void probe(const uint8_t* A, const uint8_t* B, float* D, int mode) {
  // A/B given as per-lane 32-byte fragments already laid out on the host
  const int l = threadIdx.x;
  i32x8 a, b;
  memcpy(&a, A + l * 32, 32);
  memcpy(&b, B + l * 32, 32);
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  for (int r = 0; r < 4; ++r) D[l * 4 + r] = c[r];
}

// candidate k index of byte j held by lane l
static int kmap(int mode, int l, int j) {
  const int g = l >> 4;
  switch (mode) {
    case 0: return 32 * g + j;                                        // contiguous 32
    case 1: return j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16);      // two 16-halves
    case 2: return (j / 8) * 32 + 8 * g + (j % 8);                    // 8-byte interleave
    case 3: return j < 16 ? 16 * g + j : 64 + 16 * g + j - 16;        // (same as 1)
    default: return -1;
  }
}

int main() {
  int Aref[16][128], Bref[128][16];
  unsigned s = 12345;
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 128; ++k) { s = s * 1103515245 + 12345; Aref[i][k] = (s >> 16) % 4; }
  for (int k = 0; k < 128; ++k)
    for (int j = 0; j < 16; ++j) { s = s * 1103515245 + 12345; Bref[k][j] = (s >> 16) % 3 + (j == k % 16); }
  double ref[16][16];
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j) {
      double acc = 0;
      for (int k = 0; k < 128; ++k) acc += Aref[i][k] * Bref[k][j];
      ref[i][j] = acc;
    }
  uint8_t *dA, *dB;
  float* dD;
  hipMalloc(&dA, 64 * 32);
  hipMalloc(&dB, 64 * 32);
  hipMalloc(&dD, 64 * 4 * 4);
  for (int mode = 0; mode < 3; ++mode) {
    uint8_t hA[64 * 32], hB[64 * 32];
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 32; ++j) {
        const int k = kmap(mode, l, j);
        hA[l * 32 + j] = enc(Aref[l & 15][k]);
        hB[l * 32 + j] = enc(Bref[k][l & 15]);
      }
    hipMemcpy(dA, hA, sizeof(hA), hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof(hB), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, mode);
    float hD[256];
    hipMemcpy(hD, dD, sizeof(hD), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        const int col = l & 15, row = (l >> 4) * 4 + r;
        if (hD[l * 4 + r] != (float)ref[row][col]) ++bad;
      }
    printf("mode %d: mismatches %d / 256 (D[0][0]=%g ref %g)\n", mode, bad, hD[0], ref[0][0]);
  }
  return 0;
}
