// Probe the v_mfma_f32_32x32x16_bf16 operand / result lane maps on hardware.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
// A[32][16] row-major, B[16][32] row-major in global; assumed maps:
// lane l: A[l&31][8*(l>>5)+j], B[8*(l>>5)+j][l&31]; D lane l reg r: D[(r&3)+8*(r>>2)+4*(l>>5)][l&31]
__global__ void k(const float* A, const float* B, float* D, float* Draw) {
  int l = threadIdx.x, r = l & 31, h = l >> 5;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)A[r * 16 + 8 * h + j]; b[j] = (__bf16)B[(8 * h + j) * 32 + r]; }
  f32x16 acc = {};
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  for (int g = 0; g < 16; ++g) {
    D[((g & 3) + 8 * (g >> 2) + 4 * h) * 32 + r] = acc[g];
    Draw[l * 16 + g] = acc[g];
  }
}
int main() {
  float hA[512], hB[512], hD[1024], hR[1024];
  for (int i = 0; i < 512; ++i) { hA[i] = (float)((i * 7) % 5 - 2); hB[i] = (float)((i * 3) % 7 - 3); }
  float *A, *B, *D, *R;
  hipMalloc(&A, 2048); hipMalloc(&B, 2048); hipMalloc(&D, 4096); hipMalloc(&R, 4096);
  hipMemcpy(A, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(B, hB, 2048, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, A, B, D, R);
  hipMemcpy(hD, D, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
    float s = 0; for (int kk = 0; kk < 16; ++kk) s += hA[i * 16 + kk] * hB[kk * 32 + j];
    if (s != hD[i * 32 + j]) ++bad;
  }
  printf("layout mismatches: %d of 1024\n", bad);
  return 0;
}
