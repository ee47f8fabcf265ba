// Dev probe: operand / result lane layout of v_mfma_f32_4x4x4_16b_bf16 (16 independent 4x4x4
// blocks per wave) on gfx950.  Prints per lane its A, B (4 bf16 each, small integers) and D (4 f32)
// as text; tools/mfma4_probe.py fits the layout.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ short bf(float f) { return (short)(__float_as_uint(f) >> 16); }

__global__ void probe(float* out) {
  const int l = threadIdx.x;
  s16x4 a, b;
  float av[4], bv[4];
  for (int k = 0; k < 4; ++k) {
    av[k] = (float)((l * 7 + k * 3) % 11 - 5);
    bv[k] = (float)((l * 5 + k * 13) % 7 - 3);
    a[k] = bf(av[k]);
    b[k] = bf(bv[k]);
  }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  f32x4 d = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, c, 0, 0, 0);
  for (int k = 0; k < 4; ++k) {
    out[l * 12 + k] = av[k];
    out[l * 12 + 4 + k] = bv[k];
    out[l * 12 + 8 + k] = d[k];
  }
}

int main() {
  float* d;
  if (hipMalloc(&d, 64 * 12 * sizeof(float)) != hipSuccess) return 1;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  float h[64 * 12];
  if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 2;
  for (int l = 0; l < 64; ++l) {
    for (int k = 0; k < 12; ++k) printf("%g ", h[l * 12 + k]);
    printf("\n");
  }
  return 0;
}
