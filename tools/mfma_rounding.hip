// Lab (not product code): how v_mfma_f32_32x32x16_bf16 rounds when it adds its products to the
// accumulator.  C = +-1, one product of +-m * 2^-23 (m = 1.25, 1.5, 1.75) at k = 0, the other 15 zero:
// round-to-nearest-even gives +-(1 + round(m) 2^-23), truncation +-(1 + floor(m) 2^-23).  Also a
// 16-product sum of 2^-26 terms onto 1 (exact sum first: 1 + 2^-22; one by one RNE: 1).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k(float cval, float prod, int all16, float* out) {
  const int l = threadIdx.x;
  bf8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int kk = 8 * (l >> 5) + j;
    a[j] = (__bf16)1.f;
    b[j] = (__bf16)((all16 || kk == 0) ? prod : 0.f);
  }
  f16v c;
  for (int i = 0; i < 16; ++i) c[i] = cval;
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  if (l == 0) out[0] = c[0];
}

int main() {
  float* d;
  hipMalloc(&d, 4);
  const float u = 1.0f / (1 << 23);
  struct { float c, p; int all; const char* what; } cases[] = {
      {1.f, 1.25f * u, 0, "1 + 1.25ulp"}, {1.f, 1.5f * u, 0, "1 + 1.5ulp"}, {1.f, 1.75f * u, 0, "1 + 1.75ulp"},
      {-1.f, -1.5f * u, 0, "-1 - 1.5ulp"}, {-1.f, -1.75f * u, 0, "-1 - 1.75ulp"}, {1.f, -0.5f * u, 0, "1 - 0.5ulp"},
      {1.f, u / 8, 1, "1 + 16 x ulp/8"}};
  for (auto& cs : cases) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, cs.c, cs.p, cs.all, d);
    float h;
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("%-16s -> 1 + %.4f ulp (raw %.9g)\n", cs.what, (double(h) - double(cs.c)) / u * (cs.c < 0 ? -1 : 1) + 0.0, h);
  }
  return 0;
}
