// Kernel lab (not product code): ablations of the pipelined split-bf16 NN GEMM (compress_split.hip,
// gemm_nn_split3_body's ABL bits) at the configs[3] forward shape, timed with hipEvents.  Outputs of
// ablated runs are garbage by design; only ABL = 0 is checked (against the library's kernel).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include tools/gemm_ablate.hip -o tools/bin/gemm_ablate
#include "lab_forms.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace mrp_host {
Tuning& tuning() {
  static Tuning t;
  return t;
}
}  // namespace mrp_host

namespace mrp_cs {
template <int ABL>
__global__ void __launch_bounds__(512, 1) abl_kernel(Args a) {
#if defined(__HIP_DEVICE_COMPILE__)  // the body's builtins exist only in the device pass
  gemm_nn_split3_body<4, 2, ABL>(a);
#endif
}
}  // namespace mrp_cs
using namespace mrp_cs;

template <int ABL>
float run(Args a, int iters, hipStream_t st) {
  using G = Geo3<4, 2>;
  a.mtiles = (a.M + G::TM - 1) / G::TM;
  const int grid = a.mtiles * (int)((a.ncols + TN - 1) / TN);
  hipFuncSetAttribute(reinterpret_cast<const void*>(&abl_kernel<ABL>), hipFuncAttributeMaxDynamicSharedMemorySize,
                      G::LDS_BYTES);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  std::vector<float> ts;
  for (int r = 0; r < 5; ++r) {
    hipEventRecord(e0, st);
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(abl_kernel<ABL>, dim3(grid), dim3(512), G::LDS_BYTES, st, a);
    hipEventRecord(e1, st);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    ts.push_back(ms * 1000 / iters);
  }
  std::sort(ts.begin(), ts.end());
  return ts[2];
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 64, C = argc > 2 ? atoi(argv[2]) : 2048, P = argc > 3 ? atoi(argv[3]) : 64;
  const size_t plane = (size_t)n * C * P;
  float *x, *ag, *y;
  void* pk;
  hipMalloc(&x, plane * 4);
  hipMalloc(&ag, plane * 4);
  hipMalloc(&y, plane * 4);
  hipMalloc(&pk, (size_t)C * 2 * C * 6);
  std::vector<float> h(plane);
  for (size_t i = 0; i < plane; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
  hipMemcpy(x, h.data(), plane * 4, hipMemcpyHostToDevice);
  hipMemcpy(ag, h.data(), plane * 4, hipMemcpyHostToDevice);
  hipMemset(pk, 0x3c, (size_t)C * 2 * C * 6);
  hipStream_t st;
  hipStreamCreate(&st);
  Args a = {};
  a.ap = static_cast<const u4*>(pk);
  a.b0 = x, a.b0s = (int64_t)C * P, a.b1 = ag, a.b1s = (int64_t)C * P;
  a.c0 = y, a.c0s = (int64_t)C * P, a.c1 = y, a.c1s = (int64_t)C * P;
  a.bias = nullptr, a.ncols = (int64_t)n * P, a.M = C, a.K = 2 * C, a.k0 = C, a.m0 = C, a.P = P;
  const double flop = 2.0 * C * 2.0 * C * n * P;
  for (int rep = 0; rep < 2; ++rep) {
    float t;
#define R(ABL)                                                                                          \
  t = run<ABL>(a, 10, st);                                                                               \
  printf("ABL=%2d (%s%s%s%s) %8.1f us %6.1f TF/s\n", ABL, (ABL & 1) ? "noDMA " : "", (ABL & 2) ? "noBload " : "", \
         (ABL & 4) ? "noBarrier " : "", (ABL & 8) ? "noSplit" : "", t, flop / t / 1e6);
    R(0) R(1) R(2) R(3) R(4) R(8) R(10) R(15)
  }
  return 0;
}
