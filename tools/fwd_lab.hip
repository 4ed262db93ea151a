// fwd_lab.hip — forward-only timing lab (not product code): the product film_fwd at forced
// (channels per block, plane segments per workgroup) geometries against plain float4 copies of the
// same byte count, to locate the copy ceiling the forward is chasing.  Finding (round 1): one slice
// per lane (plane split over workgroups) streams like the best grid-stride copy; a software
// prefetch of the next slice (tried as a template flag) gained 3-5 % at two or more slices per
// lane and nothing at one.  HIP events, median of `iters` launches.
// Also the fused backward at forced lanes-per-plane (lpc > 64: a plane spans several waves).
// Usage: fwd_lab [B N C HW iters [bwd_only]]
#include "../multi-robot-perception-gnn-1_amd/csrc/film_mean_fwd.hip"
#include "../multi-robot-perception-gnn-1_amd/csrc/film_mean_bwd.hip"
#include "../multi-robot-perception-gnn-1_amd/csrc/film_mean_bwd_1_8.hip"
#include "../multi-robot-perception-gnn-1_amd/csrc/film_mean_bwd_9_12.hip"
#include "../multi-robot-perception-gnn-1_amd/csrc/film_mean_bwd_13_16.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

namespace lab {
using mrp::f4;
// grid-stride copy, U independent float4 per thread per trip, optionally nontemporal
template <int U, bool NTL>
__global__ void __launch_bounds__(256) copy_u(const f4* __restrict__ in, f4* __restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NTL ? __builtin_nontemporal_load(in + i + k * stride) : in[i + k * stride];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      if (NTL)
        __builtin_nontemporal_store(v[k], out + i + k * stride);
      else
        out[i + k * stride] = v[k];
    }
  }
  for (; i < n; i += stride) out[i] = in[i];
}
}  // namespace lab

template <typename F>
static float time_ms(F&& launch, int iters) {
  hipEvent_t s, e;
  CK(hipEventCreate(&s));
  CK(hipEventCreate(&e));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int i = 0; i < iters; ++i) {
    CK(hipEventRecord(s));
    launch();
    CK(hipEventRecord(e));
    CK(hipEventSynchronize(e));
    float ms;
    CK(hipEventElapsedTime(&ms, s, e));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  CK(hipEventDestroy(s));
  CK(hipEventDestroy(e));
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32;
  const int N = argc > 2 ? atoi(argv[2]) : 8;
  const int C = argc > 3 ? atoi(argv[3]) : 512;
  const int HW = argc > 4 ? atoi(argv[4]) : 32;
  const int iters = argc > 5 ? atoi(argv[5]) : 30;
  if (N != 8 || HW * HW % 4 != 0) {
    fprintf(stderr, "fwd_lab: N=8 only\n");
    return 2;
  }
  const int P = HW * HW, Nt = B * N, E = B * N * (N - 1);
  const size_t feat = (size_t)Nt * C * P;
  float *x, *out, *gb;
  CK(hipMalloc(&x, feat * 4));
  CK(hipMalloc(&out, feat * 4));
  CK(hipMalloc(&gb, (size_t)E * C * 2 * 4));
  {
    std::vector<float> h(feat);
    for (size_t i = 0; i < feat; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(x, h.data(), feat * 4, hipMemcpyHostToDevice));
    std::vector<float> hg((size_t)E * C * 2);
    for (size_t i = 0; i < hg.size(); ++i) hg[i] = (float)((i * 40503u) % 1000) / 1000.f;
    CK(hipMemcpy(gb, hg.data(), hg.size() * 4, hipMemcpyHostToDevice));
  }
  const double alg = (double)feat * 8 + (double)E * C * 2 * 4;
  printf("workload B=%d N=%d C=%d %dx%d complete: alg bytes %.1f MB\n", B, N, C, HW, HW, alg / 1e6);
  auto report = [&](const char* name, float ms, double bytes) {
    printf("%-44s %9.1f us  %7.0f GB/s  %5.1f%% of 8 TB/s\n", name, ms * 1e3, bytes / ms / 1e6,
           bytes / ms / 1e6 / 80.0);
    fflush(stdout);
  };
  const size_t n4 = feat / 4;
  char nm[96];
  const bool bwd_only = argc > 6;
  for (int grid : {8192, 16384, 32768, 65536}) {
    if (bwd_only) break;
    snprintf(nm, sizeof nm, "copy U1 nt grid=%d", grid);
    report(nm, time_ms([&] { hipLaunchKernelGGL((lab::copy_u<1, true>), dim3(grid), dim3(256), 0, 0, (const mrp::f4*)x, (mrp::f4*)out, n4); }, iters), (double)feat * 8);
    snprintf(nm, sizeof nm, "copy U1 plain grid=%d", grid);
    report(nm, time_ms([&] { hipLaunchKernelGGL((lab::copy_u<1, false>), dim3(grid), dim3(256), 0, 0, (const mrp::f4*)x, (mrp::f4*)out, n4); }, iters), (double)feat * 8);
  }
  // product entry point
  report("product mrp_film_mean_fwd", time_ms([&] {
    CK((hipError_t)mrp_film_mean_fwd(x, (int64_t)C * P, gb, nullptr, nullptr, nullptr, nullptr, B, N, MRP_GRAPH_COMPLETE, Nt, E, C, P,
                          MRP_AGG_FILM_MEAN | MRP_AGG_GB_LOGITS, out, (int64_t)C * P, nullptr));
  }, iters), alg);
  {
    float* cat;
    CK(hipMalloc(&cat, feat * 8));
    report("product mrp_film_mean_cat_fwd (x + agg)", time_ms([&] {
      CK((hipError_t)mrp_film_mean_cat_fwd(x, (int64_t)C * P, gb, nullptr, nullptr, nullptr, nullptr, B, N, MRP_GRAPH_COMPLETE, Nt, E, C, P,
                                MRP_AGG_FILM_MEAN | MRP_AGG_GB_LOGITS, cat, 2 * (int64_t)C * P, nullptr));
    }, iters), alg + (double)feat * 4);
    CK(hipFree(cat));
  }
  for (int cpb : {4, 2}) {
    if (bwd_only) break;
    for (int ps : {1, 2, 4, 8}) {
      const int lpc = 64;
      mrp::AggArgs a = {};
      a.x = x; a.xs = (int64_t)C * P; a.gb = gb; a.out = out; a.os = (int64_t)C * P; a.C = C; a.P = P; a.PV = P / 4;
      a.mode = MRP_AGG_FILM_MEAN; a.logits = 1; a.lpc = lpc; a.cpb = cpb; a.ncb = (C + cpb - 1) / cpb; a.psplit = ps;
      const size_t lds = mrp_host::lds_fwd<8>(cpb);
      const unsigned grid = (unsigned)(B * a.ncb * ps);
      snprintf(nm, sizeof nm, "film_fwd lpc=%d cpb=%d psplit=%d grid=%u", lpc, cpb, ps, grid);
      report(nm, time_ms([&] { hipLaunchKernelGGL((mrp::film_fwd<8, 4, true>), dim3(grid), dim3(lpc * cpb), lds, 0, a); }, iters), alg);
    }
  }
  {
    float *gout, *dx, *dgb;
    CK(hipMalloc(&gout, feat * 4));
    CK(hipMalloc(&dx, feat * 4));
    CK(hipMalloc(&dgb, (size_t)E * C * 2 * 4));
    CK(hipMemset(gout, 0, feat * 4));
    const double balg = (double)feat * 12 + (double)E * C * 2 * 4 * 2;
    report("product mrp_film_mean_bwd", time_ms([&] {
      CK((hipError_t)mrp_film_mean_bwd(gout, (int64_t)C * P, x, (int64_t)C * P, gb, nullptr, nullptr, nullptr, nullptr, B, N,
                                       MRP_GRAPH_COMPLETE, Nt, E, C, P, MRP_AGG_FILM_MEAN | MRP_AGG_GB_LOGITS, dx,
                                       (int64_t)C * P, nullptr, 0, dgb, nullptr));
    }, iters), balg);
    for (int lpc : {8, 16, 32, 64, 128, 256}) {
      if (lpc > P / 4) break;
      const int cpb = std::max(1, std::min(256 / lpc, 32));
      mrp::AggArgs a = {};
      a.x = x; a.xs = (int64_t)C * P; a.g = gout; a.gs = (int64_t)C * P; a.gb = gb; a.out = dx; a.os = (int64_t)C * P;
      a.dgb = dgb; a.C = C; a.P = P; a.PV = P / 4; a.mode = MRP_AGG_FILM_MEAN; a.logits = 1; a.lpc = lpc; a.cpb = cpb;
      a.ncb = (C + cpb - 1) / cpb; a.want_dx = 1; a.want_dgb = 1;
      const size_t lds = mrp_host::lds_bwd<8>(cpb, true, lpc);
      const unsigned grid = (unsigned)(B * a.ncb);
      snprintf(nm, sizeof nm, "film_bwd_fused lpc=%d cpb=%d grid=%u", lpc, cpb, grid);
      report(nm, time_ms([&] { hipLaunchKernelGGL((mrp::film_bwd_fused<8, 8, 4, true, false, 1>), dim3(grid), dim3(lpc * cpb), lds, 0, a); }, iters), balg);
    }
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  return 0;
}
