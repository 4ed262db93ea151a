// Kernel lab (not product code): the split-bf16 compress GEMMs (forward, data gradient, weight
// gradient) at the BASELINE config shapes through the library's C ABI, variant against variant
// (mrp_tuning_set knobs), checked element-wise against each other and on sampled outputs against a
// float64 host product, timed with hipEvents (median of rounds, variants interleaved per round).
//
// build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/gemm_lab.cpp -I include \
//        -L multi-robot-perception-gnn-1_amd/lib -lmrp_gnn -Wl,-rpath,'$ORIGIN/../multi-robot-perception-gnn-1_amd/lib' -o tools/bin/gemm_lab
// usage: gemm_lab [op fwd|dgrad|wgrad|all] [shape name|all] [variants "4,5"] [iters] [knob]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "mrp_gnn.h"

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                       \
    }                                                                                \
  } while (0)
#define CKL(x)                                                      \
  do {                                                              \
    int e_ = (x);                                                   \
    if (e_ != 0) {                                                  \
      fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, e_); \
      exit(3);                                                      \
    }                                                               \
  } while (0)

struct Shape {
  const char* name;
  int n, C, P;
};
static const Shape kShapes[] = {{"cfg1", 128, 512, 1024}, {"cfg2", 256, 1280, 64}, {"cfg3", 64, 2048, 64},
                                {"cfg4", 128, 1024, 256}, {"head", 256, 512, 1024}, {"small", 6, 256, 64}};

static float* dalloc_rand(size_t n, std::mt19937& rng, float scale, std::vector<float>* host) {
  std::vector<float> h(n);
  std::normal_distribution<float> d(0.f, 1.f);
  for (auto& v : h) v = d(rng) * scale;
  float* p;
  CK(hipMalloc(&p, n * 4));
  CK(hipMemcpy(p, h.data(), n * 4, hipMemcpyHostToDevice));
  if (host) *host = std::move(h);
  return p;
}

int main(int argc, char** argv) {
  std::string op = argc > 1 ? argv[1] : "all";
  std::string shp = argc > 2 ? argv[2] : "all";
  std::string vs = argc > 3 ? argv[3] : "4,5";
  int iters = argc > 4 ? atoi(argv[4]) : 10;
  const char* knob = argc > 5 ? argv[5] : "gemm_split";
  std::vector<int> variants;
  for (size_t i = 0; i < vs.size();) {
    size_t j = vs.find(',', i);
    if (j == std::string::npos) j = vs.size();
    variants.push_back(atoi(vs.substr(i, j - i).c_str()));
    i = j + 1;
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  bool all_ok = true;
  for (const Shape& s : kShapes) {
    if (shp != "all" && shp != s.name) continue;
    if (shp == "all" && std::string(s.name) == "small") continue;
    const int n = s.n, C = s.C, P = s.P;
    const size_t plane = (size_t)n * C * P;
    std::mt19937 rng(1234);
    std::vector<float> hx, ha, hw, hb, hg;
    float* x = dalloc_rand(plane, rng, 1.f, &hx);
    float* a = dalloc_rand(plane, rng, 1.f, &ha);
    float* gy = dalloc_rand(plane, rng, 1.f, &hg);
    float* w = dalloc_rand((size_t)C * 2 * C, rng, 1.f / std::sqrt(2.f * C), &hw);
    float* b = dalloc_rand(C, rng, 1.f, &hb);
    float *y, *gx, *ga, *gw, *gb;
    CK(hipMalloc(&y, plane * 4));
    CK(hipMalloc(&gx, plane * 4));
    CK(hipMalloc(&ga, plane * 4));
    CK(hipMalloc(&gw, (size_t)C * 2 * C * 4));
    CK(hipMalloc(&gb, (size_t)C * 4));
    void *pf, *pb;
    CK(hipMalloc(&pf, mrp_compress_split_pack_bytes(C, 2 * C)));
    CK(hipMalloc(&pb, mrp_compress_split_pack_bytes(2 * C, C)));
    CKL(mrp_compress_split_pack(w, 2 * C, 0, C, 2 * C, pf, st));
    CKL(mrp_compress_split_pack(w, 2 * C, 1, 2 * C, C, pb, st));
    int64_t wsb = mrp_compress_bwd_weight_split_workspace(n, C, P);
    void* ws = nullptr;
    if (wsb > 0) CK(hipMalloc(&ws, wsb));
    const double flop = 2.0 * C * 2.0 * C * (double)n * P;
    for (const char* o : {"fwd", "dgrad", "wgrad"}) {
      if (op != "all" && op != o) continue;
      auto run = [&]() {
        if (!strcmp(o, "fwd"))
          CKL(mrp_compress_fwd_split(x, (int64_t)C * P, a, (int64_t)C * P, n, C, P, pf, b, y, (int64_t)C * P, st));
        else if (!strcmp(o, "dgrad"))
          CKL(mrp_compress_bwd_data_split(gy, (int64_t)C * P, n, C, P, pb, gx, (int64_t)C * P, ga, (int64_t)C * P, st));
        else
          CKL(mrp_compress_bwd_weight_split(gy, (int64_t)C * P, x, (int64_t)C * P, a, (int64_t)C * P, n, C, P, gw, gb,
                                            ws, wsb, st));
      };
      // outputs per variant for cross-checks
      std::vector<std::vector<float>> outs;
      std::vector<std::vector<double>> times(variants.size());
      for (size_t vi = 0; vi < variants.size(); ++vi) {
        CKL(mrp_tuning_set(knob, variants[vi]));
        run();
        CK(hipStreamSynchronize(st));
        std::vector<float> h;
        if (!strcmp(o, "fwd")) {
          h.resize(plane);
          CK(hipMemcpy(h.data(), y, plane * 4, hipMemcpyDeviceToHost));
        } else if (!strcmp(o, "dgrad")) {
          h.resize(2 * plane);
          CK(hipMemcpy(h.data(), gx, plane * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h.data() + plane, ga, plane * 4, hipMemcpyDeviceToHost));
        } else {
          h.resize((size_t)C * 2 * C + C);
          CK(hipMemcpy(h.data(), gw, (size_t)C * 2 * C * 4, hipMemcpyDeviceToHost));
          CK(hipMemcpy(h.data() + (size_t)C * 2 * C, gb, C * 4, hipMemcpyDeviceToHost));
        }
        outs.push_back(std::move(h));
      }
      // float64 reference on sampled outputs
      std::mt19937 srng(99);
      double max_err[16] = {0}, max_ref = 0;
      const int NS = 256;
      for (int t = 0; t < NS; ++t) {
        double ref;
        size_t idx;
        if (!strcmp(o, "fwd")) {
          int nd = srng() % n, m = srng() % C, px = srng() % P;
          ref = hb[m];
          for (int k = 0; k < 2 * C; ++k) {
            const float* src = k < C ? &hx[((size_t)nd * C + k) * P + px] : &ha[((size_t)nd * C + (k - C)) * P + px];
            ref += (double)hw[(size_t)m * 2 * C + k] * *src;
          }
          idx = ((size_t)nd * C + m) * P + px;
        } else if (!strcmp(o, "dgrad")) {
          int nd = srng() % n, m = srng() % (2 * C), px = srng() % P;
          ref = 0;
          for (int k = 0; k < C; ++k) ref += (double)hw[(size_t)k * 2 * C + m] * hg[((size_t)nd * C + k) * P + px];
          idx = m < C ? ((size_t)nd * C + m) * P + px : plane + ((size_t)nd * C + (m - C)) * P + px;
        } else {
          int m = srng() % C, c2 = srng() % (2 * C);
          ref = 0;
          for (int nd = 0; nd < n; ++nd)
            for (int px = 0; px < P; ++px) {
              const double g = hg[((size_t)nd * C + m) * P + px];
              const double sv = c2 < C ? hx[((size_t)nd * C + c2) * P + px] : ha[((size_t)nd * C + c2 - C) * P + px];
              ref += g * sv;
            }
          idx = (size_t)m * 2 * C + c2;
        }
        max_ref = std::max(max_ref, std::fabs(ref));
        for (size_t vi = 0; vi < variants.size(); ++vi)
          max_err[vi] = std::max(max_err[vi], std::fabs((double)outs[vi][idx] - ref));
      }
      // element-wise against the first variant
      std::vector<double> dmax(variants.size(), 0.0);
      for (size_t vi = 1; vi < variants.size(); ++vi)
        for (size_t i = 0; i < outs[0].size(); ++i)
          dmax[vi] = std::max(dmax[vi], (double)std::fabs(outs[vi][i] - outs[0][i]));
      // timing: rounds, variants interleaved
      for (int r = 0; r < 5; ++r)
        for (size_t vi = 0; vi < variants.size(); ++vi) {
          CKL(mrp_tuning_set(knob, variants[vi]));
          run();
          CK(hipEventRecord(e0, st));
          for (int i = 0; i < iters; ++i) run();
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          times[vi].push_back(ms * 1e-3 / iters);
        }
      for (size_t vi = 0; vi < variants.size(); ++vi) {
        auto t = times[vi];
        std::sort(t.begin(), t.end());
        const double rel = max_err[vi] / max_ref;
        const bool ok = rel < 2e-6;
        all_ok = all_ok && ok;
        printf("%-5s %-6s n=%d C=%d P=%d  %s=%d  %8.1f us (min %8.1f)  %6.1f TF/s  f64 err %.2e  vs v0 %.2e %s\n", s.name,
               o, n, C, P, knob, variants[vi], t[2] * 1e6, t[0] * 1e6, flop / t[2] / 1e12, rel, dmax[vi] / max_ref,
               ok ? "" : "FAIL");
        fflush(stdout);
      }
    }
    CKL(mrp_tuning_set(knob, -1));
    for (void* p : {(void*)x, (void*)a, (void*)gy, (void*)w, (void*)b, (void*)y, (void*)gx, (void*)ga, (void*)gw,
                    (void*)gb, pf, pb})
      CK(hipFree(p));
    if (ws) CK(hipFree(ws));
  }
  printf(all_ok ? "ALL OK\n" : "SOME FAIL\n");
  return all_ok ? 0 : 1;
}
