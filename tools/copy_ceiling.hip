// copy_ceiling.hip — kernel lab (not product code): the streaming ceiling of MI355X at the byte counts
// and read/write mixes of the aggregation kernels at every BASELINE config shape, timed the way
// bench.py times the product kernels (a HIP graph of `iters` launches over rotating buffer sets whose
// footprint exceeds 2 x the 256 MB Infinity Cache, one event pair around the replay).
//   forward mix:  read R, write W (R ~ W)          -> out[i] = in[i]
//   backward mix: read 2W, write W                  -> out[i] = a[i] + b[i]
// and each mix in the aggregation kernels' gather pattern (gather_nt, gather2_nt).
// Kernels: grid-stride float4, nontemporal, 256 threads, one float4 per thread per trip, grid sized
// to the element count (best of the round-1 copy sweep).  Prints us and the fraction of 8 TB/s.
// Build: hipcc --offload-arch=gfx950 -O3 tools/copy_ceiling.hip -o tools/bin/copy_ceiling
#include <hip/hip_runtime.h>

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

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy1(const f4* __restrict__ in, f4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

__global__ void __launch_bounds__(256) add2(const f4* __restrict__ a, const f4* __restrict__ b, f4* __restrict__ out,
                                            size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i) + __builtin_nontemporal_load(b + i), out + i);
}

// film_fwd's data movement without its prologue: thread = one 16-byte slice of one channel plane of
// one graph; it reads that slice of all NT nodes (planes node_stride apart) and writes NT slices
// (here: each output the sum of the other nodes' slices).  Grid = graphs x channels x slices.
template <int NT>
__global__ void __launch_bounds__(256) gather_nt(const f4* __restrict__ in, f4* __restrict__ out, size_t node_stride4,
                                                 size_t graph_items) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;  // (graph, c, slice) within a graph's plane set
  const size_t g = t / graph_items, r = t - g * graph_items;
  const f4* src = in + g * NT * node_stride4 + r;
  f4* dst = out + g * NT * node_stride4 + r;
  f4 v[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(src + u * node_stride4);
#pragma unroll
  for (int w = 0; w < NT; ++w) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NT; ++u)
      if (u != w) acc += v[u];
    __builtin_nontemporal_store(acc, dst + w * node_stride4);
  }
}

// film_bwd_fused's data movement without its Gram, reduction and epilogue: thread = one 16-byte slice;
// it reads that slice of all NT nodes of grad_out AND of x, and writes NT slices of grad_x (each the
// sum of the other nodes' grad_out slices plus its own x slice, so every load is used).
template <int NT>
__global__ void __launch_bounds__(256) gather2_nt(const f4* __restrict__ g, const f4* __restrict__ x,
                                                  f4* __restrict__ out, size_t node_stride4, size_t graph_items) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  const size_t gi = t / graph_items, r = t - gi * graph_items;
  const size_t base = gi * NT * node_stride4 + r;
  f4 v[NT], w[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(g + base + u * node_stride4);
#pragma unroll
  for (int u = 0; u < NT; ++u) w[u] = __builtin_nontemporal_load(x + base + u * node_stride4);
#pragma unroll
  for (int k = 0; k < NT; ++k) {
    f4 acc = w[k];
#pragma unroll
    for (int u = 0; u < NT; ++u)
      if (u != k) acc += v[u];
    __builtin_nontemporal_store(acc, out + base + k * node_stride4);
  }
}

template <int NT>
static double time_gather(int nsets, int iters, const std::vector<void*>& bufs, size_t n4, size_t node4,
                          bool bwd = false) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t graph_items = node4;  // per graph: (channel, slice) items = float4 of one node
  const unsigned grid = (unsigned)((n4 / NT + 255) / 256);
  auto launch = [&](int i) {
    const int s = i % nsets;
    if (bwd)
      hipLaunchKernelGGL(gather2_nt<NT>, dim3(grid), dim3(256), 0, st, (const f4*)bufs[3 * s],
                         (const f4*)bufs[3 * s + 1], (f4*)bufs[3 * s + 2], node4, node4);
    else
      hipLaunchKernelGGL(gather_nt<NT>, dim3(grid), dim3(256), 0, st, (const f4*)bufs[3 * s], (f4*)bufs[3 * s + 2],
                         node4, node4);
  };
  (void)graph_items;
  for (int i = 0; i < 2 * nsets; ++i) launch(i);
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(st));
  return best * 1e3 / iters;
}

static double time_graph(int nsets, int iters, const std::vector<void*>& bufs, size_t n4, bool bwd) {
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const unsigned grid = (unsigned)((n4 + 255) / 256);
  auto launch = [&](int i) {
    const int s = i % nsets;
    if (bwd)
      hipLaunchKernelGGL(add2, dim3(grid), dim3(256), 0, st, (const f4*)bufs[3 * s], (const f4*)bufs[3 * s + 1],
                         (f4*)bufs[3 * s + 2], n4);
    else
      hipLaunchKernelGGL(copy1, dim3(grid), dim3(256), 0, st, (const f4*)bufs[3 * s], (f4*)bufs[3 * s + 2], n4);
  };
  for (int i = 0; i < 2 * nsets; ++i) launch(i);  // warm
  CK(hipStreamSynchronize(st));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeGlobal));
  for (int i = 0; i < iters; ++i) launch(i);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(st));
  return best * 1e3 / iters;  // us per launch
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  struct Shape {
    const char* name;
    long B, N, C, HW;
  } shapes[] = {{"north_star", 32, 8, 512, 32}, {"cfg1", 16, 8, 512, 32}, {"cfg2", 32, 8, 1280, 8},
                {"cfg3", 8, 8, 2048, 8}, {"cfg4", 8, 16, 1024, 16}};
  // spin the clocks up first
  {
    std::vector<void*> b(3);
    const size_t n4 = (size_t)64 << 20;
    for (auto& p : b) CK(hipMalloc(&p, n4 * 16));
    for (int i = 0; i < 3; ++i) time_graph(1, 200, b, n4, false);
    for (auto p : b) CK(hipFree(p));
  }
  for (const Shape& s : shapes) {
    const size_t plane_bytes = (size_t)s.B * s.N * s.C * s.HW * s.HW * 4;
    const size_t n4 = plane_bytes / 16;
    for (int bwd = 0; bwd < 2; ++bwd) {
      const size_t set_bytes = plane_bytes * (bwd ? 3 : 2);
      int nsets = (int)((((size_t)600 << 20) + set_bytes - 1) / set_bytes);
      if (nsets < 1) nsets = 1;
      std::vector<void*> bufs(3 * nsets, nullptr);
      for (int i = 0; i < nsets; ++i)
        for (int k = 0; k < 3; ++k)
          if (bwd || k != 1) CK(hipMalloc(&bufs[3 * i + k], plane_bytes));
      const double us = time_graph(nsets, iters, bufs, n4, bwd);
      const double bytes = (double)plane_bytes * (bwd ? 3 : 2);
      printf("%-10s %s %8.1f MB  %8.2f us  %5.1f %% of 8 TB/s  (%d rotating sets)\n", s.name, bwd ? "2r1w" : "1r1w",
             bytes / 1e6, us, bytes / (us * 1e-6) / 8e12 * 100, nsets);
      {  // the aggregation's gather pattern: N node planes per thread (forward: of x; backward: of
         // grad_out and x), N outputs
        const size_t node4 = (size_t)s.C * s.HW * s.HW / 4;
        const double ug = s.N == 8 ? time_gather<8>(nsets, iters, bufs, n4, node4, bwd)
                                   : time_gather<16>(nsets, iters, bufs, n4, node4, bwd);
        printf("%-10s %s%ld %8.1f MB  %8.2f us  %5.1f %% of 8 TB/s\n", s.name, bwd ? "gather_bwd" : "gather", s.N,
               bytes / 1e6, ug, bytes / (ug * 1e-6) / 8e12 * 100);
      }
      fflush(stdout);
      for (auto p : bufs)
        if (p) CK(hipFree(p));
    }
  }
  return 0;
}
