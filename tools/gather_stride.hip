// gather_stride.hip — kernel lab (not product code): does film_fwd's gather pattern (each thread reads
// one 16-byte slice of all N node planes and writes N slices) lose bandwidth to the node planes being
// a power-of-two distance apart (C H W 4 = 2 MiB at the headline)?  Times the gather at the headline
// size with the node stride exact and padded by 256 B .. 64 KiB, HIP graph over rotating buffer sets
// (> 2 x the 256 MB Infinity Cache), best of 3 replays.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_stride.hip -o tools/bin/gather_stride
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
constexpr int NT = 8;

// thread = one 16-byte slice of one (graph, channel plane); node u's plane at u * stride4
__global__ void __launch_bounds__(256) gather8(const f4* __restrict__ in, f4* __restrict__ out, size_t stride4,
                                               size_t items) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  const size_t g = t / items, r = t - g * items;
  const f4* src = in + g * NT * stride4 + r;
  f4* dst = out + g * NT * stride4 + r;
  f4 v[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(src + u * stride4);
#pragma unroll
  for (int w = 0; w < NT; ++w) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NT; ++u)
      if (u != w) acc += v[u];
    __builtin_nontemporal_store(acc, dst + w * stride4);
  }
}

// the same, with the node order rotated per 8-lane group (lanes 8g .. 8g + 7 load node (k + g) mod 8
// with their k-th load and store node (w + g) mod 8 k-th): every load / store instruction of a wave
// touches 8 node planes (128 B each) instead of one 1 KiB run of one plane
__global__ void __launch_bounds__(256) gather8_rot(const f4* __restrict__ in, f4* __restrict__ out, size_t stride4,
                                                   size_t items) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  const size_t g = t / items, r = t - g * items;
  const int rot = (threadIdx.x >> 3) & 7;
  const f4* src = in + g * NT * stride4 + r;
  f4* dst = out + g * NT * stride4 + r;
  f4 v[NT];
#pragma unroll
  for (int k = 0; k < NT; ++k) v[k] = __builtin_nontemporal_load(src + ((k + rot) & 7) * stride4);
#pragma unroll
  for (int w = 0; w < NT; ++w) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < NT; ++k)
      if (k != w) acc += v[k];
    __builtin_nontemporal_store(acc, dst + ((w + rot) & 7) * stride4);
  }
}

// the plain gather with the workgroup order scattered: block b works on block (b * 40503) mod nblocks,
// so the workgroups resident together touch offsets spread over the whole tensor
__global__ void __launch_bounds__(256) gather8_scatter(const f4* __restrict__ in, f4* __restrict__ out,
                                                       size_t stride4, size_t items) {
  const size_t blk = ((size_t)blockIdx.x * 40503u) % gridDim.x;
  const size_t t = blk * (size_t)256 + threadIdx.x;
  const size_t g = t / items, r = t - g * items;
  const f4* src = in + g * NT * stride4 + r;
  f4* dst = out + g * NT * stride4 + r;
  f4 v[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(src + u * stride4);
#pragma unroll
  for (int w = 0; w < NT; ++w) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NT; ++u)
      if (u != w) acc += v[u];
    __builtin_nontemporal_store(acc, dst + w * stride4);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 40;
  const long B = 32, C = 512, HW = 32;
  const size_t items = (size_t)C * HW * HW / 4;  // float4 per node plane set
  const size_t pads[] = {0, 64, 256, 1024, 4096};  // in float4 (0, 1 KiB, 4 KiB, 16 KiB, 64 KiB)
  for (int rotv = 0; rotv < 3; ++rotv)
  for (size_t pad : pads) {
    if (rotv && pad > 64) continue;
    const size_t stride4 = items + pad;
    const size_t bytes_alloc = (size_t)B * NT * stride4 * 16;
    const int nsets = (int)((((size_t)600 << 20) + 2 * bytes_alloc - 1) / (2 * bytes_alloc));
    std::vector<void*> bufs(2 * nsets);
    for (auto& p : bufs) {
      CK(hipMalloc(&p, bytes_alloc));
      CK(hipMemset(p, 0, bytes_alloc));
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    const unsigned grid = (unsigned)((B * items + 255) / 256);
    auto launch = [&](int i) {
      const int s = i % nsets;
      if (rotv == 2)
        hipLaunchKernelGGL(gather8_scatter, dim3(grid), dim3(256), 0, st, (const f4*)bufs[2 * s], (f4*)bufs[2 * s + 1],
                           stride4, items);
      else if (rotv)
        hipLaunchKernelGGL(gather8_rot, dim3(grid), dim3(256), 0, st, (const f4*)bufs[2 * s], (f4*)bufs[2 * s + 1],
                           stride4, items);
      else
        hipLaunchKernelGGL(gather8, dim3(grid), dim3(256), 0, st, (const f4*)bufs[2 * s], (f4*)bufs[2 * s + 1], stride4,
                           items);
    };
    for (int i = 0; i < 200; ++i) launch(i);  // clocks up
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
    const double us = best * 1e3 / iters;
    const double bytes = 2.0 * B * NT * items * 16;
    printf("%s node stride = plane + %6zu B: %7.2f us  %5.1f %% of 8 TB/s (%d sets)\n", rotv == 2 ? "scatter" : rotv ? "rotated" : "plain  ", pad * 16, us,
           bytes / (us * 1e-6) / 8e12 * 100, nsets);
    fflush(stdout);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    CK(hipStreamDestroy(st));
    for (auto p : bufs) CK(hipFree(p));
  }
  return 0;
}
