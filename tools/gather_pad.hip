// gather_pad.hip — kernel lab (not product code): does the node stride of the (node, C, H, W) layout set
// the aggregation forward's streaming ceiling?  film_fwd's data movement (copy_ceiling.hip gather_nt:
// a thread reads one 16-byte slice of all 8 nodes of its graph, planes node_stride apart, and writes 8)
// at the headline size (B = 32, N = 8, C = 512, 32 x 32: node stride 2 MiB) with the input and/or the
// output node stride padded by `pad` bytes, against the plain 1r1w copy of the same bytes; HIP-graph
// timed over rotating buffer sets like bench.py; also the gather split over two lanes and a persistent
// pipelined gather.  Prints us per launch.
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_pad.hip -o tools/bin/gather_pad
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                 \
    }                                                                                          \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int NT = 8;

__global__ void __launch_bounds__(256) copy1(const f4* __restrict__ in, f4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

// thread = (graph, slice r of a node's C*P floats); in / out node strides (float4 units) si / so
__global__ void __launch_bounds__(256) gather(const f4* __restrict__ in, f4* __restrict__ out, size_t items,
                                              size_t si, size_t so, size_t total) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  if (t >= total) return;
  const size_t g = t / items, r = t - g * items;
  const f4* src = in + g * NT * si + r;
  f4* dst = out + g * NT * so + r;
  f4 v[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(src + u * si);
#pragma unroll
  for (int w = 0; w < NT; ++w) {
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < NT; ++u)
      if (u != w) acc += v[u];
    __builtin_nontemporal_store(acc, dst + w * so);
  }
}

// the same bytes with each slice's 8 nodes split over two lanes (lanes 0-31: nodes 0-3, lanes 32-63:
// nodes 4-7 of the same 32 slices): each lane loads 4 planes, forms the partial sums of all 8 outputs
// over its nodes, swaps the 4 its partner writes (__shfl_xor 32) and stores 4 planes
__global__ void __launch_bounds__(256) gather_half(const f4* __restrict__ in, f4* __restrict__ out, size_t items,
                                                   size_t si, size_t so, size_t total) {
  const size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const size_t slice = (t >> 6) * 32 + (lane & 31);  // 32 slices per wave
  if (slice >= total) return;
  const size_t g = slice / items, r = slice - g * items;
  const f4* src = in + g * NT * si + r;
  f4* dst = out + g * NT * so + r;
  f4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(src + (4 * h + u) * si);
  f4 mine[4], theirs[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    f4 pm = {0.f, 0.f, 0.f, 0.f}, po = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u != w) pm += v[u];  // my outputs 4 h + w: my nodes except w
      po += v[u];              // the partner's outputs: all my nodes
    }
    mine[w] = pm;
    theirs[w] = po;
  }
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    f4 rcv;
#pragma unroll
    for (int k = 0; k < 4; ++k) rcv[k] = __shfl_xor(theirs[w][k], 32, 64);
    __builtin_nontemporal_store(mine[w] + rcv, dst + (4 * h + w) * so);
  }
}

// persistent grid-stride gather, the next slice's 8 planes requested before the current slice's
// outputs are formed and stored (two register sets)
__global__ void __launch_bounds__(256) gather_pipe(const f4* __restrict__ in, f4* __restrict__ out, size_t items,
                                                   size_t si, size_t total) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t t = blockIdx.x * (size_t)256 + threadIdx.x;
  if (t >= total) return;
  auto base = [&](size_t tt) { const size_t g = tt / items; return g * NT * si + (tt - g * items); };
  f4 v[NT], nv[NT];
  size_t b = base(t);
#pragma unroll
  for (int u = 0; u < NT; ++u) v[u] = __builtin_nontemporal_load(in + b + u * si);
  while (true) {
    const size_t tn = t + stride;
    const bool more = tn < total;
    const size_t bn = more ? base(tn) : b;
    if (more) {
#pragma unroll
      for (int u = 0; u < NT; ++u) nv[u] = __builtin_nontemporal_load(in + bn + u * si);
    }
#pragma unroll
    for (int w = 0; w < NT; ++w) {
      f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < NT; ++u)
        if (u != w) acc += v[u];
      __builtin_nontemporal_store(acc, out + b + w * si);
    }
    if (!more) break;
#pragma unroll
    for (int u = 0; u < NT; ++u) v[u] = nv[u];
    t = tn;
    b = bn;
  }
}

template <class F>
static double time_it(hipStream_t st, int iters, F launch) {
  for (int i = 0; i < 8; ++i) launch(i);
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
  return best * 1e3 / iters;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20;
  const size_t B = 32, C = 512, P = 1024;
  const size_t node4 = C * P / 4;  // float4 per node
  const size_t items = node4, total = B * items;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const long pads[] = {0};
  const size_t maxpad4 = (1 << 20) / 16;
  const size_t cap4 = B * NT * (node4 + maxpad4);
  const int nsets = 2;  // 2 x (in + out) x 1.1 GB > 2 x the 256 MB Infinity Cache
  std::vector<f4*> in(nsets), out(nsets);
  for (int s = 0; s < nsets; ++s) {
    CK(hipMalloc(&in[s], cap4 * 16));
    CK(hipMalloc(&out[s], cap4 * 16));
    CK(hipMemset(in[s], 0, cap4 * 16));
  }
  const unsigned grid_g = (unsigned)((total + 255) / 256);
  const size_t n4 = B * NT * node4;
  for (int rep = 0; rep < 2; ++rep) {
    const double tc = time_it(st, iters, [&](int i) {
      hipLaunchKernelGGL(copy1, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, in[i % nsets], out[i % nsets], n4);
    });
    printf("copy 1r1w                      %8.2f us\n", tc);
    {
      const unsigned grid_h = (unsigned)((2 * total + 255) / 256);
      const double th = time_it(st, iters, [&](int i) {
        hipLaunchKernelGGL(gather_half, dim3(grid_h), dim3(256), 0, st, in[i % nsets], out[i % nsets], items, node4,
                           node4, total);
      });
      printf("gather8 split over 2 lanes     %8.2f us\n", th);
    }
    for (int wpc : {4, 8, 16}) {  // persistent: workgroups per CU
      const double tp = time_it(st, iters, [&](int i) {
        hipLaunchKernelGGL(gather_pipe, dim3(256 * wpc), dim3(256), 0, st, in[i % nsets], out[i % nsets], items, node4,
                           total);
      });
      printf("gather8 persistent, %2d wg/CU   %8.2f us\n", wpc, tp);
    }
    for (long pad : pads) {
      for (int which = 0; which < 3; ++which) {  // 0: both padded, 1: input only, 2: output only
        if (pad == 0 && which) continue;
        const size_t si = node4 + ((which == 0 || which == 1) ? pad / 16 : 0);
        const size_t so = node4 + ((which == 0 || which == 2) ? pad / 16 : 0);
        const double t = time_it(st, iters, [&](int i) {
          hipLaunchKernelGGL(gather, dim3(grid_g), dim3(256), 0, st, in[i % nsets], out[i % nsets], items, si, so, total);
        });
        printf("gather8 pad %8ld B (%s) %8.2f us\n", pad, which == 0 ? "in+out" : (which == 1 ? "in    " : "out   "), t);
        fflush(stdout);
      }
    }
  }
  return 0;
}
