// kernel_lab.hip — timing lab for the FiLM-mean forward on MI355X (not product code).
//
// Builds the north-star workload (B graphs x N robots, complete graphs, C x H x W fp32) and times
// the product kernel against bandwidth references with HIP events:
//   stream_copy   : grid-stride float4 copy of the same byte count (read Nt*C*P, write Nt*C*P)
//   plane_copy<N> : the product's lane mapping with out_v = x_v (no prologue, no math)
//   film_fwd<N,4> : the product kernel at several (lanes-per-channel, channels-per-block) geometries
// Usage: kernel_lab [B N C HW iters]
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

template <typename T>
__global__ void __launch_bounds__(256) stream_copy(const T* __restrict__ in, T* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) out[i] = in[i];
}

template <int NT>
__global__ void __launch_bounds__(256) plane_copy(mrp::AggArgs a) {
  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = a.goff[b];
  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = cb * a.cpb + grp;
  if (c >= a.C) return;
  const float* xb = a.x + (int64_t)node0 * a.xs + (int64_t)c * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
  for (int j = li; j < a.PV; j += a.lpc) {
    f4 v[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) v[u] = *reinterpret_cast<const f4*>(xb + (int64_t)u * a.xs + j * 4);
#pragma unroll
    for (int u = 0; u < NT; ++u) *reinterpret_cast<f4*>(ob + (int64_t)u * a.os + j * 4) = v[u];
  }
}

// ---- ablation variants of the forward (lab copies of mrp::film_fwd) ----
// PRO: build LDS tiles (else constant weights); MATH: FiLM math (else copy x_v);
// NTL: nontemporal loads/stores; PERSIST: grid-stride over (graph, channel block) items.
template <int NT, bool PRO, bool MATH, bool NTL, bool PERSIST>
__global__ void __launch_bounds__(256) fwd_var(mrp::AggArgs a, int items) {
  constexpr int SZ = mrp::Tile<NT>::SZ;
  constexpr int NTP = mrp::Tile<NT>::NTP;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Ga = smem;
  float* Gb = Ga + a.cpb * SZ;
  float* degf = Gb + a.cpb * SZ;
  unsigned* emask = reinterpret_cast<unsigned*>(degf + NTP);
  for (int item = blockIdx.x; item < items; item += (PERSIST ? gridDim.x : items)) {
    const int b = item / a.ncb;
    const int cb = item - b * a.ncb;
    const int node0 = a.goff[b];
    const int n = min(a.goff[b + 1] - node0, NT);
    const int c0 = cb * a.cpb;
    if (PRO) {
      if (PERSIST) __syncthreads();
      mrp::build_tiles_csr<NT, false>(a, node0, n, c0, Ga, Gb, degf, emask);
      __syncthreads();
    }
    const int grp = threadIdx.x / a.lpc;
    const int li = threadIdx.x - grp * a.lpc;
    const int c = c0 + grp;
    if (c >= a.C) continue;
    const float* xb = a.x + (int64_t)node0 * a.xs + (int64_t)c * a.P;
    float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
    const float* A = Ga + grp * SZ;
    const float* Bt = Gb + grp * SZ;
    for (int j = li; j < a.PV; j += a.lpc) {
      const int64_t off = (int64_t)j * 4;
      f4 xv[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const f4* p = reinterpret_cast<const f4*>(xb + (int64_t)u * a.xs + off);
        xv[u] = NTL ? __builtin_nontemporal_load(p) : *p;
      }
#pragma unroll
      for (int v = 0; v < NT; ++v) {
        f4 acc;
        if (MATH) {
          const unsigned em = PRO ? __builtin_amdgcn_readfirstlane(emask[v]) : (0xffu & ~(1u << v));
          acc = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            if (!((em >> u) & 1u)) continue;
            const float ga = PRO ? A[v * NTP + u] : 0.5f;
            const float gbv = PRO ? Bt[v * NTP + u] : 0.25f;
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = __fadd_rn(acc[k], __fadd_rn(__fmul_rn(ga, xv[u][k]), gbv));
          }
          const float d = PRO ? degf[v] : 7.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) acc[k] = acc[k] / d;
        } else {
          acc = xv[v];
        }
        f4* q = reinterpret_cast<f4*>(ob + (int64_t)v * a.os + off);
        if (NTL) __builtin_nontemporal_store(acc, q); else *q = acc;
      }
    }
  }
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
  const int KNN = argc > 6 ? atoi(argv[6]) : 0;  // 0: complete graphs; k: k in-edges per node (CSR path)
  const int P = HW * HW;
  const int Nt = B * N;
  const int E = KNN ? B * N * KNN : B * N * (N - 1);
  std::vector<int> indptr(Nt + 1), src(E), eid(E), goff(B + 1);
  int k = 0;
  for (int b = 0; b < B; ++b) {
    goff[b] = b * N;
    for (int v = 0; v < N; ++v) {
      indptr[b * N + v] = k;
      if (KNN) {
        // k sources per destination, ascending local ids (a k-NN-shaped graph), edge ids = CSR order
        std::vector<int> us;
        for (int i = 1; i <= KNN; ++i) us.push_back((v + i) % N);
        std::sort(us.begin(), us.end());
        for (int u : us) { src[k] = b * N + u; eid[k] = k; ++k; }
      } else {
        // complete i-major graphs, CSR by destination
        for (int u = 0; u < N; ++u) {
          if (u == v) continue;
          src[k] = b * N + u;
          eid[k] = b * N * (N - 1) + u * (N - 1) + (v < u ? v : v - 1);
          ++k;
        }
      }
    }
  }
  indptr[Nt] = k;
  goff[B] = Nt;
  const size_t feat = (size_t)Nt * C * P;
  float *x, *out, *gb, *gout;
  int *d_indptr, *d_src, *d_eid, *d_goff;
  CK(hipMalloc(&x, feat * 4));
  CK(hipMalloc(&gout, feat * 4));  // backward's grad_out: its own buffer (aliasing x would hit cache)
  CK(hipMalloc(&out, feat * 4));
  CK(hipMalloc(&gb, (size_t)E * C * 2 * 4));
  CK(hipMalloc(&d_indptr, (Nt + 1) * 4));
  CK(hipMalloc(&d_src, E * 4));
  CK(hipMalloc(&d_eid, E * 4));
  CK(hipMalloc(&d_goff, (B + 1) * 4));
  CK(hipMemcpy(d_indptr, indptr.data(), (Nt + 1) * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_src, src.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_eid, eid.data(), E * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_goff, goff.data(), (B + 1) * 4, hipMemcpyHostToDevice));
  {
    std::vector<float> h(feat);
    for (size_t i = 0; i < feat; ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(x, h.data(), feat * 4, hipMemcpyHostToDevice));
    for (size_t i = 0; i < feat; ++i) h[i] = (float)((i * 97u) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(gout, h.data(), feat * 4, hipMemcpyHostToDevice));
    std::vector<float> hg((size_t)E * C * 2);
    for (size_t i = 0; i < hg.size(); ++i) hg[i] = (float)((i * 40503u) % 1000) / 1000.f;
    CK(hipMemcpy(gb, hg.data(), hg.size() * 4, hipMemcpyHostToDevice));
  }
  const double alg = (double)feat * 8 + (double)E * C * 2 * 4;
  printf("workload B=%d N=%d C=%d %dx%d %s: alg bytes %.1f MB\n", B, N, C, HW, HW, KNN ? "knn" : "complete",
         alg / 1e6);
  auto report = [&](const char* name, float ms, double bytes) {
    printf("%-40s %9.1f us  %7.0f GB/s  %5.1f%% of 8 TB/s\n", name, ms * 1e3, bytes / ms / 1e6,
           bytes / ms / 1e6 / 80.0);
  };
  {
    const size_t n4 = feat / 4;
    for (int grid : {1024, 2048, 4096, 8192}) {
      char nm[64];
      snprintf(nm, sizeof nm, "stream_copy f4 grid=%d", grid);
      float ms = time_ms([&] { hipLaunchKernelGGL(lab::stream_copy<mrp::f4>, dim3(grid), dim3(256), 0, 0,
                                                  (const mrp::f4*)x, (mrp::f4*)out, n4); }, iters);
      report(nm, ms, (double)feat * 8);
      snprintf(nm, sizeof nm, "stream_copy f2 grid=%d", grid);
      ms = time_ms([&] { hipLaunchKernelGGL(lab::stream_copy<mrp::f2>, dim3(grid), dim3(256), 0, 0,
                                            (const mrp::f2*)x, (mrp::f2*)out, n4 * 2); }, iters);
      report(nm, ms, (double)feat * 8);
    }
  }
  auto args_for = [&](int lpc, int cpb) {
    mrp::AggArgs a = {};
    a.x = x; a.xs = (int64_t)C * P; a.gb = gb; a.indptr = d_indptr; a.src = d_src; a.eid = d_eid; a.goff = d_goff;
    a.out = out; a.os = (int64_t)C * P; a.C = C; a.P = P; a.PV = P / 4; a.mode = 0; a.lpc = lpc; a.cpb = cpb;
    a.ncb = (C + cpb - 1) / cpb;
    return a;
  };
  if (N == 8 && !KNN) {
    for (int lpc : {64, 32, 16}) {
      for (int cpb : {4, 8, 16}) {
        if (lpc * cpb > 256 || lpc * cpb < 64) continue;
        mrp::AggArgs a = args_for(lpc, cpb);
        const int grid = B * a.ncb, thr = lpc * cpb;
        char nm[64];
        snprintf(nm, sizeof nm, "plane_copy<8> lpc=%d cpb=%d", lpc, cpb);
        float ms = time_ms([&] { hipLaunchKernelGGL(lab::plane_copy<8>, dim3(grid), dim3(thr), 0, 0, a); }, iters);
        report(nm, ms, (double)feat * 8);
        snprintf(nm, sizeof nm, "film_fwd<8,4,complete> lpc=%d cpb=%d", lpc, cpb);
        const size_t lds = (size_t)(2 * cpb * mrp::Tile<8>::SZ + 2 * mrp::Tile<8>::NTP) * 4;
        ms = time_ms([&] { hipLaunchKernelGGL((mrp::film_fwd<8, 4, true>), dim3(grid), dim3(thr), lds, 0, a); }, iters);
        report(nm, ms, alg);
      }
    }
  }

  if (N == 8 && !KNN) {
    // occupancy sweep of the product forward: cap the workgroups per CU with padded LDS
    const mrp_host::Geometry g = mrp_host::make_geometry(C, P, 4, 16, 64, mrp::kMaxChanPerBlock);
    mrp::AggArgs a = args_for(g.lpc, g.cpb);
    const int grid = B * a.ncb;
    const size_t base = mrp_host::lds_fwd<8>(g.cpb);
    for (int cap : {0, 2, 3, 4, 5, 6, 8}) {
      const size_t lds = cap ? std::max(base, (size_t)(160 * 1024 / cap) - 256) : base;
      char nm[64];
      snprintf(nm, sizeof nm, "film_fwd occupancy cap=%d wg/cu lds=%zu", cap, lds);
      float ms = time_ms([&] { hipLaunchKernelGGL((mrp::film_fwd<8, 4, true>), dim3(grid), dim3(g.threads), lds, 0, a); },
                         iters);
      report(nm, ms, alg);
    }
    for (int grid2 : {256, 512, 768}) {
      char nm[64];
      snprintf(nm, sizeof nm, "stream_copy f4 grid=%d", grid2);
      float ms = time_ms([&] { hipLaunchKernelGGL(lab::stream_copy<mrp::f4>, dim3(grid2), dim3(256), 0, 0,
                                                  (const mrp::f4*)x, (mrp::f4*)out, feat / 4); }, iters);
      report(nm, ms, (double)feat * 8);
    }
  }

  if (N == 8 && !KNN) {
    mrp::AggArgs a = args_for(64, 4);
    const int items = B * a.ncb;
    const size_t lds = (size_t)(2 * 4 * mrp::Tile<8>::SZ + 2 * mrp::Tile<8>::NTP) * 4;
#define VAR(PRO, MATH, NTL, PERSIST, GRID)                                                               \
    {                                                                                                    \
      const int grid_ = (GRID);                                                                          \
      float ms_ = time_ms([&] { hipLaunchKernelGGL((lab::fwd_var<8, PRO, MATH, NTL, PERSIST>), dim3(grid_), \
                                                   dim3(256), lds, 0, a, items); }, iters);               \
      char nm_[96];                                                                                      \
      snprintf(nm_, sizeof nm_, "var pro=%d math=%d nt=%d persist=%d grid=%d", PRO, MATH, NTL, PERSIST, grid_); \
      report(nm_, ms_, alg);                                                                             \
    }
    VAR(true, true, false, false, items)
    VAR(false, true, false, false, items)
    VAR(true, false, false, false, items)
    VAR(false, false, false, false, items)
    VAR(true, true, true, false, items)
    VAR(false, false, true, false, items)
    VAR(true, true, false, true, 1024)
    VAR(true, true, false, true, 2048)
    VAR(false, false, false, true, 1024)
    VAR(true, true, true, true, 1024)
    VAR(false, false, true, true, 1024)
    VAR(false, true, false, true, 1024)
  }
  if (N == 8 && !KNN) {
    // backward variants: slice width (VEC) and waves/SIMD bound
    float* dgb;
    CK(hipMalloc(&dgb, (size_t)E * C * 2 * 4));
    const double bwd_bytes = (double)feat * 12 + (double)E * C * 2 * 8;
    auto bargs = [&](int vec) {
      mrp::AggArgs a = {};
      a.x = x; a.xs = (int64_t)C * P; a.g = gout; a.gs = (int64_t)C * P; a.gb = gb; a.goff = d_goff;
      a.indptr = d_indptr; a.src = d_src; a.eid = d_eid; a.out = out; a.os = (int64_t)C * P; a.dgb = dgb;
      a.C = C; a.P = P; a.PV = P / vec; a.mode = 0; a.lpc = 64; a.cpb = 4; a.ncb = C / 4;
      a.want_dx = 1; a.want_dgb = 1; a.logits = 1;
      return a;
    };
    const size_t lds = (size_t)(2 * 4 * mrp::Tile<8>::SZ + 4 * mrp::Tile<8>::NTP + mrp::Tile<8>::NTP) * 4;
#define BVAR(VEC, MINW)                                                                                  \
    {                                                                                                    \
      mrp::AggArgs a = bargs(VEC);                                                                       \
      float ms_ = time_ms([&] { hipLaunchKernelGGL((mrp::film_bwd_fused<8, 8, VEC, true, false, MINW>),         \
                                                   dim3(B * a.ncb), dim3(256), lds, 0, a); }, iters);    \
      char nm_[96];                                                                                      \
      snprintf(nm_, sizeof nm_, "bwd_fused<8> vec=%d minw=%d", VEC, MINW);                              \
      report(nm_, ms_, bwd_bytes);                                                                       \
    }
    BVAR(4, 1)
    BVAR(4, 3)
    BVAR(2, 1)
    BVAR(2, 3)
    BVAR(2, 4)
    CK(hipFree(dgb));
  }
  if (KNN >= 1 && KNN <= 4 && N > 8) {
    // regular (per-edge-slot) backward: lanes per channel plane x slice width
    float* dgb;
    CK(hipMalloc(&dgb, (size_t)E * C * 2 * 4));
    const double bwd_bytes = (double)feat * 12 + (double)E * C * 2 * 8;
    auto rargs = [&](int vec, int lpc) {
      mrp::AggArgs a = {};
      const int cpb = std::min(16, 256 / lpc);
      a.x = x; a.xs = (int64_t)C * P; a.g = gout; a.gs = (int64_t)C * P; a.gb = gb; a.goff = d_goff;
      a.indptr = d_indptr; a.src = d_src; a.eid = d_eid; a.out = out; a.os = (int64_t)C * P; a.dgb = dgb;
      a.C = C; a.P = P; a.PV = P / vec; a.mode = 0; a.lpc = lpc; a.cpb = cpb; a.ncb = (C + cpb - 1) / cpb;
      a.want_dx = 1; a.want_dgb = 1; a.logits = 1; a.kdeg = KNN;
      return a;
    };
#define RVAR(NT, VEC, LPC)                                                                               \
    if (N == NT) {                                                                                       \
      mrp::AggArgs a = rargs(VEC, LPC);                                                                  \
      const size_t lds_ = lds_regular<NT, 4>(a.cpb);                                                     \
      float ms_ = time_ms([&] { hipLaunchKernelGGL((mrp::film_bwd_regular<NT, 4, VEC, false>),           \
                                                   dim3(B * a.ncb), dim3(a.cpb * LPC), lds_, 0, a); }, iters); \
      char nm_[96];                                                                                      \
      snprintf(nm_, sizeof nm_, "bwd_regular<%d> vec=%d lpc=%d cpb=%d", NT, VEC, LPC, a.cpb);           \
      report(nm_, ms_, bwd_bytes);                                                                       \
    }
    RVAR(16, 2, 64)
    RVAR(16, 2, 32)
    RVAR(16, 2, 16)
    RVAR(16, 2, 8)
    RVAR(16, 1, 64)
    RVAR(16, 1, 32)
    RVAR(16, 1, 16)
    RVAR(16, 1, 8)
    CK(hipFree(dgb));
  }
  {
    // product dispatch at forced geometries: lanes per channel plane (cpb = min(16, 256/lpc))
    float* dgb;
    CK(hipMalloc(&dgb, (size_t)E * C * 2 * 4));
    const double bwd_bytes = (double)feat * 12 + (double)E * C * 2 * 8;
    const int kind = KNN ? (int)MRP_GRAPH_REGULAR(KNN) : (int)MRP_GRAPH_COMPLETE;
    for (int bwd = 0; bwd < 2; ++bwd) {
      for (int vec : {4, 2, 1}) {
        for (int lpc : {64, 32, 16, 8, 4}) {
          if (bwd && KNN && N > 8 && vec == 4) continue;  // the regular kernel has no 16-byte variant
          if (bwd && !(KNN && N > 8) && vec == 2) continue;
          if (lpc > P / vec) continue;
          Geometry g;
          g.vec = vec;
          g.lpc = lpc;
          g.cpb = std::min(C, 256 / lpc);
          g.threads = g.cpb * lpc;
          g.ncb = (C + g.cpb - 1) / g.cpb;
          g.grid = (int64_t)B * g.ncb;
          mrp::AggArgs a = {};
          a.x = x; a.xs = (int64_t)C * P; a.gb = gb; a.indptr = d_indptr; a.src = d_src; a.eid = d_eid;
          a.goff = d_goff; a.out = out; a.os = (int64_t)C * P; a.C = C; a.P = P; a.PV = P / vec; a.mode = 0;
          a.lpc = g.lpc; a.cpb = g.cpb; a.ncb = g.ncb; a.logits = 1;
          if (bwd) {
            a.g = gout; a.gs = (int64_t)C * P; a.dgb = dgb; a.want_dx = 1; a.want_dgb = 1;
            a.kdeg = KNN;
          }
          float ms = time_ms([&] {
            CK(bwd ? dispatch_bwd(N, kind == MRP_GRAPH_COMPLETE, a, g, nullptr)
                   : dispatch_fwd(N, kind == MRP_GRAPH_COMPLETE, a, g, nullptr));
          }, iters);
          char nm[96];
          snprintf(nm, sizeof nm, "%s vec=%d lpc=%d cpb=%d grid=%lld", bwd ? "bwd" : "fwd", vec, lpc, g.cpb,
                   (long long)g.grid);
          report(nm, ms, bwd ? bwd_bytes : alg);
        }
      }
    }
    CK(hipFree(dgb));
  }
  if (N == 8 && !KNN) {
    // fused backward: slice width x occupancy floor (MINW = waves per SIMD the compiler must fit)
    float* dgb2;
    CK(hipMalloc(&dgb2, (size_t)E * C * 2 * 4));
    const double bwd_bytes = (double)feat * 12 + (double)E * C * 2 * 8;
    auto run = [&](auto kern, int vec, int lpc, int minw) {
      if (lpc > P / vec) return;
      const int cpb = std::min(C, std::min(256 / lpc, 32));
      mrp::AggArgs a = {};
      a.x = x; a.xs = (int64_t)C * P; a.gb = gb; a.goff = d_goff; a.out = out; a.os = (int64_t)C * P;
      a.C = C; a.P = P; a.PV = P / vec; a.mode = 0; a.lpc = lpc; a.cpb = cpb; a.ncb = (C + cpb - 1) / cpb;
      a.logits = 1; a.g = gout; a.gs = (int64_t)C * P; a.dgb = dgb2; a.want_dx = 1; a.want_dgb = 1;
      const int grid = B * a.ncb;
      const size_t lds = mrp_host::lds_bwd<8>(cpb, true);
      float ms = time_ms([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(cpb * lpc), lds, 0, a); }, iters);
      char nm[96];
      snprintf(nm, sizeof nm, "bwd_fused vec=%d minw=%d lpc=%d cpb=%d", vec, minw, lpc, cpb);
      report(nm, ms, bwd_bytes);
    };
    for (int lpc : {4, 8, 16, 32}) {
      run(mrp::film_bwd_fused<8, 8, 4, true, false, 1>, 4, lpc, 1);
      run(mrp::film_bwd_fused<8, 8, 4, true, false, 2>, 4, lpc, 2);
      run(mrp::film_bwd_fused<8, 8, 4, true, false, 3>, 4, lpc, 3);
      run(mrp::film_bwd_fused<8, 8, 2, true, false, 1>, 2, lpc, 1);
      run(mrp::film_bwd_fused<8, 8, 2, true, false, 3>, 2, lpc, 3);
      run(mrp::film_bwd_fused<8, 8, 2, true, false, 4>, 2, lpc, 4);
    }
    CK(hipFree(dgb2));
  }
  // product entry points (default geometry), both graph kinds
  float* dgb_prod;
  CK(hipMalloc(&dgb_prod, (size_t)E * C * 2 * 4));
  for (int kind : {(int)MRP_GRAPH_CSR, (int)MRP_GRAPH_COMPLETE, (int)MRP_GRAPH_REGULAR(KNN)}) {
    if (KNN && kind == MRP_GRAPH_COMPLETE) continue;
    if (!KNN && MRP_GRAPH_IS_REGULAR(kind)) continue;
    char nm[96];
    float ms = time_ms([&] {
      CK((hipError_t)mrp_film_mean_fwd(x, (int64_t)C * P, gb, d_indptr, d_src, d_eid, d_goff, B, N, kind, Nt, E, C,
                                       P, 0, out, (int64_t)C * P, nullptr));
    }, iters);
    const char* kn = kind == MRP_GRAPH_CSR ? "csr" : kind == MRP_GRAPH_COMPLETE ? "complete" : "regular";
    snprintf(nm, sizeof nm, "mrp_film_mean_fwd kind=%s", kn);
    report(nm, ms, alg);
    {
      float* catb;
      CK(hipMalloc(&catb, (size_t)Nt * 2 * C * P * 4));
      ms = time_ms([&] {
        CK((hipError_t)mrp_film_mean_cat_fwd(x, (int64_t)C * P, gb, d_indptr, d_src, d_eid, d_goff, B, N, kind, Nt,
                                             E, C, P, 0, catb, (int64_t)2 * C * P, nullptr));
      }, iters);
      snprintf(nm, sizeof nm, "mrp_film_mean_cat_fwd kind=%s", kn);
      report(nm, ms, alg + (double)feat * 4);  // + the copy of x
      CK(hipFree(catb));
    }
    ms = time_ms([&] {
      CK((hipError_t)mrp_film_mean_bwd(gout, (int64_t)C * P, x, (int64_t)C * P, gb, d_indptr, d_src, d_eid, d_goff, B,
                                       N, kind, Nt, E, C, P, MRP_AGG_GB_LOGITS, out, (int64_t)C * P, nullptr, 0,
                                       dgb_prod, nullptr));
    }, iters);
    snprintf(nm, sizeof nm, "mrp_film_mean_bwd kind=%s (dx+dgb)", kn);
    // bwd alg bytes: read G and x, write dx, read gb, write dgb
    report(nm, ms, (double)feat * 12 + (double)E * C * 2 * 8);
  }
  CK(hipFree(x));
  CK(hipFree(out));
  CK(hipFree(gb));
  return 0;
}
