// film_mean.hip — gfx950 (MI355X / CDNA4) kernels for the FiLM-mean GCN aggregation.
//
// Hot path replaced (xjh19971/multi-robot-perception-gnn-1):
//   GCN.forward                      dgl/model/models.py:219-226
//     g.update_all(edge_udf, node_udf)                 :223
//     edge_udf: m_e = gamma_e * x_src + beta_e         :210-211
//     node_udf: out_v = mailbox['m'].mean(1)           :207-208
//
// Design:
//   * One workgroup = one per-frame graph (<= 16 nodes) x a block of channels.
//     Its prologue turns the graph's in-edges and the interleaved (E, C, 2)
//     gamma/beta rows into dense per-channel N x N weight tiles in LDS.
//   * The main loop is one coalesced HBM sweep over the channel planes: every lane
//     owns a 16-byte slice p of one channel plane, loads that slice of all N source
//     nodes once (N x dwordx4), and emits all N destination slices from registers.
//     Each source map is therefore read exactly once, instead of deg(v) times plus
//     the E x C x H x W message/mailbox tensors DGL materialises.
//   * The forward keeps the reference's rounding order exactly for edges listed in
//     ascending source order (complete i-major graphs, our kNN builder):
//     m = fl(fl(gamma*x) + beta), acc = fl(acc + m) in source order, out = fl(acc / deg).
//     Non-neighbours are skipped (wave-uniform edge mask).  No FMA contraction.
//   * Backward: grad_x via the transposed tiles, d gamma / d beta as per-edge
//     P-length dot products (Gram of grad_out and x planes) reduced with wave shuffles;
//     no atomics, every output element written by one lane -> deterministic.
//   * Everything is HBM-bound (about N/4 flop per byte), so no MFMA here.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrp_gnn.h"

namespace mrp {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kBlock = 256;        // threads per workgroup (4 waves)
constexpr int kMaxChanPerBlock = 16;

struct AggArgs {
  const float* x;   // source node features (fwd: x, bwd: x)
  int64_t xs;       // node stride (elements)
  const float* g;   // bwd: grad_out
  int64_t gs;
  const float* gb;  // (E, C, 2) interleaved gamma/beta
  const int32_t* indptr;
  const int32_t* src;
  const int32_t* eid;
  const int32_t* goff;
  float* out;       // fwd: out, bwd: grad_x
  int64_t os;
  float* dgb;       // bwd: grad of gb (E, C, 2)
  int32_t C, P, PV, mode;
  int32_t lpc;      // lanes per channel plane (power of two <= 64)
  int32_t cpb;      // channels per workgroup
  int32_t ncb;      // channel blocks per graph
  int32_t want_dx, want_dgb;
};

template <int VEC>
struct Frag {
  float v[VEC];
};

template <int VEC>
__device__ __forceinline__ Frag<VEC> load_frag(const float* p) {
  Frag<VEC> f;
  if constexpr (VEC == 4) {
    const f4 t = *reinterpret_cast<const f4*>(p);
    f.v[0] = t.x; f.v[1] = t.y; f.v[2] = t.z; f.v[3] = t.w;
  } else {
    f.v[0] = *p;
  }
  return f;
}

template <int VEC>
__device__ __forceinline__ void store_frag(float* p, const Frag<VEC>& f) {
  if constexpr (VEC == 4) {
    f4 t;
    t.x = f.v[0]; t.y = f.v[1]; t.z = f.v[2]; t.w = f.v[3];
    *reinterpret_cast<f4*>(p) = t;
  } else {
    *p = f.v[0];
  }
}

template <int NT>
struct Tile {
  static constexpr int NTP = (NT + 3) & ~3;  // padded row -> 16-byte aligned LDS rows
  static constexpr int SZ = NT * NTP;        // floats per channel tile
};

// ---------------------------------------------------------------------------
// Prologue: dense per-channel weight tiles from the CSR-by-destination graph.
//
//   FWD  : Ga[cl][v][u] = sum of gamma over edges u->v (1 per edge for COPY),
//          Gb[cl][v][u] = sum of beta  over edges u->v (0 for COPY),
//          degf[v]      = in-degree (float).
//   BWD  : Wt[cl][u][v] = s_v * Ga[cl][v][u]  (transposed, scaled by the reduce
//          scale s_v = 1/deg v (mean) or 1 (sum)); sc[v] = s_v.
// Each (channel, v) row is built by one thread walking v's in-edges in CSR order,
// so there are no LDS races, including for multi-edges.
// ---------------------------------------------------------------------------
template <int NT, bool BWD>
__device__ __forceinline__ void build_tiles(const AggArgs& a, int node0, int n, int c0,
                                            float* Ga, float* Gb, float* sc, unsigned* emask) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  const int tid = threadIdx.x;
  const int nth = blockDim.x;
  const int tot = a.cpb * SZ;
  for (int i = tid; i < tot; i += nth) {
    Ga[i] = 0.f;
    if (!BWD) Gb[i] = 0.f;
  }
  __syncthreads();
  for (int t = tid; t < a.cpb * NT; t += nth) {
    const int cl = t % a.cpb;  // channel fastest: neighbouring lanes read neighbouring gb pairs
    const int v = t / a.cpb;
    const int c = c0 + cl;
    if (v < n && c < a.C) {
      const int beg = a.indptr[node0 + v];
      const int end = a.indptr[node0 + v + 1];
      const int deg = end - beg;
      float s = 1.f;
      if (BWD && a.mode != MRP_AGG_FILM_SUM && deg > 0) s = 1.f / (float)deg;
      unsigned mask = 0u;
      for (int k = beg; k < end; ++k) {
        const int u = a.src[k] - node0;
        if ((unsigned)u >= (unsigned)n) continue;  // edge leaves the graph: rejected on the host
        mask |= 1u << u;
        float gam = 1.f, bet = 0.f;
        if (a.mode != MRP_AGG_COPY_MEAN) {
          const float* q = a.gb + ((int64_t)a.eid[k] * a.C + c) * 2;
          gam = q[0];
          bet = q[1];
        }
        if (BWD) {
          Ga[cl * SZ + u * NTP + v] += s * gam;
        } else {
          Ga[cl * SZ + v * NTP + u] += gam;
          Gb[cl * SZ + v * NTP + u] += bet;
        }
      }
      if (cl == 0) {
        sc[v] = BWD ? s : (float)deg;
        if (!BWD) emask[v] = mask;
      }
    } else if (cl == 0) {
      sc[v] = 0.f;
      if (!BWD) emask[v] = 0u;
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Forward.  out[v] = reduce_{e=(u->v)} (gamma_e * x_u + beta_e), zero if deg v == 0.
// ---------------------------------------------------------------------------
template <int NT, int VEC>
__global__ void __launch_bounds__(kBlock) film_fwd(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Ga = smem;
  float* Gb = Ga + a.cpb * SZ;
  float* degf = Gb + a.cpb * SZ;
  unsigned* emask = reinterpret_cast<unsigned*>(degf + NTP);

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = a.goff[b];
  const int n = min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;  // whole workgroup: empty graph
  const int c0 = cb * a.cpb;

  build_tiles<NT, false>(a, node0, n, c0, Ga, Gb, degf, emask);

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  if (grp >= a.cpb || c >= a.C) return;

  const float* xb = a.x + (int64_t)node0 * a.xs + (int64_t)c * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
  const float* A = Ga + grp * SZ;
  const float* Bt = Gb + grp * SZ;
  const bool film = a.mode != MRP_AGG_COPY_MEAN;
  const bool mean = a.mode != MRP_AGG_FILM_SUM;

  for (int j = li; j < a.PV; j += a.lpc) {
    const int64_t off = (int64_t)j * VEC;
    Frag<VEC> xv[NT];
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int uu = u < n ? u : n - 1;  // clamp (ragged batch); weight is 0 there
      xv[u] = load_frag<VEC>(xb + (int64_t)uu * a.xs + off);
    }
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      if (v >= n) break;
      // Edge mask of v: channel independent, so wave-uniform -> scalar branches.
      const unsigned em = __builtin_amdgcn_readfirstlane(emask[v]);
      Frag<VEC> acc;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
#pragma unroll
      for (int u4 = 0; u4 < NTP; u4 += 4) {
        const f4 wa = *reinterpret_cast<const f4*>(A + v * NTP + u4);
        const f4 wb = *reinterpret_cast<const f4*>(Bt + v * NTP + u4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int u = u4 + q;
          if (u >= NT) break;
          if (!((em >> u) & 1u)) continue;  // not a neighbour: never touched (as in DGL)
          const float ga = wa[q];
          const float gbv = wb[q];
#pragma unroll
          for (int k = 0; k < VEC; ++k) {
            float m;
            if (film) m = __fadd_rn(__fmul_rn(ga, xv[u].v[k]), gbv);
            else m = __fmul_rn(ga, xv[u].v[k]);
            acc.v[k] = __fadd_rn(acc.v[k], m);
          }
        }
      }
      const float d = degf[v];
      if (mean && d > 0.f) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc.v[k] = acc.v[k] / d;
      }
      store_frag<VEC>(ob + (int64_t)v * a.os + off, acc);
    }
  }
}

// ---------------------------------------------------------------------------
// Backward, grad_x only (used for NT > 8, where the fused kernel's Gram
// accumulators would not fit in registers):  grad_x[u] = sum_v Wt[u][v] * G[v].
// ---------------------------------------------------------------------------
template <int NT, int VEC>
__global__ void __launch_bounds__(kBlock) film_bwd_dx(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Wt = smem;
  float* sc = Wt + a.cpb * SZ;

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = a.goff[b];
  const int n = min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;

  build_tiles<NT, true>(a, node0, n, c0, Wt, nullptr, sc, nullptr);

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  if (grp >= a.cpb || c >= a.C) return;

  const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
  const float* W = Wt + grp * SZ;

  for (int j = li; j < a.PV; j += a.lpc) {
    const int64_t off = (int64_t)j * VEC;
    Frag<VEC> gv[NT];
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      const int vv = v < n ? v : n - 1;
      gv[v] = load_frag<VEC>(gbase + (int64_t)vv * a.gs + off);
    }
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      if (u >= n) break;
      Frag<VEC> acc;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
#pragma unroll
      for (int v4 = 0; v4 < NTP; v4 += 4) {
        const f4 w = *reinterpret_cast<const f4*>(W + u * NTP + v4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = v4 + q;
          if (v >= NT) break;
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(w[q], gv[v].v[k], acc.v[k]);
        }
      }
      store_frag<VEC>(ob + (int64_t)u * a.os + off, acc);
    }
  }
}

// Reduce a value over the lpc lanes of one channel group (lpc is a power of two).
__device__ __forceinline__ float group_sum(float x, int lpc) {
  for (int m = lpc >> 1; m > 0; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

// ---------------------------------------------------------------------------
// Backward, fused: one sweep reads G and x once, writes grad_x (if VB == NT and
// want_dx) and accumulates the per-channel Gram D[v][u] = sum_p G_v * x_u and
// S[v] = sum_p G_v for a block of VB destination rows; then writes
//   grad_gb[e, c] = (s_v * D[v][u], s_v * S[v])    for every edge e = (u -> v).
// For NT > 8 the kernel runs with VB = 4 and loops over destination blocks.
// ---------------------------------------------------------------------------
template <int NT, int VB, int VEC>
__global__ void __launch_bounds__(kBlock) film_bwd_fused(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Wt = smem;                     // [cpb][NT][NTP]   scaled, transposed
  float* Dl = Wt + a.cpb * SZ;          // [cpb][NT][NTP]   Gram (unscaled)
  float* Sl = Dl + a.cpb * SZ;          // [cpb][NTP]       sum_p G_v
  float* sc = Sl + a.cpb * NTP;         // [NTP]            s_v

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = a.goff[b];
  const int n = min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;

  build_tiles<NT, true>(a, node0, n, c0, Wt, nullptr, sc, nullptr);

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  const bool active = grp < a.cpb && c < a.C;

  const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c * a.P;
  const float* xbase = a.x + (int64_t)node0 * a.xs + (int64_t)c * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
  const float* W = Wt + grp * SZ;
  const bool do_dx = (VB == NT) && a.want_dx;

#pragma unroll 1
  for (int vb = 0; vb < NT; vb += VB) {
    float D[VB][NT];
    float S[VB];
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      S[i] = 0.f;
#pragma unroll
      for (int u = 0; u < NT; ++u) D[i][u] = 0.f;
    }
    if (active) {
      for (int j = li; j < a.PV; j += a.lpc) {
        const int64_t off = (int64_t)j * VEC;
        Frag<VEC> gv[VB];
        Frag<VEC> xv[NT];
#pragma unroll
        for (int i = 0; i < VB; ++i) {
          const int v = vb + i;
          const int vv = v < n ? v : n - 1;
          gv[i] = load_frag<VEC>(gbase + (int64_t)vv * a.gs + off);
        }
        if (a.want_dgb) {
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            const int uu = u < n ? u : n - 1;
            xv[u] = load_frag<VEC>(xbase + (int64_t)uu * a.xs + off);
          }
        }
        if (do_dx) {
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            if (u >= n) break;
            Frag<VEC> acc;
#pragma unroll
            for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
#pragma unroll
            for (int v4 = 0; v4 < NTP; v4 += 4) {
              const f4 w = *reinterpret_cast<const f4*>(W + u * NTP + v4);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int v = v4 + q;
                if (v >= NT) break;
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(w[q], gv[v].v[k], acc.v[k]);
              }
            }
            store_frag<VEC>(ob + (int64_t)u * a.os + off, acc);
          }
        }
        if (a.want_dgb) {
#pragma unroll
          for (int i = 0; i < VB; ++i) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) S[i] += gv[i].v[k];
#pragma unroll
            for (int u = 0; u < NT; ++u) {
#pragma unroll
              for (int k = 0; k < VEC; ++k) D[i][u] = fmaf(gv[i].v[k], xv[u].v[k], D[i][u]);
            }
          }
        }
      }
    }
    if (a.want_dgb) {
      // Reduce across the lanes of each channel group (all lanes of the wave take
      // part in the shuffles; inactive groups contribute zeros to their own group).
#pragma unroll
      for (int i = 0; i < VB; ++i) {
        S[i] = group_sum(S[i], a.lpc);
#pragma unroll
        for (int u = 0; u < NT; ++u) D[i][u] = group_sum(D[i][u], a.lpc);
      }
      if (active && li == 0) {
#pragma unroll
        for (int i = 0; i < VB; ++i) {
          const int v = vb + i;
          if (v < NT) {
            Sl[grp * NTP + v] = S[i];
#pragma unroll
            for (int u = 0; u < NT; ++u) Dl[grp * SZ + v * NTP + u] = D[i][u];
          }
        }
      }
    }
  }
  if (!a.want_dgb) return;
  __syncthreads();
  // Per-edge outputs.  Thread -> (channel fastest, destination v); the in-edges
  // of v are walked in CSR order.  Every edge of the graph has exactly one
  // destination here, so each grad_gb element is written once.
  for (int t = threadIdx.x; t < a.cpb * NT; t += blockDim.x) {
    const int cl = t % a.cpb;
    const int v = t / a.cpb;
    const int cc = c0 + cl;
    if (v >= n || cc >= a.C) continue;
    const int beg = a.indptr[node0 + v];
    const int end = a.indptr[node0 + v + 1];
    const float s = sc[v];
    const float dbeta = s * Sl[cl * NTP + v];
    for (int k = beg; k < end; ++k) {
      const int u = a.src[k] - node0;
      float dgam = 0.f, dbet = 0.f;
      if ((unsigned)u < (unsigned)n) {
        dgam = s * Dl[cl * SZ + v * NTP + u];
        dbet = dbeta;
      }
      float* q = a.dgb + ((int64_t)a.eid[k] * a.C + cc) * 2;
      q[0] = dgam;
      q[1] = dbet;
    }
  }
}

}  // namespace mrp

// ===========================================================================
// Host side: validation, geometry, template dispatch, C ABI.
// ===========================================================================
namespace {

using mrp::AggArgs;

struct Geometry {
  int vec, lpc, cpb, threads, ncb;
  int64_t grid;
};

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

Geometry make_geometry(int C, int P, bool vec4) {
  Geometry g;
  g.vec = vec4 ? 4 : 1;
  const int pv = P / g.vec;
  int lpc = 1;
  while (lpc * 2 <= pv && lpc * 2 <= 64) lpc *= 2;
  int cpb = mrp::kBlock / lpc;
  if (cpb > mrp::kMaxChanPerBlock) cpb = mrp::kMaxChanPerBlock;
  if (cpb > C) cpb = C;
  g.lpc = lpc;
  g.cpb = cpb;
  g.threads = cpb * lpc;
  g.ncb = (C + cpb - 1) / cpb;
  g.grid = 0;
  return g;
}

template <int NT>
size_t lds_fwd(int cpb) {
  return (size_t)(2 * cpb * mrp::Tile<NT>::SZ + 2 * mrp::Tile<NT>::NTP) * sizeof(float);
}
template <int NT>
size_t lds_dx(int cpb) {
  return (size_t)(cpb * mrp::Tile<NT>::SZ + mrp::Tile<NT>::NTP) * sizeof(float);
}
template <int NT>
size_t lds_bwd(int cpb) {
  return (size_t)(2 * cpb * mrp::Tile<NT>::SZ + cpb * mrp::Tile<NT>::NTP + mrp::Tile<NT>::NTP) *
         sizeof(float);
}

template <int NT>
hipError_t launch_fwd_nt(const AggArgs& a, const Geometry& g, hipStream_t st) {
  const size_t lds = lds_fwd<NT>(g.cpb);
  if (g.vec == 4)
    hipLaunchKernelGGL((mrp::film_fwd<NT, 4>), dim3((unsigned)g.grid), dim3(g.threads), lds, st, a);
  else
    hipLaunchKernelGGL((mrp::film_fwd<NT, 1>), dim3((unsigned)g.grid), dim3(g.threads), lds, st, a);
  return hipGetLastError();
}

template <int NT>
hipError_t launch_bwd_nt(const AggArgs& a, const Geometry& g, hipStream_t st) {
  if constexpr (NT <= 8) {
    const size_t lds = lds_bwd<NT>(g.cpb);
    if (g.vec == 4)
      hipLaunchKernelGGL((mrp::film_bwd_fused<NT, NT, 4>), dim3((unsigned)g.grid), dim3(g.threads), lds,
                         st, a);
    else
      hipLaunchKernelGGL((mrp::film_bwd_fused<NT, NT, 1>), dim3((unsigned)g.grid), dim3(g.threads), lds,
                         st, a);
    return hipGetLastError();
  } else {
    if (a.want_dx) {
      const size_t lds = lds_dx<NT>(g.cpb);
      if (g.vec == 4)
        hipLaunchKernelGGL((mrp::film_bwd_dx<NT, 4>), dim3((unsigned)g.grid), dim3(g.threads), lds, st, a);
      else
        hipLaunchKernelGGL((mrp::film_bwd_dx<NT, 1>), dim3((unsigned)g.grid), dim3(g.threads), lds, st, a);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    if (a.want_dgb) {
      AggArgs b = a;
      b.want_dx = 0;
      const size_t lds = lds_bwd<NT>(g.cpb);
      if (g.vec == 4)
        hipLaunchKernelGGL((mrp::film_bwd_fused<NT, 4, 4>), dim3((unsigned)g.grid), dim3(g.threads), lds,
                           st, b);
      else
        hipLaunchKernelGGL((mrp::film_bwd_fused<NT, 4, 1>), dim3((unsigned)g.grid), dim3(g.threads), lds,
                           st, b);
      return hipGetLastError();
    }
    return hipSuccess;
  }
}

#define MRP_DISPATCH_NT(NTV, FN, ...) \
  switch (NTV) {                      \
    case 1: return FN<1>(__VA_ARGS__);   \
    case 2: return FN<2>(__VA_ARGS__);   \
    case 3: return FN<3>(__VA_ARGS__);   \
    case 4: return FN<4>(__VA_ARGS__);   \
    case 5: return FN<5>(__VA_ARGS__);   \
    case 6: return FN<6>(__VA_ARGS__);   \
    case 7: return FN<7>(__VA_ARGS__);   \
    case 8: return FN<8>(__VA_ARGS__);   \
    case 9: return FN<9>(__VA_ARGS__);   \
    case 10: return FN<10>(__VA_ARGS__); \
    case 11: return FN<11>(__VA_ARGS__); \
    case 12: return FN<12>(__VA_ARGS__); \
    case 13: return FN<13>(__VA_ARGS__); \
    case 14: return FN<14>(__VA_ARGS__); \
    case 15: return FN<15>(__VA_ARGS__); \
    case 16: return FN<16>(__VA_ARGS__); \
    default: return hipErrorInvalidValue; \
  }

hipError_t dispatch_fwd(int nt, const AggArgs& a, const Geometry& g, hipStream_t st) {
  MRP_DISPATCH_NT(nt, launch_fwd_nt, a, g, st)
}
hipError_t dispatch_bwd(int nt, const AggArgs& a, const Geometry& g, hipStream_t st) {
  MRP_DISPATCH_NT(nt, launch_bwd_nt, a, g, st)
}

bool common_args_ok(const int32_t* indptr, const int32_t* src, const int32_t* eid,
                    const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                    int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P, int32_t mode) {
  if (num_graphs < 0 || num_nodes < 0 || num_edges < 0 || C < 0 || P < 0) return false;
  if (max_nodes < 0 || max_nodes > MRP_MAX_NODES) return false;
  if (mode < MRP_AGG_FILM_MEAN || mode > MRP_AGG_COPY_MEAN) return false;
  if (num_graphs > 0 && graph_off == nullptr) return false;
  if (num_nodes > 0 && indptr == nullptr) return false;
  if (num_edges > 0 && (src == nullptr || eid == nullptr)) return false;
  if ((int64_t)num_graphs * max_nodes < (int64_t)num_nodes) return false;
  return true;
}

}  // namespace

extern "C" {

int mrp_abi_version(void) { return 1; }

const char* mrp_error_string(int code) { return hipGetErrorString(static_cast<hipError_t>(code)); }

int mrp_film_mean_fwd(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                      const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                      int32_t max_nodes, int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P,
                      int32_t mode, float* out, int64_t out_node_stride, void* stream) {
  if (!common_args_ok(indptr, src, eid, graph_off, num_graphs, max_nodes, num_nodes, num_edges, C, P, mode))
    return hipErrorInvalidValue;
  if (num_graphs == 0 || num_nodes == 0 || max_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (x == nullptr || out == nullptr || x_node_stride < plane || out_node_stride < plane)
    return hipErrorInvalidValue;
  if (mode != MRP_AGG_COPY_MEAN && num_edges > 0 && gb == nullptr) return hipErrorInvalidValue;
  const bool vec4 = (P % 4 == 0) && (x_node_stride % 4 == 0) && (out_node_stride % 4 == 0) && aligned16(x) &&
                    aligned16(out);
  Geometry g = make_geometry(C, P, vec4);
  g.grid = (int64_t)num_graphs * g.ncb;
  if (g.grid > 0x7fffffff) return hipErrorInvalidValue;
  AggArgs a = {};
  a.x = x;
  a.xs = x_node_stride;
  a.gb = gb;
  a.indptr = indptr;
  a.src = src;
  a.eid = eid;
  a.goff = graph_off;
  a.out = out;
  a.os = out_node_stride;
  a.C = C;
  a.P = P;
  a.PV = P / g.vec;
  a.mode = mode;
  a.lpc = g.lpc;
  a.cpb = g.cpb;
  a.ncb = g.ncb;
  return dispatch_fwd(max_nodes, a, g, static_cast<hipStream_t>(stream));
}

int mrp_film_mean_bwd(const float* grad_out, int64_t g_node_stride, const float* x, int64_t x_node_stride,
                      const float* gb, const int32_t* indptr, const int32_t* src, const int32_t* eid,
                      const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes, int32_t num_nodes,
                      int32_t num_edges, int32_t C, int32_t P, int32_t mode, float* grad_x,
                      int64_t gx_node_stride, float* grad_gb, void* stream) {
  if (!common_args_ok(indptr, src, eid, graph_off, num_graphs, max_nodes, num_nodes, num_edges, C, P, mode))
    return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool copy = mode == MRP_AGG_COPY_MEAN;
  if (grad_gb != nullptr && num_edges > 0 && C > 0 && (copy || num_nodes == 0 || P == 0)) {
    // gamma/beta do not influence the output: their gradient is zero.
    hipError_t e = hipMemsetAsync(grad_gb, 0, (size_t)num_edges * C * 2 * sizeof(float), st);
    if (e != hipSuccess) return e;
  }
  const bool want_dgb = grad_gb != nullptr && !copy && num_edges > 0;
  const bool want_dx = grad_x != nullptr;
  if (!want_dgb && !want_dx) return hipSuccess;
  if (num_graphs == 0 || num_nodes == 0 || max_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (grad_out == nullptr || g_node_stride < plane) return hipErrorInvalidValue;
  if (want_dx && gx_node_stride < plane) return hipErrorInvalidValue;
  if (want_dgb && (x == nullptr || x_node_stride < plane)) return hipErrorInvalidValue;
  if (!copy && num_edges > 0 && gb == nullptr) return hipErrorInvalidValue;
  bool vec4 = (P % 4 == 0) && (g_node_stride % 4 == 0) && aligned16(grad_out);
  if (want_dx) vec4 = vec4 && (gx_node_stride % 4 == 0) && aligned16(grad_x);
  if (want_dgb) vec4 = vec4 && (x_node_stride % 4 == 0) && aligned16(x);
  Geometry g = make_geometry(C, P, vec4);
  g.grid = (int64_t)num_graphs * g.ncb;
  if (g.grid > 0x7fffffff) return hipErrorInvalidValue;
  AggArgs a = {};
  a.x = x;
  a.xs = x_node_stride;
  a.g = grad_out;
  a.gs = g_node_stride;
  a.gb = gb;
  a.indptr = indptr;
  a.src = src;
  a.eid = eid;
  a.goff = graph_off;
  a.out = grad_x;
  a.os = gx_node_stride;
  a.dgb = grad_gb;
  a.C = C;
  a.P = P;
  a.PV = P / g.vec;
  a.mode = mode;
  a.lpc = g.lpc;
  a.cpb = g.cpb;
  a.ncb = g.ncb;
  a.want_dx = want_dx ? 1 : 0;
  a.want_dgb = want_dgb ? 1 : 0;
  return dispatch_bwd(max_nodes, a, g, st);
}

}  // extern "C"
