#pragma once
// film_mean_kernels.hpp — gfx950 (MI355X / CDNA4) kernels for the FiLM-mean GCN aggregation
//
// Hot path replaced (xjh19971/multi-robot-perception-gnn-1):
//   GCN.forward                      dgl/model/models.py:219-226
//     g.update_all(edge_udf, node_udf)                 :223
//     edge_udf: m_e = gamma_e * x_src + beta_e         :210-211
//     node_udf: out_v = mailbox['m'].mean(1)           :207-208
//
// Design:
//   * One workgroup = one per-frame graph (<= 16 nodes) x a block of channels.  Its prologue
//     turns the graph's edges and the interleaved (E, C, 2) gamma/beta rows into dense
//     per-channel N x N weight tiles in LDS.  Two graph kinds:
//       - COMPLETE: the reference's only topology (dgl/dataloader.py:88-95), every graph with
//         exactly NT nodes, edges numbered graph by graph i-major: edge ids are arithmetic, one
//         gamma/beta load per LDS slot, and the neighbour mask (u != v) is compile-time;
//       - CSR: any graph (k-NN, ragged batches, multi-edges, self-loops): in-edges walked from
//         the CSR-by-destination arrays.
//   * The main loop is one coalesced HBM sweep over the channel planes: every lane owns a
//     16-byte slice of one channel plane, loads that slice of all N source nodes once
//     (N x dwordx4, nontemporal: read once), and emits all N destination slices from registers
//     (nontemporal stores).  Each source map is read exactly once, instead of deg(v) times plus
//     the E x C x H x W message and mailbox tensors DGL materialises.  The first slice's loads are
//     issued before the prologue's LDS writes so the weight build hides under them.
//   * The forward keeps the reference's rounding order exactly when each node's in-edges are in
//     ascending source order (complete i-major graphs, our k-NN builder):
//     m = fl(fl(gamma*x) + beta), acc = fl(acc + m) in source order, out = fl(acc / deg).
//     Non-neighbours are skipped, never multiplied by zero.  Built with -ffp-contract=off.
//   * Backward: grad_x via the transposed tiles, d gamma / d beta as per-edge P-length dot
//     products (Gram of grad_out and x planes) reduced with wave shuffles; no atomics, every
//     output element written by one lane -> deterministic.
//   * Everything is HBM-bound (about N/4 flop per byte), so no MFMA here.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <type_traits>

#include "fast_math.hpp"
#include "tuning.hpp"
#include "mrp_gnn.h"

namespace mrp {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kBlock = 256;  // threads per workgroup (4 waves)
constexpr int kMaxChanPerBlock = 16;

struct AggArgs {
  const float* x;  // source node features (fwd: x, bwd: x)
  int64_t xs;      // node stride (elements)
  const float* g;  // bwd: grad_out
  int64_t gs;
  const float* gb;  // (E, C, 2) interleaved gamma/beta
  const int32_t* indptr;
  const int32_t* src;
  const int32_t* eid;
  const int32_t* goff;
  float* out;  // fwd: out, bwd: grad_x
  int64_t os;
  float* dgb;  // bwd: grad of gb (E, C, 2)
  const float* dxb;  // bwd: optional grad_x base (added to grad_x), node stride dxbs
  int64_t dxbs;
  int32_t C, P, PV, mode;
  int32_t lpc;  // lanes per channel plane (power of two <= 64; <= 256 in film_bwd_fused: lpc/64 waves)
  int32_t cpb;  // channels per workgroup
  int32_t ncb;  // channel blocks per graph
  int32_t want_dx, want_dgb;
  int32_t logits;  // gb holds pre-sigmoid logits (MRP_AGG_GB_LOGITS): apply sigmoid on load
  int32_t kdeg;    // MRP_GRAPH_REGULAR: every node's in-degree (else 0)
  float* xc;       // forward: optional copy of x (the first half of a concatenation buffer)
  int64_t xcs;     // its node stride
  int32_t psplit;  // forward: plane segments per (graph, channel block) (0 or 1: whole plane)
  // epilogue (mrp_agg_epilogue): forward out = agg_scale*a + self_scale*x[v] + x0_scale*x0[v];
  // backward: grad_out reaches the aggregate scaled by agg_scale (folded into the reduce scale s_v),
  // and self_scale*grad_out[u] is added to grad_x[u].  epi = 0: plain (agg_scale 1, the rest 0).
  int32_t epi;
  float agg_scale, self_scale, x0_scale;
  const float* x0;
  int64_t x0s;
  int32_t nmax;  // max_nodes (COMPLETE graphs: every graph's node count)
};

// Forward epilogue of destination `node`, channel c, slice at `off` (see AggArgs::epi).
template <int VEC>
__device__ __forceinline__ void apply_epilogue(const AggArgs& a, float* acc, const float* xself, int node, int c,
                                               int64_t off) {
  if (a.agg_scale != 1.f) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fmul_rn(a.agg_scale, acc[k]);
  }
  if (a.self_scale != 0.f) {
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(a.self_scale, xself[k]));
  }
  if (a.x0 != nullptr) {
    const float* p = a.x0 + (int64_t)node * a.x0s + (int64_t)c * a.P + off;
    float z[VEC];
    if constexpr (VEC == 4) {
      const f4 t = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
      z[0] = t.x; z[1] = t.y; z[2] = t.z; z[3] = t.w;
    } else if constexpr (VEC == 2) {
      const f2 t = __builtin_nontemporal_load(reinterpret_cast<const f2*>(p));
      z[0] = t.x; z[1] = t.y;
    } else {
      z[0] = __builtin_nontemporal_load(p);
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], __fmul_rn(a.x0_scale, z[k]));
  }
}

__device__ __forceinline__ float sigmoidf(float z) { return mrp_math::sigmoid(z); }  // fast_math.hpp

// d/dz of gamma/beta = sigmoid(z): grad * s * (1 - s)
__device__ __forceinline__ float2 sigmoid_backward(float2 grad, float2 z) {
  const float sg = sigmoidf(z.x), sb = sigmoidf(z.y);
  return make_float2(grad.x * sg * (1.f - sg), grad.y * sb * (1.f - sb));
}

template <int VEC>
struct Frag {
  float v[VEC];
};

template <int VEC, bool NTL>
__device__ __forceinline__ Frag<VEC> load_frag(const float* p) {
  Frag<VEC> f;
  if constexpr (VEC == 4) {
    const f4* q = reinterpret_cast<const f4*>(p);
    const f4 t = NTL ? __builtin_nontemporal_load(q) : *q;
    f.v[0] = t.x;
    f.v[1] = t.y;
    f.v[2] = t.z;
    f.v[3] = t.w;
  } else if constexpr (VEC == 2) {
    const f2* q = reinterpret_cast<const f2*>(p);
    const f2 t = NTL ? __builtin_nontemporal_load(q) : *q;
    f.v[0] = t.x;
    f.v[1] = t.y;
  } else {
    f.v[0] = NTL ? __builtin_nontemporal_load(p) : *p;
  }
  return f;
}

template <int VEC, bool NTL>
__device__ __forceinline__ void store_frag(float* p, const Frag<VEC>& f) {
  if constexpr (VEC == 4) {
    f4 t;
    t.x = f.v[0];
    t.y = f.v[1];
    t.z = f.v[2];
    t.w = f.v[3];
    if (NTL)
      __builtin_nontemporal_store(t, reinterpret_cast<f4*>(p));
    else
      *reinterpret_cast<f4*>(p) = t;
  } else if constexpr (VEC == 2) {
    f2 t;
    t.x = f.v[0];
    t.y = f.v[1];
    if (NTL)
      __builtin_nontemporal_store(t, reinterpret_cast<f2*>(p));
    else
      *reinterpret_cast<f2*>(p) = t;
  } else {
    if (NTL)
      __builtin_nontemporal_store(f.v[0], p);
    else
      *p = f.v[0];
  }
}

// Wave-uniform base + 32-bit lane byte offset: lets the compiler use the SGPR-base form of
// global_load/store (saddr + 32-bit vaddr) instead of a 64-bit VGPR address per access — with N
// source and N destination planes per slice those addresses are most of a kernel's VGPRs.
__device__ __forceinline__ const float* at_bytes(const float* base, uint32_t off) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off);
}
__device__ __forceinline__ float* at_bytes(float* base, uint32_t off) {
  return reinterpret_cast<float*>(reinterpret_cast<char*>(base) + off);
}

template <int NT>
struct Tile {
  static constexpr int NTP = (NT + 3) & ~3;  // padded row -> 16-byte aligned LDS rows
  // floats per channel tile, padded by 4: consecutive channels' tiles start 4 banks apart, so the
  // channel groups of one wave (4-8 channels at 8x8 planes) read their broadcast weights without
  // the 4-8-way LDS bank conflicts an unpadded 64- or 256-float stride gives (rocprof r02: 70 % of
  // LDS cycles were conflicts at 8x8)
  static constexpr int SZ = NT * NTP + 4;
  // row stride of the backward's per-channel sums S[v] (16-byte rows: written as vectors): 12 floats
  // at N = 8 puts the 8 channels a half-wave reads in the epilogue (complete_epi_slot) on 8 banks
  static constexpr int SLS = NTP + 4;
};

// Edge id of u -> v (u != v) in a complete graph of n nodes whose edges start at ebase and are
// numbered i-major over ordered pairs (dgl/dataloader.py:88-95).
__device__ __forceinline__ int64_t complete_eid(int64_t ebase, int n, int u, int v) {
  return ebase + (int64_t)u * (n - 1) + (v < u ? v : v - 1);
}

// t -> (channel within the block, rest) with channel fastest.  cpb is wave-uniform and almost always
// a power of two: then a mask and a shift instead of an integer division.
__device__ __forceinline__ void split_channel(const AggArgs& a, int t, int& cl, int& rest) {
  if ((a.cpb & (a.cpb - 1)) == 0) {
    cl = t & (a.cpb - 1);
    rest = t >> __builtin_ctz((unsigned)a.cpb);
  } else {
    cl = t % a.cpb;
    rest = t / a.cpb;
  }
}

// ---------------------------------------------------------------------------
// Prologue, CSR graphs: dense per-channel weight tiles from the CSR-by-destination graph.
//
//   FWD  : Ga[cl][v][u] = sum of gamma over edges u->v (1 per edge for COPY),
//          Gb[cl][v][u] = sum of beta  over edges u->v (0 for COPY),
//          sc[v] = in-degree (float), emask[v] = neighbour bits.
//   BWD  : Ga[cl][u][v] = s_v * sum of gamma over edges u->v  (transposed, scaled by the reduce
//          scale s_v = 1/deg v (mean) or 1 (sum)); sc[v] = s_v.
// Each (channel, v) row is built by one thread walking v's in-edges in CSR order, so there are
// no LDS races, including for multi-edges.
// ---------------------------------------------------------------------------
template <int NT, bool BWD>
__device__ __forceinline__ void build_tiles_csr(const AggArgs& a, int node0, int n, int c0, float* Ga,
                                                float* Gb, float* sc, unsigned* emask) {
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
    int cl, v;  // channel fastest: neighbouring lanes read neighbouring gb pairs
    split_channel(a, t, cl, v);
    const int c = c0 + cl;
    if (v < n && c < a.C) {
      // MRP_GRAPH_REGULAR(k): every node has k in-edges, so its CSR row starts at k * node (the
      // graph kind guarantees it; the host checked) — one dependent load level less
      const int beg = a.kdeg > 0 ? (node0 + v) * a.kdeg : a.indptr[node0 + v];
      const int end = a.kdeg > 0 ? beg + a.kdeg : a.indptr[node0 + v + 1];
      const int deg = end - beg;
      float s = 1.f;
      if (BWD && a.mode != MRP_AGG_FILM_SUM && deg > 0) s = 1.f / (float)deg;
      if (BWD) s *= a.agg_scale;  // epilogue: grad_out reaches the aggregate scaled
      unsigned mask = 0u;
      // In-edges in chunks of KC, every load of a chunk issued before any is consumed (indices
      // clamped instead of branched around, so the loads stay independent); accumulation stays
      // in CSR order, so multi-edges sum deterministically.
      constexpr int KC = NT < 8 ? NT : 8;  // edges per chunk (bounded: the first slice's loads are live here)
      for (int k0 = beg; k0 < end; k0 += KC) {
        int us[KC];
        float2 gbv[KC];
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const int k = min(k0 + i, end - 1);
          us[i] = a.src[k] - node0;
          gbv[i] = a.mode != MRP_AGG_COPY_MEAN
                       ? *reinterpret_cast<const float2*>(a.gb + ((int64_t)a.eid[k] * a.C + c) * 2)
                       : make_float2(1.f, 0.f);
        }
        if (a.logits && a.mode != MRP_AGG_COPY_MEAN) {
#pragma unroll
          for (int i = 0; i < KC; ++i) gbv[i] = make_float2(sigmoidf(gbv[i].x), sigmoidf(gbv[i].y));
        }
#pragma unroll
        for (int i = 0; i < KC; ++i) {
          const int u = us[i];
          if (k0 + i >= end || (unsigned)u >= (unsigned)n) continue;  // past v's list / leaves the graph
          mask |= 1u << u;
          if (BWD) {
            Ga[cl * SZ + u * NTP + v] += s * gbv[i].x;
          } else {
            Ga[cl * SZ + v * NTP + u] += gbv[i].x;
            Gb[cl * SZ + v * NTP + u] += gbv[i].y;
          }
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
}

// ---------------------------------------------------------------------------
// Prologue, COMPLETE graphs of exactly NT nodes: the gamma/beta of LDS slot (cl, v, u) is one
// load at an arithmetic edge id, so the whole tile set is one round of independent loads.
// Split in two so the caller can issue its first feature loads between them:
//   complete_fetch : per-thread registers <- gamma/beta of the slots this thread owns
//   complete_store : registers -> LDS (FWD layout [v][u] gamma and beta; BWD layout [u][v]
//                    scaled gamma)
// ---------------------------------------------------------------------------
// Slot t of a COMPLETE prologue -> (channel cl, destination v, source u), channel fastest
// (neighbouring lanes read neighbouring gamma/beta pairs): slot = t / cpb in [v][u] order.  With
// 16-channel workgroups (the 8x8 planes) a 32-lane half of a wave holds 16 channels x 2 slots, and a
// 68-float tile stride puts channels c and c + 8 on the same dword bank (mod 32, the ds_write_b32
// banking), so there (a) TR: consecutive slots step v, i.e. along a row of the backward's
// transposed [u][v] tiles (the forward's [v][u] tiles: u), and (b) within each aligned group of 4
// slots channels 8-15 take the other two slots than channels 0-7 (slot ^ 2) — every half-wave's
// stores then cover 32 banks (rocprof r03: 9 % of the forward's and 22 % of the backward's LDS
// cycles were conflicts at 8x8 planes without it).
template <int NT, bool TR>
__device__ __forceinline__ void complete_slot(const AggArgs& a, int t, int& cl, int& v, int& u) {
  int slot;
  split_channel(a, t, cl, slot);
  if ((NT * NT) % 4 == 0 && a.cpb == 16) {
    slot ^= (cl & 8) >> 2;
    const int hi = slot / NT, lo = slot - hi * NT;
    v = TR ? lo : hi;
    u = TR ? hi : lo;
  } else {
    v = slot / NT;
    u = slot - v * NT;
  }
}

// The backward epilogue's slot order.  16-channel workgroups: bits 3 and 5 of t swapped, so a
// 32-lane half holds 8 channels x 4 consecutive slots (one destination v) and its reads of the Gram
// [v][u], of S[v] (SLS) and of the per-slot sigmoid values (sg_index) each cover distinct banks;
// other channel counts: the prologue's order.
template <int NT>
__device__ __forceinline__ void complete_epi_slot(const AggArgs& a, int t, int& cl, int& v, int& u) {
  if ((NT * NT) % 4 == 0 && a.cpb == 16) {
    const int ts = (t & ~0x28) | ((t & 8) << 2) | ((t & 32) >> 2);
    cl = ts & 15;
    const int slot = ts >> 4;
    v = slot / NT;
    u = slot - v * NT;
  } else {
    complete_slot<NT, true>(a, t, cl, v, u);
  }
}
// Index of slot (cl, v, u) in the backward's per-slot sigmoid buffer.  16 channels: slot-major with
// the channel XORed with 8 on every other pair of sources, so both the prologue's 16-lane stores (one
// slot, 16 channels) and the epilogue's 32-lane reads (8 channels x 4 sources) are conflict-free;
// otherwise the prologue's t.
template <int NT>
__device__ __forceinline__ int sg_index(const AggArgs& a, int cl, int v, int u) {
  const int slot = v * NT + u;
  return slot * a.cpb + (((NT * NT) % 4 == 0 && a.cpb == 16) ? cl ^ (((slot >> 1) & 1) << 3) : cl);
}

template <int NT>
struct CompleteSlots {
  static constexpr int kSlots = NT * NT;
  static constexpr int kPer = (kMaxChanPerBlock * kSlots + kBlock - 1) / kBlock;  // max slots per thread
};

template <int NT, bool TR>
__device__ __forceinline__ void complete_fetch(const AggArgs& a, int64_t ebase, int c0, int base, float2* reg) {
  constexpr int S = CompleteSlots<NT>::kSlots;
  const int tot = a.cpb * S;
#pragma unroll
  for (int r = 0; r < CompleteSlots<NT>::kPer; ++r) {
    const int t = base + threadIdx.x + r * blockDim.x;
    float2 val = make_float2(0.f, 0.f);
    if (t < tot) {
      int cl, v, u;
      complete_slot<NT, TR>(a, t, cl, v, u);
      const int c = c0 + cl;
      if (u != v && c < a.C) {
        if (a.mode == MRP_AGG_COPY_MEAN) {
          val = make_float2(1.f, 0.f);
        } else {
          // raw value: the sigmoid (logits) is applied in complete_store, so the caller's feature
          // loads issue before this load has to return
          val = *reinterpret_cast<const float2*>(a.gb + (complete_eid(ebase, NT, u, v) * a.C + c) * 2);
        }
      }
    }
    reg[r] = val;
  }
}

template <int NT, bool BWD>
__device__ __forceinline__ void complete_store(const AggArgs& a, int base, const float2* reg, float* Ga, float* Gb,
                                               float2* Sg = nullptr) {
  constexpr int S = CompleteSlots<NT>::kSlots;
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  const int tot = a.cpb * S;
  const float s = ((BWD && a.mode != MRP_AGG_FILM_SUM && NT > 1) ? 1.f / (float)(NT - 1) : 1.f) *
                  (BWD ? a.agg_scale : 1.f);
  const bool act = a.logits && a.mode != MRP_AGG_COPY_MEAN;
#pragma unroll
  for (int r = 0; r < CompleteSlots<NT>::kPer; ++r) {
    const int t = base + threadIdx.x + r * blockDim.x;
    if (t < tot) {
      int cl, v, u;
      complete_slot<NT, BWD>(a, t, cl, v, u);
      float2 w = reg[r];
      // (diagonal and out-of-range slots hold 0 and turn into 0.5 here: never read)
      if (act) w = make_float2(sigmoidf(w.x), sigmoidf(w.y));
      if (BWD) {
        Ga[cl * SZ + u * NTP + v] = s * w.x;
        // sigmoid(z) of slot (cl, v, u), reused by the epilogue (slot-major: its lane order differs)
        if (Sg != nullptr) Sg[sg_index<NT>(a, cl, v, u)] = w;
      } else {
        Ga[cl * SZ + v * NTP + u] = w.x;
        Gb[cl * SZ + v * NTP + u] = w.y;
      }
    }
  }
}

// Remaining slot chunks (only when a small workgroup owns more than kPer slots per thread).
template <int NT, bool BWD>
__device__ __forceinline__ void complete_rest(const AggArgs& a, int64_t ebase, int c0, float* Ga, float* Gb,
                                              float2* Sg = nullptr) {
  const int chunk = CompleteSlots<NT>::kPer * blockDim.x;
  for (int base = chunk; base < a.cpb * CompleteSlots<NT>::kSlots; base += chunk) {
    float2 reg[CompleteSlots<NT>::kPer];
    complete_fetch<NT, BWD>(a, ebase, c0, base, reg);
    complete_store<NT, BWD>(a, base, reg, Ga, Gb, Sg);
  }
}

// ---------------------------------------------------------------------------
// Forward.  out[v] = reduce_{e=(u->v)} (gamma_e * x_u + beta_e), zero if deg v == 0.
// ---------------------------------------------------------------------------
// MODE >= 0: the FiLM mode as a compile-time constant (the hot path: COMPLETE, MRP_AGG_FILM_MEAN,
// N <= 8): no per-term select between the modes, and the mean's division by N - 1 as the exact
// three-instruction quotient (fast_math.hpp) for a whole slice at once.  MODE = -1: mode at run time.
template <int NT, int VEC, bool COMPLETE, int MODE = -1>
__global__ void __launch_bounds__(kBlock) film_fwd(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  constexpr bool kBatchDiv = COMPLETE && MODE == MRP_AGG_FILM_MEAN && NT >= 2;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Ga = smem;
  float* Gb = Ga + a.cpb * SZ;
  float* degf = Gb + a.cpb * SZ;
  unsigned* emask = reinterpret_cast<unsigned*>(degf + NTP);

  // psplit > 1: the plane is cut into psplit contiguous segments, one workgroup each.  The launcher
  // picks psplit so that every lane owns ONE slice: many short workgroups stream like a plain
  // grid-stride copy (178 vs 210 us at the bench size, tools/fwd_lab.hip), and the prologue they
  // repeat is a few KiB of gamma/beta from L2.
  const int ps = a.psplit > 1 ? a.psplit : 1;
  const int item = blockIdx.x / ps;
  const int seg = blockIdx.x - item * ps;
  const int b = item / a.ncb;
  const int cb = item - b * a.ncb;
  const int seglen = (a.PV + ps - 1) / ps;
  const int jbeg = seg * seglen;
  const int jend = min(a.PV, jbeg + seglen);
  const int node0 = COMPLETE ? b * NT : a.goff[b];
  const int n = COMPLETE ? NT : min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;  // whole workgroup: empty graph
  const int c0 = cb * a.cpb;

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  const bool active = grp < a.cpb && c < a.C;
  // uniform per-graph/channel-block bases, per-lane 32-bit byte offsets (see at_bytes)
  const float* xb = a.x + (int64_t)node0 * a.xs + (int64_t)c0 * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c0 * a.P;
  const uint32_t lane_plane = (uint32_t)grp * (uint32_t)a.P * 4u;

  // prologue part 1 (COMPLETE): gamma/beta into registers
  float2 reg[CompleteSlots<NT>::kPer];
  const int64_t ebase = (int64_t)b * NT * (NT - 1);
  if (COMPLETE) complete_fetch<NT, false>(a, ebase, c0, 0, reg);
  // first slice of the sweep, issued before the weight tiles are needed
  int j = jbeg + li;
  // element k of every source's slice in one NT-wide vector value: when the compiler keeps a
  // neighbour loop rolled (CSR, NT > 8) the source index is a dynamic extract from registers,
  // not an indexed private array (which spilled 272 B/lane to scratch at NT = 16)
  typedef float vnt __attribute__((ext_vector_type(NT <= 4 ? 4 : (NT <= 8 ? 8 : 16))));
  vnt xv[VEC];
  auto load_slice = [&](int jj) {
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int uu = u < n ? u : n - 1;  // clamp (ragged batch); never used for output
      const Frag<VEC> f = load_frag<VEC, true>(at_bytes(xb + (int64_t)uu * a.xs, lane_plane + (uint32_t)jj * VEC * 4u));
#pragma unroll
      for (int k = 0; k < VEC; ++k) xv[k][u] = f.v[k];
    }
  };
  if (active && j < jend) load_slice(j);
  // prologue part 2: tiles into LDS
  if (COMPLETE) {
    complete_store<NT, false>(a, 0, reg, Ga, Gb);
    complete_rest<NT, false>(a, ebase, c0, Ga, Gb);
  } else
    build_tiles_csr<NT, false>(a, node0, n, c0, Ga, Gb, degf, emask);
  __syncthreads();
  if (!active) return;

  const bool film = MODE >= 0 ? MODE != MRP_AGG_COPY_MEAN : a.mode != MRP_AGG_COPY_MEAN;
  const bool mean = MODE >= 0 ? MODE != MRP_AGG_FILM_SUM : a.mode != MRP_AGG_FILM_SUM;
  // CSR: neighbour masks and in-degrees are channel-independent -> wave-uniform; read them from LDS
  // once into scalar registers instead of once per slice
  unsigned emv[COMPLETE ? 1 : NT];
  float degv[COMPLETE ? 1 : NT];
  if constexpr (!COMPLETE) {
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      emv[v] = __builtin_amdgcn_readfirstlane(emask[v]);
      degv[v] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, degf[v])));
    }
  }

  while (j < jend) {
    const int64_t off = (int64_t)j * VEC;
    const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
    // Re-read the tiles from LDS every slice: laundering the tile offset stops the compiler from
    // hoisting all N*N weights into registers (which would cost occupancy or spill).
    int tile = grp * SZ;
    asm volatile("" : "+v"(tile));
    const float* A = Ga + tile;
    const float* Bt = Gb + tile;
    // kBatchDiv: the sums of a group of VG destinations are divided as one set (one range check)
    constexpr int VG = kBatchDiv ? (NT < 4 ? NT : 4) : 1;
    Frag<VEC> accs[VG];
    float mn = __builtin_inff(), mx = 0.f;
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      if (!COMPLETE && v >= n) break;
      // neighbour mask of v: compile-time for COMPLETE, else channel-independent -> wave-uniform
      unsigned em;
      if constexpr (COMPLETE)
        em = ((1u << NT) - 1u) & ~(1u << v);
      else
        em = emv[v];
      Frag<VEC> acc;
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
#pragma unroll
      for (int u4 = 0; u4 < NTP; u4 += 4) {
        if (!COMPLETE && ((em >> u4) & 15u) == 0u) continue;  // no neighbour in this quad: skip its LDS reads
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
            const float m = film ? __fadd_rn(__fmul_rn(ga, xv[k][u]), gbv) : __fmul_rn(ga, xv[k][u]);
            acc.v[k] = __fadd_rn(acc.v[k], m);
          }
        }
      }
      if constexpr (kBatchDiv) {
        accs[v % VG] = acc;
#pragma unroll
        for (int k = 0; k < VEC; ++k) {
          mn = fminf(mn, __builtin_fabsf(acc.v[k]));
          mx = fmaxf(mx, __builtin_fabsf(acc.v[k]));
        }
        if (v % VG != VG - 1 && v != NT - 1) continue;
        const int v0 = v - v % VG;
        if (__builtin_expect(!mrp_math::div_fast_ok(mn, mx), 0)) {
#pragma unroll
          for (int i = 0; i < VG; ++i)
#pragma unroll
            for (int k = 0; k < VEC; ++k) accs[i].v[k] = accs[i].v[k] / (float)(NT - 1);
        } else {
#pragma unroll
          for (int i = 0; i < VG; ++i)
#pragma unroll
            for (int k = 0; k < VEC; ++k) accs[i].v[k] = mrp_math::div_fast<NT - 1>(accs[i].v[k]);
        }
        mn = __builtin_inff();
        mx = 0.f;
#pragma unroll
        for (int i = 0; i < VG; ++i) {
          if (v0 + i > v) break;
          if (a.epi) {
            float xself[VEC];
#pragma unroll
            for (int k = 0; k < VEC; ++k) xself[k] = xv[k][v0 + i];
            apply_epilogue<VEC>(a, accs[i].v, xself, node0 + v0 + i, c, off);
          }
          store_frag<VEC, true>(at_bytes(ob + (int64_t)(v0 + i) * a.os, lane_off), accs[i]);
        }
        continue;
      }
      float d;
      if constexpr (COMPLETE)
        d = (float)(NT - 1);
      else
        d = degv[v];
      if (mean && d > 0.f) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc.v[k] = acc.v[k] / d;
      }
      if (a.epi) {
        float xself[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) xself[k] = xv[k][v];
        apply_epilogue<VEC>(a, acc.v, xself, node0 + v, c, off);
      }
      store_frag<VEC, true>(at_bytes(ob + (int64_t)v * a.os, lane_off), acc);
    }

    if (a.xc != nullptr) {
      // cat((x, aggregate), 1): the slices of x are in registers already; writing them here saves
      // the separate copy's read of x
      float* xcb = a.xc + (int64_t)node0 * a.xcs + (int64_t)c0 * a.P;
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        if (u >= n) break;
        Frag<VEC> f;
#pragma unroll
        for (int k = 0; k < VEC; ++k) f.v[k] = xv[k][u];
        store_frag<VEC, true>(at_bytes(xcb + (int64_t)u * a.xcs, lane_off), f);
      }
    }
    j += a.lpc;
    if (j < jend) load_slice(j);
  }
}

// ---------------------------------------------------------------------------
// Forward for REGULAR graphs (every node has exactly K = a.kdeg <= KMAX in-edges: k-NN frames).
// Per-edge-slot weights instead of the dense N x N tiles: slot (v, j) is v's j-th in-edge in CSR
// (= edge id = DGL mailbox) order, its (gamma, beta) for the workgroup's channels and its local
// source u(v, j) sit in LDS.  The sweep makes exactly K multiply-adds per destination and element,
// with no per-neighbour branches: u(v, j) is the same for the whole workgroup, so x_u is a
// wave-uniform dynamic index into the slice registers (lowered to M0-relative moves, no scratch).
// Summation order = slot order, as the mailbox mean: acc = fl(acc + fl(fl(gamma x_u) + beta)),
// out = fl(acc / K).  Like film_fwd with COMPLETE graphs, the plane may be split over psplit
// workgroups (the prologue is two rounds of loads: edge ids, then gamma/beta, both in flight
// together with the first slice).
// ---------------------------------------------------------------------------
//
// KC > 0: the in-degree is the compile-time KC (a power of two; the launcher checks a.kdeg == KC) and
// the mode is a mean: the slot loop has no exit test and the mean's division is the exact product
// by 1/KC (x * 2^-k is the correctly rounded x / 2^k), instead of the ~10-instruction IEEE division
// per destination and element.  KC = 0: runtime K and mode.
template <int NT, int KMAX, int VEC, int KC = 0>
__global__ void __launch_bounds__(kBlock) film_fwd_regular(AggArgs a) {
  static_assert(KC == 0 || (KC <= KMAX && (KC & (KC - 1)) == 0), "compile-time degree: a power of two");
  constexpr int NS = NT * KMAX;
  constexpr int WS = NS + 2;     // per-channel stride of the slot weights (float2), padded 4 banks
  constexpr int WPD = KMAX / 4;  // 32-bit words of packed 8-bit slot sources per destination
  static_assert(KMAX % 4 == 0, "slots are packed four to a word");
  extern __shared__ float4 smem_f4[];
  float2* Wl = reinterpret_cast<float2*>(smem_f4);                  // [cpb][WS] (gamma, beta) per slot
  unsigned* slot_u = reinterpret_cast<unsigned*>(Wl + a.cpb * WS);  // [NT * WPD] packed local sources

  const int ps = a.psplit > 1 ? a.psplit : 1;
  const int item = blockIdx.x / ps;
  const int seg = blockIdx.x - item * ps;
  const int b = item / a.ncb;
  const int cb = item - b * a.ncb;
  const int seglen = (a.PV + ps - 1) / ps;
  const int jbeg = seg * seglen;
  const int jend = min(a.PV, jbeg + seglen);
  const int node0 = a.goff[b];
  const int n = min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;
  const int K = KC > 0 ? KC : a.kdeg;

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  const bool active = grp < a.cpb && c < a.C;
  // uniform per-graph/channel-block bases, per-lane 32-bit byte offsets (see at_bytes)
  const float* xb = a.x + (int64_t)node0 * a.xs + (int64_t)c0 * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c0 * a.P;
  const uint32_t lane_plane = (uint32_t)grp * (uint32_t)a.P * 4u;

  // First slice's loads, issued before the prologue's two dependent rounds.  Element k of every
  // source's slice lives in one NT-wide vector value, so the wave-uniform source index is a dynamic
  // extract from a register tuple (s_set_gpr_idx / v_movrels), not an indexed private array.
  typedef float vnt __attribute__((ext_vector_type(NT <= 8 ? 8 : 16)));
  int j = jbeg + li;
  vnt xs[VEC];
  auto load_slice = [&](int jj) {
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int uu = u < n ? u : n - 1;
      const Frag<VEC> f = load_frag<VEC, true>(at_bytes(xb + (int64_t)uu * a.xs, lane_plane + (uint32_t)jj * VEC * 4u));
#pragma unroll
      for (int k = 0; k < VEC; ++k) xs[k][u] = f.v[k];
    }
  };

  // Prologue.  Loads retire in issue order (vmcnt), so whatever the prologue waits for must be
  // issued before the first slice's loads, or waiting for it waits for the slices too.  Order:
  // slot sources and edge ids -> first slice -> gamma/beta (need only the edge ids) -> LDS, one
  // barrier.  Every thread fetches the edge ids of its own (channel, slot) items (v's CSR row is
  // [K v, K (v+1)) for REGULAR graphs, so no indptr), so no barrier sits between the two rounds.
  constexpr int IPT = 2;  // (channel, slot) items per thread fetched ahead of the slice (the rest after)
  const int nitem = a.cpb * NS;
  const bool film = a.mode != MRP_AGG_COPY_MEAN;
  auto slot_eid = [&](int t, int& cl, int& slot) -> int {
    split_channel(a, t, cl, slot);  // channel fastest: neighbouring lanes read neighbouring pairs
    const int v = slot / KMAX, jj = slot - v * KMAX;
    if (t >= nitem || v >= n || jj >= K || c0 + cl >= a.C) return -1;
    return a.eid[(node0 + v) * K + jj];
  };
  auto fetch_w = [&](int e, int cl) -> float2 {
    if (e < 0) return make_float2(0.f, 0.f);     // empty slot: multiply by 0, add 0
    if (!film) return make_float2(1.f, 0.f);     // gamma 1, beta 0: fl(fl(1*x) + 0) = x
    return *reinterpret_cast<const float2*>(a.gb + ((int64_t)e * a.C + c0 + cl) * 2);
  };
  auto store_w = [&](float2 w, int e, int cl, int slot) {
    if (e >= 0 && film && a.logits) w = make_float2(sigmoidf(w.x), sigmoidf(w.y));
    Wl[cl * WS + slot] = w;
  };
  // the graph's slot sources (channel-independent), WPD words of four 8-bit sources per destination;
  // thread t builds word t (its loads issued here, ahead of the slice) and, in workgroups narrower
  // than NT * WPD threads (one channel of a small plane), words t + blockDim.x, ... after the slice
  const bool has_word = threadIdx.x < NT * WPD;
  auto word_srcs = [&](int wi, int (&sr)[4]) {
    const int v = wi / WPD, q = wi - v * WPD;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int jj = q * 4 + i;
      sr[i] = v < n && jj < K ? a.src[(node0 + v) * K + jj] - node0 : 0;
    }
  };
  auto pack_word = [&](const int (&sr)[4]) {
    unsigned word = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // a source outside the graph is rejected on the host; clamp it anyway (in-bounds register index)
      const int u = (unsigned)sr[i] < (unsigned)n ? sr[i] : 0;
      word |= (unsigned)u << (8 * i);
    }
    return word;
  };
  int srcs[4];
  if (has_word) word_srcs(threadIdx.x, srcs);
  int ie[IPT];  // (channel, slot) of an item are recomputed below rather than held across the slice
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    int cl, slot;
    ie[i] = slot_eid(threadIdx.x + i * blockDim.x, cl, slot);
  }
  if (active && j < jend) load_slice(j);
  float2 iw[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    int cl, slot;
    split_channel(a, threadIdx.x + i * blockDim.x, cl, slot);
    iw[i] = fetch_w(ie[i], cl);
  }
  if (has_word) slot_u[threadIdx.x] = pack_word(srcs);
  for (int wi = threadIdx.x + blockDim.x; wi < NT * WPD; wi += blockDim.x) {  // narrow workgroups only
    int sr[4];
    word_srcs(wi, sr);
    slot_u[wi] = pack_word(sr);
  }
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    int cl, slot;
    split_channel(a, threadIdx.x + i * blockDim.x, cl, slot);
    if (threadIdx.x + i * blockDim.x < nitem) store_w(iw[i], ie[i], cl, slot);
  }
  for (int t = threadIdx.x + IPT * blockDim.x; t < nitem; t += blockDim.x) {  // narrow workgroups only
    int cl, slot;
    const int e = slot_eid(t, cl, slot);
    store_w(fetch_w(e, cl), e, cl, slot);
  }
  __syncthreads();
  if (!active) return;

  const bool mean = a.mode != MRP_AGG_FILM_SUM;
  const float d = (float)K;
  while (j < jend) {
    const int64_t off = (int64_t)j * VEC;
    const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
    // every destination row is computed (full unroll); rows past the graph's nodes are not stored
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      int wbase = grp * WS;  // laundered: weights stay in LDS (broadcast reads), not hoisted
      asm volatile("" : "+v"(wbase));
      const float2* Wc = Wl + wbase;
      unsigned uw[WPD];
#pragma unroll
      for (int q = 0; q < WPD; ++q) uw[q] = __builtin_amdgcn_readfirstlane(slot_u[v * WPD + q]);
      float acc[VEC];
#pragma unroll
      for (int k = 0; k < VEC; ++k) acc[k] = 0.f;
#pragma unroll
      for (int jj = 0; jj < (KC > 0 ? KC : KMAX); ++jj) {
        if (KC == 0 && jj >= K) break;  // wave-uniform
        const int u = (uw[jj >> 2] >> (8 * (jj & 3))) & 0xffu;
        const float2 w = Wc[v * KMAX + jj];
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc[k] = __fadd_rn(acc[k], __fadd_rn(__fmul_rn(w.x, xs[k][u]), w.y));
      }
      if constexpr (KC > 0) {
        constexpr float r = 1.0f / (float)KC;  // exact: KC is a power of two
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc[k] = __fmul_rn(acc[k], r);
      } else if (mean) {
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc[k] = acc[k] / d;
      }
      if (a.epi) {
        float xself[VEC];
#pragma unroll
        for (int k = 0; k < VEC; ++k) xself[k] = xs[k][v];
        apply_epilogue<VEC>(a, acc, xself, node0 + v, c, off);
      }
      if (v < n) {
        Frag<VEC> o;
#pragma unroll
        for (int k = 0; k < VEC; ++k) o.v[k] = acc[k];
        store_frag<VEC, true>(at_bytes(ob + (int64_t)v * a.os, lane_off), o);
      }
    }
    if (a.xc != nullptr) {
      float* xcb = a.xc + (int64_t)node0 * a.xcs + (int64_t)c0 * a.P;
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        if (u >= n) break;
        Frag<VEC> f;
#pragma unroll
        for (int k = 0; k < VEC; ++k) f.v[k] = xs[k][u];
        store_frag<VEC, true>(at_bytes(xcb + (int64_t)u * a.xcs, lane_off), f);
      }
    }
    j += a.lpc;
    if (j < jend) load_slice(j);
  }
}

// ---------------------------------------------------------------------------
// Backward, grad_x only (used for NT > 8, where the fused kernel's Gram accumulators would not
// fit in registers):  grad_x[u] = sum_v Wt[u][v] * G[v].
// ---------------------------------------------------------------------------
template <int NT, int VEC, bool COMPLETE, bool DXB>
__global__ void __launch_bounds__(kBlock) film_bwd_dx(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Wt = smem;
  float* sc = Wt + a.cpb * SZ;

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = COMPLETE ? b * NT : a.goff[b];
  const int n = COMPLETE ? NT : min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;

  if (COMPLETE) {
    float2 reg[CompleteSlots<NT>::kPer];
    complete_fetch<NT, true>(a, (int64_t)b * NT * (NT - 1), c0, 0, reg);
    complete_store<NT, true>(a, 0, reg, Wt, nullptr);
    complete_rest<NT, true>(a, (int64_t)b * NT * (NT - 1), c0, Wt, nullptr);
  } else {
    build_tiles_csr<NT, true>(a, node0, n, c0, Wt, nullptr, sc, nullptr);
  }
  __syncthreads();

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  if (grp >= a.cpb || c >= a.C) return;

  // uniform bases, per-lane 32-bit byte offsets (at_bytes); slices as NT-wide vectors (no scratch)
  const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c0 * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c0 * a.P;
  const float* dxbase = a.dxb != nullptr ? a.dxb + (int64_t)node0 * a.dxbs + (int64_t)c0 * a.P : nullptr;
  const uint32_t lane_plane = (uint32_t)grp * (uint32_t)a.P * 4u;
  typedef float vnt __attribute__((ext_vector_type(NT <= 4 ? 4 : (NT <= 8 ? 8 : 16))));

  for (int j = li; j < a.PV; j += a.lpc) {
    const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
    int tile = grp * SZ;  // laundered: keep the weights in LDS, not hoisted into registers
    asm volatile("" : "+v"(tile));
    const float* W = Wt + tile;
    vnt gv[VEC];
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      const int vv = v < n ? v : n - 1;
      const Frag<VEC> f = load_frag<VEC, true>(at_bytes(gbase + (int64_t)vv * a.gs, lane_off));
#pragma unroll
      for (int k = 0; k < VEC; ++k) gv[k][v] = f.v[k];
    }
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      if (!COMPLETE && u >= n) break;
      Frag<VEC> acc;
      if (DXB) {  // grad_x_base: a separate instantiation (it costs registers)
        acc = load_frag<VEC, true>(at_bytes(dxbase + (int64_t)u * a.dxbs, lane_off));
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
      }
      if (a.self_scale != 0.f) {  // residual epilogue: d out / d x[u] includes self_scale
#pragma unroll
        for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(a.self_scale, gv[k][u], acc.v[k]);
      }
#pragma unroll
      for (int v4 = 0; v4 < NTP; v4 += 4) {
        const f4 w = *reinterpret_cast<const f4*>(W + u * NTP + v4);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int v = v4 + q;
          if (v >= NT) break;
          if (COMPLETE && v == u) continue;
#pragma unroll
          for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(w[q], gv[k][v], acc.v[k]);
        }
      }
      store_frag<VEC, true>(at_bytes(ob + (int64_t)u * a.os, lane_off), acc);
    }
  }
}

// Cross-lane move with a DPP control (no LDS traffic).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xf, 0xf, true));
}

// Reduce a value over the lpc lanes of one channel group (lpc is a power of two <= 64); every lane
// of the group ends with the sum.  Butterfly: xor 1 and xor 2 by quad_perm, 4 <-> 4 by
// row_half_mirror, 8 <-> 8 by row_mirror (all DPP modifiers on the add), then xor 16 / xor 32 by
// ds_bpermute.  Steps wider than the group are skipped by a uniform branch.
template <int L>
__device__ __forceinline__ float group_sum(float x) {
  if constexpr (L >= 2) x += dpp_mov<0xB1>(x);   // quad_perm [1,0,3,2]
  if constexpr (L >= 4) x += dpp_mov<0x4E>(x);   // quad_perm [2,3,0,1]
  if constexpr (L >= 8) x += dpp_mov<0x141>(x);  // row_half_mirror
  if constexpr (L >= 16) x += dpp_mov<0x140>(x);  // row_mirror
  if constexpr (L >= 32) x += __shfl_xor(x, 16, 64);
  if constexpr (L >= 64) x += __shfl_xor(x, 32, 64);
  return x;
}

// Reduce-scatter of 64 values over an aligned group of L = 2^t lanes (L <= 64): on return lane gl of
// the group holds in v[0 .. 64 / L) the group sums of values [gl 64 / L, (gl + 1) 64 / L).  At each
// step a lane keeps one half of its current range and sends its partner the other, so the sums cost
// 64 - 64 / L exchanges instead of the all-reduce's 64 log2 L (group_sum on every value).  Steps run
// from the group's top lane bit down — xor 32 and xor 16 by ds_bpermute, then row_mirror,
// row_half_mirror and the two quad perms by DPP: a mirror pairs lanes that differ in the low bits
// too, but the range a lane holds depends only on the bits above the step's, which a mirror keeps.
// Each sum is formed on one lane in a fixed order: deterministic.
template <int CNT, int BIT>
__device__ __forceinline__ void rs_step(float (&v)[64], int lane) {
  constexpr int H = CNT / 2;
  const bool up = (lane >> BIT) & 1;
#pragma unroll
  for (int j = 0; j < H; ++j) {  // element j and j + H only: one pass, few values live at once
    const float send = up ? v[j] : v[j + H];
    float r;
    if constexpr (BIT == 5)
      r = __shfl_xor(send, 32, 64);
    else if constexpr (BIT == 4)
      r = __shfl_xor(send, 16, 64);
    else if constexpr (BIT == 3)
      r = dpp_mov<0x140>(send);  // row_mirror: i <-> 15 - i
    else if constexpr (BIT == 2)
      r = dpp_mov<0x141>(send);  // row_half_mirror: i <-> 7 - i
    else if constexpr (BIT == 1)
      r = dpp_mov<0x4E>(send);  // quad_perm [2,3,0,1]
    else
      r = dpp_mov<0xB1>(send);  // quad_perm [1,0,3,2]
    v[j] = (up ? v[j + H] : v[j]) + r;
  }
}

template <int L>
__device__ __forceinline__ void reduce_scatter64(float (&v)[64], int lane) {
  // the step at lane bit b follows the log2(L) - 1 - b steps above it: 128 2^b / L values left
  if constexpr (L >= 64) rs_step<128 * 32 / L, 5>(v, lane);
  if constexpr (L >= 32) rs_step<128 * 16 / L, 4>(v, lane);
  if constexpr (L >= 16) rs_step<128 * 8 / L, 3>(v, lane);
  if constexpr (L >= 8) rs_step<128 * 4 / L, 2>(v, lane);
  if constexpr (L >= 4) rs_step<128 * 2 / L, 1>(v, lane);
  if constexpr (L >= 2) rs_step<128 / L, 0>(v, lane);
}

// film_bwd_fused, complete 8-node graphs: reduce-scatter the lane's 64 values (Gram D[i][u] at i 8 + u,
// S[i] in the diagonal slot) over the group's L lanes, then each lane of an active group stores its
// 64 / L sums: S[i] to sl[i], D[i][u] to dl[i NTP + u]
// film_bwd_fused, complete 8-node graphs, planes of >= 64 lanes: reduce-scatter the lane's 64 values
// (Gram D[i][u] at i 8 + u, S[i] in the diagonal slot) over the wave, then lane l of an active group
// stores sum l: S[i] to sl[i], D[i][u] to dl[i NTP + u]
template <int L, int NTP>
__device__ __forceinline__ void rs_store(float (&vals)[64], int li, bool active, float* sl, float* dl) {
  static_assert(L == 64, "one sum per lane");
  reduce_scatter64<L>(vals, threadIdx.x & 63);
  if (!active) return;
  const int i = (li & 63) >> 3, u = li & 7;
  *(i == u ? sl + i : dl + i * NTP + u) = vals[0];
}

// Call f(std::integral_constant<int, L>) with L = lpc: the lane count is wave-uniform but only
// known at run time, so branch once here rather than once per reduced value (a runtime-width
// butterfly costs a scalar compare and branch per step per value).
template <class F>
__device__ __forceinline__ void with_lanes(int lpc, F&& f) {
  switch (lpc) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 8: f(std::integral_constant<int, 8>{}); break;
    case 16: f(std::integral_constant<int, 16>{}); break;
    case 32: f(std::integral_constant<int, 32>{}); break;
    default: f(std::integral_constant<int, 64>{}); break;
  }
}

// ---------------------------------------------------------------------------
// Backward, fused: one sweep reads G and x once, writes grad_x (if VB == NT and want_dx) and
// accumulates the per-channel Gram D[v][u] = sum_p G_v * x_u and S[v] = sum_p G_v for a block of
// VB destination rows; then writes
//   grad_gb[e, c] = (s_v * D[v][u], s_v * S[v])    for every edge e = (u -> v).
// For NT > 8 the kernel runs with VB = 4 and loops over destination blocks (x re-read from L2).
// ---------------------------------------------------------------------------
// PRE2: lanes own exactly two slices (the launcher checks PV == 2 lpc) and both are loaded before
// the prologue, into two register sets, so the second slice's loads are in flight while the first
// is reduced instead of being issued after it.  At N = 8 the kernel runs 2 waves per SIMD either
// way (192 VGPRs with one set), so the second set costs no occupancy.
template <int NT, int VB, int VEC, bool COMPLETE, bool DXB = false, int MINW = 1, bool PRE2 = false>
__global__ void __launch_bounds__(kBlock, MINW) film_bwd_fused(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  constexpr bool kOnePass = VB == NT;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  // lpc > 64: a channel plane spans wpc = lpc/64 waves (one slice per lane on big planes); each
  // wave reduces its own Gram partial and the epilogue adds the wpc partials in wave order
  const int wpc = a.lpc > 64 ? a.lpc >> 6 : 1;
  const int npg = a.cpb * wpc;   // Gram partials
  constexpr int SLS = Tile<NT>::SLS;
  float* Wt = smem;              // [cpb][NT][NTP]   scaled, transposed
  float* Dl = Wt + a.cpb * SZ;   // [npg][NT][NTP]   Gram (unscaled)
  float* Sl = Dl + npg * SZ;     // [npg][SLS]       sum_p G_v
  float* sc = Sl + npg * SLS;    // [NTP]            s_v
  // COMPLETE with logits: sigmoid(z) of every slot, (NT x NT x cpb) float2, slot-major,
  // so the epilogue's sigmoid backward does not fetch z from HBM a second time
  float2* Sg = (COMPLETE && a.logits) ? reinterpret_cast<float2*>(sc + NTP) : nullptr;

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = COMPLETE ? b * NT : a.goff[b];
  const int n = COMPLETE ? NT : min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  const bool active = grp < a.cpb && c < a.C;

  // uniform per-graph/channel-block bases, per-lane 32-bit byte offsets (see at_bytes)
  const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c0 * a.P;
  const float* xbase = a.x + (int64_t)node0 * a.xs + (int64_t)c0 * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c0 * a.P;
  const float* dxbase = a.dxb != nullptr ? a.dxb + (int64_t)node0 * a.dxbs + (int64_t)c0 * a.P : nullptr;
  const uint32_t lane_plane = (uint32_t)grp * (uint32_t)a.P * 4u;
  const bool do_dx = kOnePass && a.want_dx;

  // slice fragments: for the one-pass kernel the first slice is loaded before the prologue, so the
  // weight-tile build (one more round trip to HBM) hides under these loads
  Frag<VEC> gv[VB];
  Frag<VEC> xv[NT];
  Frag<VEC> gv2[PRE2 ? VB : 1];
  Frag<VEC> xv2[PRE2 ? NT : 1];
  auto load_into = [&](Frag<VEC>* G, Frag<VEC>* X, int vb, int j) {
    const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
#pragma unroll
    for (int i = 0; i < VB; ++i) {
      const int v = vb + i;
      const int vv = v < n ? v : n - 1;
      G[i] = load_frag<VEC, kOnePass>(at_bytes(gbase + (int64_t)vv * a.gs, lane_off));
    }
    // x's rows, unconditionally: without a gamma/beta gradient (x may be null) they re-read grad_out's
    // rows, unused.  Under `if (a.want_dgb)` the branch's join made hipcc copy the landed registers into
    // place at its end — an s_waitcnt vmcnt(0) between this slice's loads and the next's, so PRE2's second
    // slice set was only requested after the first had arrived (two dependent memory round trips)
    const float* xb = a.want_dgb ? xbase : gbase;
    const int64_t xstride = a.want_dgb ? a.xs : a.gs;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      const int uu = u < n ? u : n - 1;
      X[u] = load_frag<VEC, kOnePass>(at_bytes(xb + (int64_t)uu * xstride, lane_off));
    }
  };
  auto load_slice = [&](int vb, int j) { load_into(gv, xv, vb, j); };

  float2 reg[CompleteSlots<NT>::kPer];
  if (COMPLETE) complete_fetch<NT, true>(a, (int64_t)b * NT * (NT - 1), c0, 0, reg);
  if (kOnePass && active && li < a.PV) load_slice(0, li);
  if (PRE2 && active && li < a.PV) load_into(gv2, xv2, 0, li + a.lpc);
  if (COMPLETE) {
    complete_store<NT, true>(a, 0, reg, Wt, nullptr, Sg);
    complete_rest<NT, true>(a, (int64_t)b * NT * (NT - 1), c0, Wt, nullptr, Sg);
  } else {
    build_tiles_csr<NT, true>(a, node0, n, c0, Wt, nullptr, sc, nullptr);
  }
  __syncthreads();

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
      int j = li;
      if (!kOnePass && j < a.PV) load_slice(vb, j);
      while (j < a.PV) {
        const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
        int tile = grp * SZ;  // laundered: keep the weights in LDS, not hoisted into registers
        asm volatile("" : "+v"(tile));
        const float* W = Wt + tile;
        if (do_dx) {
          // grad_x_base (a separate instantiation: it costs registers): all NT rows requested before the
          // first is needed, so one memory round trip per slice is exposed instead of one per node — not
          // with PRE2, whose second register set leaves no room for them (256 + 30 registers: one wave
          // per SIMD), which loads each row where it adds it
          constexpr bool kPreBase = DXB && !PRE2;
          Frag<VEC> base[kPreBase ? NT : 1];
          if constexpr (kPreBase) {
#pragma unroll
            for (int u = 0; u < NT; ++u) {
              const int uu = u < n ? u : n - 1;
              base[u] = load_frag<VEC, true>(at_bytes(dxbase + (int64_t)uu * a.dxbs, lane_off));
            }
          }
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            if (!COMPLETE && u >= n) break;
            Frag<VEC> acc;
            if constexpr (kPreBase) {
              acc = base[u];
            } else if constexpr (DXB) {
              acc = load_frag<VEC, true>(at_bytes(dxbase + (int64_t)u * a.dxbs, lane_off));
            } else {
#pragma unroll
              for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
            }
            if (a.self_scale != 0.f) {  // residual epilogue (one pass: gv[u] is node u's grad_out)
#pragma unroll
              for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(a.self_scale, gv[u].v[k], acc.v[k]);
            }
#pragma unroll
            for (int v4 = 0; v4 < NTP; v4 += 4) {
              const f4 w = *reinterpret_cast<const f4*>(W + u * NTP + v4);
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                const int v = v4 + q;
                if (v >= NT) break;
                if (COMPLETE && v == u) continue;
#pragma unroll
                for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(w[q], gv[v].v[k], acc.v[k]);
              }
            }
            store_frag<VEC, true>(at_bytes(ob + (int64_t)u * a.os, lane_off), acc);
          }
        }
        if (a.want_dgb) {
#pragma unroll
          for (int i = 0; i < VB; ++i) {
#pragma unroll
            for (int k = 0; k < VEC; ++k) S[i] += gv[i].v[k];
#pragma unroll
            for (int u = 0; u < NT; ++u) {
              if (COMPLETE && kOnePass && u == i) continue;  // not an edge
#pragma unroll
              for (int k = 0; k < VEC; ++k) D[i][u] = fmaf(gv[i].v[k], xv[u].v[k], D[i][u]);
            }
          }
        }
        j += a.lpc;
        if (j < a.PV) {
          if constexpr (PRE2) {  // the second (last) slice is already in registers
#pragma unroll
            for (int i = 0; i < VB; ++i) gv[i] = gv2[i];
#pragma unroll
            for (int u = 0; u < NT; ++u) xv[u] = xv2[u];
          } else {
            load_slice(vb, j);
          }
        }
      }
    }
    bool reduced = false;
    if constexpr (COMPLETE && NT == 8 && VB == 8) {
      // the reference's configuration (complete 8-robot graphs) on planes of >= 64 lanes (32 x 32): the
      // 56 Gram values and 8 S values of the lane (S[i] in the diagonal slot i 8 + i, not an edge)
      // reduce-scattered over the wave, each lane then storing one sum — 63 exchanges instead of the
      // all-reduce's 384 and one store instead of 64 from lane 0 (tools/ab_libs.py: headline backward
      // 278.7 vs 281.8 us, configs[1] 145.0 vs 149.0).  At 8 lanes per plane (8 x 8) the all-reduce
      // below stays: the reduce-scatter measured 4 % slower there (configs[2] 60.0 vs 57.6 us).
      if (a.want_dgb && a.lpc >= 64) {
        __builtin_amdgcn_sched_barrier(0);  // the sweep's registers are free before the reduction starts
        float vals[64];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int u = 0; u < 8; ++u) vals[i * 8 + u] = u == i ? S[i] : D[i][u];
        // li recomputed from the thread id (lpc is a power of two): keeping it live across the sweep
        // pushed the PRE2 instantiations past 256 registers
        const int lir = (int)threadIdx.x & (a.lpc - 1);
        const int pg = wpc > 1 ? grp * wpc + (lir >> 6) : grp;
        rs_store<64, NTP>(vals, lir, active, Sl + pg * SLS, Dl + pg * SZ);
        reduced = true;
      }
    }
    if (!reduced && a.want_dgb) {
      // Reduce across the lanes of each channel group (all lanes of the wave take part in the
      // shuffles; inactive groups contribute zeros to their own group).
      with_lanes(a.lpc, [&](auto lanes) {
        constexpr int L = decltype(lanes)::value;
#pragma unroll
        for (int i = 0; i < VB; ++i) {
          S[i] = group_sum<L>(S[i]);
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            if (COMPLETE && kOnePass && u == i) continue;
            D[i][u] = group_sum<L>(D[i][u]);
          }
        }
      });
      if (active && (wpc > 1 ? (li & 63) : li) == 0) {
        const int pg = wpc > 1 ? grp * wpc + (li >> 6) : grp;
#pragma unroll
        for (int i = 0; i < VB; ++i) {
          const int v = vb + i;
          if (v < NT) {
            Sl[pg * SLS + v] = S[i];
#pragma unroll
            for (int u = 0; u < NT; ++u) Dl[pg * SZ + v * NTP + u] = D[i][u];
          }
        }
      }
    }
  }
  if (!a.want_dgb) return;
  __syncthreads();
  if (COMPLETE) {
    // Per-edge outputs: thread -> (channel fastest, slot (v, u)); arithmetic edge ids.
    const float s = ((a.mode != MRP_AGG_FILM_SUM && NT > 1) ? 1.f / (float)(NT - 1) : 1.f) * a.agg_scale;
    const int64_t ebase = (int64_t)b * NT * (NT - 1);
    for (int t = threadIdx.x; t < a.cpb * NT * NT; t += blockDim.x) {
      int cl, v, u;
      complete_epi_slot<NT>(a, t, cl, v, u);
      const int cc = c0 + cl;
      if (u == v || cc >= a.C) continue;
      float dd = Dl[cl * wpc * SZ + v * NTP + u], ss = Sl[cl * wpc * SLS + v];
      for (int w = 1; w < wpc; ++w) {
        dd += Dl[(cl * wpc + w) * SZ + v * NTP + u];
        ss += Sl[(cl * wpc + w) * SLS + v];
      }
      float2 r = make_float2(s * dd, s * ss);
      const int64_t off = (complete_eid(ebase, NT, u, v) * a.C + cc) * 2;
      if (a.logits) {
        // d z = d(gamma, beta) * sig * (1 - sig), sig = sigmoid(z) kept from the prologue
        const float2 sg = Sg[sg_index<NT>(a, cl, v, u)];
        r = make_float2(r.x * sg.x * (1.f - sg.x), r.y * sg.y * (1.f - sg.y));
      }
      *reinterpret_cast<float2*>(a.dgb + off) = r;
    }
    return;
  }
  // CSR: thread -> (channel fastest, destination v); the in-edges of v are walked in CSR order.
  // Every edge of the graph has exactly one destination here, so each grad_gb element is
  // written once.
  for (int t = threadIdx.x; t < a.cpb * NT; t += blockDim.x) {
    int cl, v;
    split_channel(a, t, cl, v);
    const int cc = c0 + cl;
    if (v >= n || cc >= a.C) continue;
    const int beg = a.indptr[node0 + v];
    const int end = a.indptr[node0 + v + 1];
    const float s = sc[v];
    float ss = Sl[cl * wpc * SLS + v];
    for (int w = 1; w < wpc; ++w) ss += Sl[(cl * wpc + w) * SLS + v];
    const float dbeta = s * ss;
    for (int k = beg; k < end; ++k) {
      const int u = a.src[k] - node0;
      float dgam = 0.f, dbet = 0.f;
      if ((unsigned)u < (unsigned)n) {
        float dd = Dl[cl * wpc * SZ + v * NTP + u];
        for (int w = 1; w < wpc; ++w) dd += Dl[(cl * wpc + w) * SZ + v * NTP + u];
        dgam = s * dd;
        dbet = dbeta;
      }
      const int64_t off = ((int64_t)a.eid[k] * a.C + cc) * 2;
      float2 r = make_float2(dgam, dbet);
      if (a.logits) r = sigmoid_backward(r, *reinterpret_cast<const float2*>(a.gb + off));
      *reinterpret_cast<float2*>(a.dgb + off) = r;
    }
  }
}

// ---------------------------------------------------------------------------
// Backward for REGULAR graphs (every node has exactly K = a.kdeg in-edges, e.g. k-NN), N > 8:
// one sweep like film_bwd_fused, but the Gram is kept per edge slot, D[v][j] = sum_p G_v x_{u(v,j)},
// N*KMAX accumulators instead of N*N.  The source u(v,j) is wave-uniform (the graph is shared by the
// workgroup), so x_{u} is a uniform dynamic index into the register array (s_set_gpr_idx), not a
// scratch access.  grad_x uses the dense transposed tiles.  Multi-edges and self-loops are just
// slots.  Deterministic like the other kernels.
// ---------------------------------------------------------------------------
template <int NT, int KMAX, int VEC, bool DXB>
__global__ void __launch_bounds__(kBlock) film_bwd_regular(AggArgs a) {
  constexpr int SZ = Tile<NT>::SZ;
  constexpr int NTP = Tile<NT>::NTP;
  constexpr int NS = NT * KMAX;  // edge slots
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Wt = smem;                          // [cpb][NT][NTP] scaled, transposed
  float* Dl = Wt + a.cpb * SZ;               // [cpb][NS]
  float* Sl = Dl + a.cpb * NS;               // [cpb][NTP]
  float* sc = Sl + a.cpb * NTP;              // [NTP]
  int* slot_u = reinterpret_cast<int*>(sc + NTP);  // [NS] local source of slot (v, j)
  int* slot_e = slot_u + NS;                       // [NS] edge id of slot (v, j)

  // one workgroup per (graph, channel block), whole planes (a plane split over several workgroups
  // with a second pass adding their partial Grams measured slower at the configs[4] shape: 113-170
  // vs 102.7 us, round 2 — each extra workgroup repeats the prologue of dependent loads)
  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int jbeg = 0;
  const int jend = a.PV;
  const int node0 = a.goff[b];
  const int n = min(a.goff[b + 1] - node0, NT);
  if (n <= 0) return;
  const int c0 = cb * a.cpb;
  const int K = a.kdeg;

  const int grp = threadIdx.x / a.lpc;
  const int li = threadIdx.x - grp * a.lpc;
  const int c = c0 + grp;
  const bool active = grp < a.cpb && c < a.C;
  // uniform per-graph/channel-block bases, per-lane 32-bit byte offsets (see at_bytes)
  const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c0 * a.P;
  const float* xbase = a.x + (int64_t)node0 * a.xs + (int64_t)c0 * a.P;
  float* ob = a.out + (int64_t)node0 * a.os + (int64_t)c0 * a.P;
  const float* dxbase = a.dxb != nullptr ? a.dxb + (int64_t)node0 * a.dxbs + (int64_t)c0 * a.P : nullptr;
  const uint32_t lane_plane = (uint32_t)grp * (uint32_t)a.P * 4u;


  // slice registers; the first slice is loaded before the prologue (slots + transposed weight tiles:
  // dependent loads) so that its latency hides under these loads
  float gv[NT][VEC];
  float xv[NT][VEC];
  auto load_slice = [&](int jj) {
    const uint32_t lane_off = lane_plane + (uint32_t)jj * VEC * 4u;
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      const int vv = v < n ? v : n - 1;
      const Frag<VEC> f = load_frag<VEC, true>(at_bytes(gbase + (int64_t)vv * a.gs, lane_off));
#pragma unroll
      for (int k = 0; k < VEC; ++k) gv[v][k] = f.v[k];
    }
    if (a.want_dgb) {
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int uu = u < n ? u : n - 1;
        const Frag<VEC> f = load_frag<VEC, true>(at_bytes(xbase + (int64_t)uu * a.xs, lane_off));
#pragma unroll
        for (int k = 0; k < VEC; ++k) xv[u][k] = f.v[k];
      }
    }
  };
  int j = jbeg + li;

  // Prologue: one (channel, destination v) item per thread builds column v of the channel's
  // transposed tile, Wt[u][v] = s_v * sum of gamma over v's slots with source u (CSR order, as the
  // CSR builder), and for channel 0 the slot table.  v's CSR row is [K v, K (v+1)) (REGULAR), so the
  // sources and edge ids are one round of loads, issued before the first slice's loads (vmcnt
  // retires in order: waiting for them must not wait for the slices); gamma follows the slice.
  // Every column entry is written, so no zero-fill pass and a single barrier.
  constexpr int IPT = 2;  // items per thread fetched ahead of the slice (the rest, narrow workgroups, after)
  const int nitem = a.cpb * NT;
  float s = a.mode != MRP_AGG_FILM_SUM && K > 0 ? 1.f / (float)K : 1.f;
  s *= a.agg_scale;  // epilogue: grad_out reaches the aggregate scaled
  struct Item {
    int cl, v;
    bool ok;
    int u[KMAX], e[KMAX];
    float gam[KMAX];
  };
  auto item_ids = [&](int t, Item& it) {
    split_channel(a, t, it.cl, it.v);  // channel fastest: neighbouring lanes read neighbouring pairs
    it.ok = t < nitem && it.v < n && c0 + it.cl < a.C;
#pragma unroll
    for (int jj = 0; jj < KMAX; ++jj) {
      const bool on = it.ok && jj < K;
      const int k = (node0 + (on ? it.v : 0)) * K + (on ? jj : 0);
      it.u[jj] = on ? a.src[k] - node0 : -1;
      it.e[jj] = on ? a.eid[k] : -1;
    }
  };
  auto item_gamma = [&](Item& it) {
#pragma unroll
    for (int jj = 0; jj < KMAX; ++jj) {
      float gm = 0.f;
      if (it.e[jj] >= 0) {
        if (a.mode == MRP_AGG_COPY_MEAN) {
          gm = 1.f;
        } else {
          gm = a.gb[((int64_t)it.e[jj] * a.C + c0 + it.cl) * 2];
          if (a.logits) gm = sigmoidf(gm);
        }
      }
      it.gam[jj] = gm;
    }
  };
  auto item_store = [&](int t, const Item& it) {
    if (t >= nitem) return;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      float w = 0.f;  // += in slot order: multi-edges sum like the CSR tile build
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj)
        if (it.u[jj] == u) w += s * it.gam[jj];
      Wt[it.cl * SZ + u * NTP + it.v] = w;
    }
    if (it.cl == 0) {
      sc[it.v] = it.ok ? s : 0.f;
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj) {
        // a source outside the graph is rejected on the host; keep the slot harmless anyway
        const bool in = (unsigned)it.u[jj] < (unsigned)n;
        slot_u[it.v * KMAX + jj] = in ? it.u[jj] : 0;
        slot_e[it.v * KMAX + jj] = in ? it.e[jj] : -1;
      }
    }
  };
  Item items[IPT];
#pragma unroll
  for (int i = 0; i < IPT; ++i) item_ids(threadIdx.x + i * blockDim.x, items[i]);
  if (active && j < jend) load_slice(j);
#pragma unroll
  for (int i = 0; i < IPT; ++i) {
    item_gamma(items[i]);
    item_store(threadIdx.x + i * blockDim.x, items[i]);
  }
  for (int t = threadIdx.x + IPT * blockDim.x; t < nitem; t += blockDim.x) {
    Item it;
    item_ids(t, it);
    item_gamma(it);
    item_store(t, it);
  }
  __syncthreads();

  float D[NS];
  float S[NT];
#pragma unroll
  for (int i = 0; i < NS; ++i) D[i] = 0.f;
#pragma unroll
  for (int v = 0; v < NT; ++v) S[v] = 0.f;

  if (active) {
    while (j < jend) {
      const uint32_t lane_off = lane_plane + (uint32_t)j * VEC * 4u;
      int tile = grp * SZ;  // laundered: keep the weights in LDS, not hoisted into registers
      asm volatile("" : "+v"(tile));
      const float* W = Wt + tile;
      if (a.want_dx) {
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          if (u >= n) break;
          Frag<VEC> acc;
          if (DXB) {
            acc = load_frag<VEC, true>(at_bytes(dxbase + (int64_t)u * a.dxbs, lane_off));
          } else {
#pragma unroll
            for (int k = 0; k < VEC; ++k) acc.v[k] = 0.f;
          }
          if (a.self_scale != 0.f) {  // residual epilogue
#pragma unroll
            for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(a.self_scale, gv[u][k], acc.v[k]);
          }
#pragma unroll
          for (int v4 = 0; v4 < NTP; v4 += 4) {
            const f4 w = *reinterpret_cast<const f4*>(W + u * NTP + v4);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int v = v4 + q;
              if (v >= NT) break;
#pragma unroll
              for (int k = 0; k < VEC; ++k) acc.v[k] = fmaf(w[q], gv[v][k], acc.v[k]);
            }
          }
          store_frag<VEC, true>(at_bytes(ob + (int64_t)u * a.os, lane_off), acc);
        }
      }
      if (a.want_dgb) {
#pragma unroll
        for (int v = 0; v < NT; ++v) {
#pragma unroll
          for (int k = 0; k < VEC; ++k) S[v] += gv[v][k];
#pragma unroll
          for (int jj = 0; jj < KMAX; ++jj) {
            if (jj >= K) break;
            const int u = __builtin_amdgcn_readfirstlane(slot_u[v * KMAX + jj]);  // wave-uniform
#pragma unroll
            for (int k = 0; k < VEC; ++k) D[v * KMAX + jj] = fmaf(gv[v][k], xv[u][k], D[v * KMAX + jj]);
          }
        }
      }
      j += a.lpc;
      if (j < jend) load_slice(j);
    }
  }
  if (!a.want_dgb) return;
  with_lanes(a.lpc, [&](auto lanes) {
    constexpr int L = decltype(lanes)::value;
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      S[v] = group_sum<L>(S[v]);
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj) D[v * KMAX + jj] = group_sum<L>(D[v * KMAX + jj]);
    }
  });
  if (active && li == 0) {
#pragma unroll
    for (int v = 0; v < NT; ++v) {
      Sl[grp * NTP + v] = S[v];
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj) Dl[grp * NS + v * KMAX + jj] = D[v * KMAX + jj];
    }
  }
  __syncthreads();
  // per-edge outputs: thread -> (channel fastest, slot)
  for (int t = threadIdx.x; t < a.cpb * NS; t += blockDim.x) {
    int cl, slot;
    split_channel(a, t, cl, slot);
    const int v = slot / KMAX;
    const int cc = c0 + cl;
    const int e = slot_e[slot];
    if (e < 0 || cc >= a.C) continue;
    const float s = sc[v];
    const int64_t off = ((int64_t)e * a.C + cc) * 2;
    float2 r = make_float2(s * Dl[cl * NS + slot], s * Sl[cl * NTP + v]);
    if (a.logits) r = sigmoid_backward(r, *reinterpret_cast<const float2*>(a.gb + off));
    *reinterpret_cast<float2*>(a.dgb + off) = r;
  }
}

// ---------------------------------------------------------------------------
// Backward for REGULAR graphs of up to 16 nodes on the matrix cores (film_bwd_regular's math):
//   grad_x[u][p] = sum_v Wt[u][v] G[v][p]              (Wt[u][v] = s_v * sum of gamma over u->v)
//   D[v][u]      = sum_p G[v][p] x[u][p]               (the per-channel Gram; slot (v, j) reads D[v][u(v,j)])
//   S[v]         = sum_p G[v][p]
// both products as v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32 accumulation), graphs padded to
// 16 nodes.  One wave = one channel plane of one graph (workgroup: 4 channels), pixels in groups of 64.
// Why: film_bwd_regular keeps N*K Gram accumulators per lane next to both operand slices (~180 VGPRs,
// 2 waves/SIMD) and walks each plane serially; here the Gram is 4 accumulator registers per lane, so
// the wave holds two pixel groups of loads in flight at ~100 VGPRs.
//
// Register layouts (lane l, q = l >> 4, j = l & 15; MFMA: A[i][k] at lane (i = j, k = q), B[k][col] at
// lane (k = q, col = j), C[4q + r][j] at lane l, element r):
//   G, "by quad":  gq[b] = G[node 4q + b][64 g + 4 j .. +3]   (b = 0..3: four 256-byte rows per load)
//     -> grad_x MFMA #c (c = pixel within the float4): A = Wt[j][4 q + b], B = gq[b][c], summed over b:
//        C[u = 4q + r][col j] = grad_x[4q + r][64 g + 4 j + c]: four float4 stores of 256-byte rows, and
//        the residual term self_scale * G[u] of element r is gq[r][c] in the same lane.
//   x, "by node":  xn[t] = x[node j][64 g + 16 t + 4 q .. +3]  (t = 0..3)
//   G by node: gq transposed through a per-wave LDS tile (in-wave ordering, no barrier)
//     -> Gram MFMA (t, c): A = G by node [t][c] (i = v = j, k = q), B = xn[t][c] (k = q, col = u = j).
// Nodes past the graph's n: G rows are zeroed (they would reach grad_x through zero weights as 0 * inf),
// x rows are clamped loads that only touch unused Gram columns.
// Requirements (launcher): P % 64 == 0, 16-byte aligned operands and node strides % 4 == 0.
// ---------------------------------------------------------------------------
typedef float mf4 __attribute__((ext_vector_type(4)));

// Template parameters:
//   COMPLETE: complete graphs of exactly n = max_nodes nodes with arithmetic edge ids (the reference
//             topology), else REGULAR(k) graphs (slot (v, j) = CSR position K v + j).
//   NPB:      nodes per 16-row block: 16 (graphs of 9..16 nodes, one channel per block) or 8 (graphs
//             of <= 8 nodes: two channels share a block as a block-diagonal system; row/column
//             16-index vn = 8 h + node, h = channel of the pair).
//   CPW:      blocks per wave, walked in turn with the next (block, pixel group)'s loads in flight
//             under the current group's MFMAs; workgroup = 4 waves = 4 CPW blocks, one prologue.
template <bool COMPLETE, int NPB, int KMAX, bool DXB, int CPW>
__global__ void __launch_bounds__(kBlock) film_bwd_mfma(AggArgs a) {
  static_assert(NPB == 16 || NPB == 8, "16-row blocks of one or two channels");
  constexpr int CB = 16 / NPB;             // channels per block
  constexpr int CPB = 4 * CPW * CB;        // channels per workgroup
  constexpr int NS = NPB * KMAX;           // REGULAR edge slots
  constexpr int WR = NPB + 1;              // per-channel Wt / D row stride (floats)
  // per-channel Wt / D stride: the prologue's 32-lane stores (CPB channels x 32 / CPB destinations)
  // land on 32 different banks (NPB = 16: 8 channels 20 banks apart mod 32; unpadded, 272 = 16 mod 32
  // was 4-way, rocprof r03: 24 % of the k-NN backward's LDS cycles)
  constexpr int CS = NPB * WR + (NPB == 16 ? 4 : 2);
  constexpr int SS = NPB + 1;              // per-channel S stride: odd, the epilogue's 8-16 channels on distinct banks
  // transpose tile row stride: 32 pixels + 8, so the 16-lane groups of the by-node ds_read_b128
  // (rows jl, column chunk q) cover distinct banks (+4 was 2-way)
  constexpr int TR = 32 + 8;
  extern __shared__ float4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  float* Wt = smem;                   // [CPB][CS]       Wt[u][v] (rows of WR); each channel's rows become D[v][u]
  float* Tt = Wt + CPB * CS;          // [4][16][TR]     per-wave transpose tile (half a pixel group)
  float* Sl = Tt + 4 * 16 * TR;       // [CPB][SS]
  int* slot_u = reinterpret_cast<int*>(Sl + CPB * SS);  // [NS] (REGULAR)
  int* slot_e = slot_u + NS;                              // [NS]

  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;
  const int node0 = COMPLETE ? b * a.nmax : a.goff[b];
  const int n = COMPLETE ? a.nmax : min(a.goff[b + 1] - node0, NPB);
  if (n <= 0) return;
  const int c0 = cb * CPB;
  const int K = COMPLETE ? n - 1 : a.kdeg;
  const int64_t ebase = (int64_t)b * n * (n - 1);  // COMPLETE: the graph's first edge
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = lane >> 4, jl = lane & 15;
  float s = a.mode != MRP_AGG_FILM_SUM && K > 0 ? 1.f / (float)K : 1.f;
  s *= a.agg_scale;  // epilogue: grad_out reaches the aggregate scaled

  // ---- prologue: thread t < CPB NPB owns (channel t % CPB, destination t / CPB): column v of that
  // channel's Wt (and, REGULAR, channel 0: v's slot row).  Order (vmcnt retires in issue order):
  // index loads, then the wave's first pixel group, then gamma (needs the edge ids) — so the two
  // dependent prologue round trips run under the first group's loads instead of before them.
  static_assert(CPB * NPB <= kBlock, "one prologue item per thread");
  constexpr int NE = COMPLETE ? NPB : KMAX;  // candidate in-edges of v
  const int pt = threadIdx.x;
  const bool pitem = pt < CPB * NPB;
  const int pcl = pt % CPB, pv = pt / CPB;
  int us[NE];
  int64_t es[NE];
  {
    const bool ok = pitem && pv < n && c0 + pcl < a.C;
#pragma unroll
    for (int jj = 0; jj < NE; ++jj) {
      if (COMPLETE) {
        const bool on = ok && jj < n && jj != pv;
        us[jj] = on ? jj : -1;
        es[jj] = on ? complete_eid(ebase, n, jj, pv) : -1;
      } else {
        const bool on = ok && jj < K;
        const int k = (node0 + (on ? pv : 0)) * K + (on ? jj : 0);
        // loaded unconditionally (k is a valid slot either way) and selected after: a load under the
        // select became a branch whose join waited for it — one memory round trip per slot in turn
        const int sv = a.src[k];
        const int ev = a.eid[k];
        us[jj] = on ? sv - node0 : -1;
        es[jj] = on ? ev : -1;
      }
    }
  }

  // 16-row index vn -> (channel of the pair, node).  This lane's G rows: vn = 4q + bb; its x row: jl.
  uint32_t goff4[4], boff4[4], ooff4[4];
  bool nvalid[4];
  int hq[4];
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    const int vn = 4 * q + bb;
    const int h = vn / NPB, node = vn % NPB;
    hq[bb] = h;
    nvalid[bb] = node < n;
    const uint32_t nd = (uint32_t)min(node, n - 1);
    const uint32_t hp = (uint32_t)h * (uint32_t)a.P * 4u + (uint32_t)jl * 16u;
    goff4[bb] = nd * (uint32_t)a.gs * 4u + hp;
    ooff4[bb] = nd * (uint32_t)a.os * 4u + hp;
    boff4[bb] = DXB ? nd * (uint32_t)a.dxbs * 4u + hp : 0u;
  }
  const int hx = jl / NPB, nx = jl % NPB;
  const int ngroups = a.P >> 6;
  float* T = Tt + w * 16 * TR;
  // the wave's blocks: channels c0 + (w + 4 i) CB + h
  const int nblk = max(0, min(CPW, (a.C - c0 - w * CB + 4 * CB - 1) / (4 * CB)));
  const int nsteps = nblk * ngroups;
  auto blk_c = [&](int i) { return c0 + (w + 4 * i) * CB; };  // first channel of block i
  // a block's second channel may lie past C (odd C): its loads then read the first channel's rows
  auto hvalid = [&](int i, int h) { return blk_c(i) + h < a.C; };

  // DXB: the grad_x base rows of a step travel with its G rows (prefetched a step ahead like them; loaded
  // at the store they exposed a full memory round trip per step: 125 vs 77 us at configs[4])
  mf4 gq[4], xn[4], gq2[4], xn2[4], bq[DXB ? 4 : 1], bq2[DXB ? 4 : 1];
  auto load_step = [&](int st, mf4 (&gr)[4], mf4 (&xr)[4], mf4 (&br)[DXB ? 4 : 1]) {
    const int i = st / ngroups, g = st - i * ngroups;
    const int c = blk_c(i);
    const float* gbase = a.g + (int64_t)node0 * a.gs + (int64_t)c * a.P;
    const bool h1 = CB == 1 || hvalid(i, 1);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) {
      const uint32_t off = goff4[bb] - (h1 ? 0u : (uint32_t)hq[bb] * (uint32_t)a.P * 4u);
      gr[bb] = __builtin_nontemporal_load(reinterpret_cast<const mf4*>(at_bytes(gbase, off + (uint32_t)g * 256u)));
    }
    if constexpr (DXB) {
      if (a.want_dx) {
        const float* dxbase = a.dxb + (int64_t)node0 * a.dxbs + (int64_t)c * a.P;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const uint32_t off = boff4[bb] - (h1 ? 0u : (uint32_t)hq[bb] * (uint32_t)a.P * 4u);
          br[bb] = __builtin_nontemporal_load(reinterpret_cast<const mf4*>(at_bytes(dxbase, off + (uint32_t)g * 256u)));
        }
      }
    }
    if (a.want_dgb) {
      const float* xbase = a.x + (int64_t)node0 * a.xs + (int64_t)c * a.P;
      const uint32_t xo = (uint32_t)min(nx, n - 1) * (uint32_t)a.xs * 4u + (uint32_t)(h1 ? hx : 0) * (uint32_t)a.P * 4u +
                          (uint32_t)q * 16u;
#pragma unroll
      for (int t = 0; t < 4; ++t)
        xr[t] = __builtin_nontemporal_load(
            reinterpret_cast<const mf4*>(at_bytes(xbase, xo + (uint32_t)g * 256u + (uint32_t)t * 64u)));
    }
  };

  if (nsteps > 0) load_step(0, gq, xn, bq);  // the first pixel group, ahead of the gamma loads
  if (pitem) {
    float gm[NE];
    // every slot's gamma requested before any is used (edge 0 for an empty slot, discarded): under
    // `es >= 0` each load was a branch whose join waited for it, NE round trips in turn
    // (copy mode: gb may be null, so grad_out's first element is read and discarded instead)
    float graw[NE];
    const bool copy = a.mode == MRP_AGG_COPY_MEAN || a.gb == nullptr;
    const float* gsrc = copy ? a.g : a.gb;
#pragma unroll
    for (int jj = 0; jj < NE; ++jj)
      graw[jj] = gsrc[copy ? 0 : ((es[jj] >= 0 ? es[jj] : 0) * a.C + c0 + pcl) * 2];
#pragma unroll
    for (int jj = 0; jj < NE; ++jj) {
      float gv = copy ? 1.f : graw[jj];
      if (!copy && a.logits) gv = sigmoidf(gv);
      gm[jj] = __int_as_float(__float_as_int(gv) & -(int)(es[jj] >= 0));  // es < 0 ? +0 : gv, by mask
    }
#pragma unroll
    for (int u = 0; u < NPB; ++u) {
      float wv = 0.f;
      if (COMPLETE) {
        wv = s * gm[u];
      } else {
#pragma unroll
        for (int jj = 0; jj < NE; ++jj)  // += in slot order: multi-edges sum like the CSR tile build
          if (us[jj] == u) wv += s * gm[jj];
      }
      Wt[pcl * CS + u * WR + pv] = wv;
    }
    if (!COMPLETE && pcl == 0) {
#pragma unroll
      for (int jj = 0; jj < KMAX; ++jj) {
        const bool in = (unsigned)us[jj] < (unsigned)n;  // outside the graph: rejected on the host
        slot_u[pv * KMAX + jj] = in ? us[jj] : 0;
        slot_e[pv * KMAX + jj] = in ? (int)es[jj] : -1;
      }
    }
  }
  __syncthreads();

  float wa[4];
  mf4 dacc = {0.f, 0.f, 0.f, 0.f};  // Gram: D[4q + r][jl] of the current block
  float sacc = 0.f;                 // S partial: row jl, this lane's pixels
  auto compute_step = [&](int st, mf4 (&gr)[4], const mf4 (&xr)[4], const mf4 (&br)[DXB ? 4 : 1]) {
    const int i = st / ngroups, g = st - i * ngroups;
    const int cbl = (w + 4 * i) * CB;  // first channel of the block within the workgroup
    const int c = c0 + cbl;
    bool rvalid[4];
#pragma unroll
    for (int bb = 0; bb < 4; ++bb) rvalid[bb] = nvalid[bb] && (CB == 1 || hvalid(i, hq[bb]));
    if (g == 0) {
      // A operand of the grad_x MFMAs: W[u = jl][v = 4 q + bb], zero off the block diagonal
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const int vn = 4 * q + bb;
        wa[bb] = (jl / NPB == vn / NPB) ? Wt[(cbl + jl / NPB) * CS + (jl % NPB) * WR + vn % NPB] : 0.f;
      }
      dacc = mf4{0.f, 0.f, 0.f, 0.f};
      sacc = 0.f;
    }
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
      if (!rvalid[bb]) gr[bb] = mf4{0.f, 0.f, 0.f, 0.f};
    if (a.want_dx) {
      float* obase = a.out + (int64_t)node0 * a.os + (int64_t)c * a.P;
      mf4 acc[4];
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        acc[cc] = mf4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) acc[cc] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[bb], gr[bb][cc], acc[cc], 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mf4 o = {acc[0][r], acc[1][r], acc[2][r], acc[3][r]};
        if (a.self_scale != 0.f) o += a.self_scale * gr[r];  // residual epilogue
        if (rvalid[r]) {
          if constexpr (DXB) o += br[r];
          __builtin_nontemporal_store(o, reinterpret_cast<mf4*>(at_bytes(obase, ooff4[r] + (uint32_t)g * 256u)));
        }
      }
    }
    if (a.want_dgb) {
      // G by row through the wave's LDS tile, 32 pixels (two t) at a time
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        if ((jl >> 3) == hh) {  // lanes with jl in [8hh, 8hh + 8) hold pixels [32hh, 32hh + 32) of the group
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) *reinterpret_cast<mf4*>(T + (4 * q + bb) * TR + 4 * (jl & 7)) = gr[bb];
        }
        // the tile is exchanged between lanes of this wave only: LDS executes a wave's accesses in
        // order, so a compiler-level barrier (no reordering across it) is all the ordering needed
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int t2 = 0; t2 < 2; ++t2) {
          const mf4 gn = *reinterpret_cast<const mf4*>(T + jl * TR + 16 * t2 + 4 * q);
          const mf4 xv = xr[2 * hh + t2];
#pragma unroll
          for (int cc = 0; cc < 4; ++cc) dacc = __builtin_amdgcn_mfma_f32_16x16x4f32(gn[cc], xv[cc], dacc, 0, 0, 0);
          sacc += (gn[0] + gn[1]) + (gn[2] + gn[3]);
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();
      }
      if (g == ngroups - 1) {
        // the block is done: its channels' Wt rows (read into wa at g == 0, by this wave only) become
        // D[v][u] (the diagonal blocks of the 16 x 16 Gram)
        sacc += __shfl_xor(sacc, 16, 64);
        sacc += __shfl_xor(sacc, 32, 64);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int vn = 4 * q + r;
          if (vn / NPB == jl / NPB) Wt[(cbl + vn / NPB) * CS + (vn % NPB) * WR + jl % NPB] = dacc[r];
        }
        if (q == 0) Sl[(cbl + hx) * SS + nx] = sacc;
      }
    }
  };

  // software pipeline over the wave's (block, pixel group) steps: two register sets, the next step's
  // loads in flight under the current step's MFMAs (step 0 was issued in the prologue)
  for (int st = 0; st < nsteps; st += 2) {
    if (st + 1 < nsteps) load_step(st + 1, gq2, xn2, bq2);
    compute_step(st, gq, xn, bq);
    if (st + 1 < nsteps) {
      if (st + 2 < nsteps) load_step(st + 2, gq, xn, bq);
      compute_step(st + 1, gq2, xn2, bq2);
    }
  }
  if (!a.want_dgb) return;
  __syncthreads();
  // per-edge outputs: thread -> (channel fastest, edge)
  const int nedge = COMPLETE ? n * (n - 1) : NS;
  for (int t = threadIdx.x; t < CPB * nedge; t += blockDim.x) {
    const int cl = t % CPB, el = t / CPB;
    const int cc = c0 + cl;
    if (cc >= a.C) continue;
    int u, v;
    int64_t e;
    if (COMPLETE) {
      u = el / (n - 1);
      const int vi = el - u * (n - 1);
      v = vi < u ? vi : vi + 1;
      e = ebase + el;
    } else {
      v = el / KMAX;
      e = slot_e[el];
      u = slot_u[el];
      if (e < 0) continue;
    }
    const int64_t off = (e * a.C + cc) * 2;
    float2 r = make_float2(s * Wt[cl * CS + v * WR + u], s * Sl[cl * SS + v]);
    if (a.logits) r = sigmoid_backward(r, *reinterpret_cast<const float2*>(a.gb + off));
    *reinterpret_cast<float2*>(a.dgb + off) = r;
  }
}

}  // namespace mrp

// ===========================================================================
// Host side: validation, geometry, template dispatch, C ABI.
// ===========================================================================
namespace mrp_host {

using mrp::AggArgs;

struct Geometry {
  int vec, lpc, cpb, threads, ncb;
  int64_t grid;
  int mfma_npb = 0;  // film_bwd_mfma: nodes per 16-row block (16 or 8); 0 = the VALU kernels
};



inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

// Lanes per channel plane: the largest power of two <= clamp(P/vec/2, lo, hi) (two slices per lane
// where the plane allows) and <= P/vec; channels per block fill the 256 threads up to max_cpb.
// Measured optima (tools/kernel_lab.hip product sweep): forward lo=16, hi=64 (64 lanes at 32x32,
// 32 at 16x16, 16 at 8x8); fused backward lo=8 (8 lanes x 32 channels at 8x8: 78 vs 87 us at
// C=1280); regular backward 16.
inline Geometry make_geometry(int C, int P, int vec, int lo, int hi, int max_cpb) {
  Geometry g;
  g.vec = vec;
  const int pv = P / g.vec;
  const int target = std::min(std::max(pv / 2, lo), hi);
  int lpc = 1;
  while (lpc * 2 <= pv && lpc * 2 <= target) lpc *= 2;
  int cpb = mrp::kBlock / lpc;
  if (cpb > max_cpb) cpb = max_cpb;
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
template <int NT, int KMAX>
size_t lds_fwd_regular(int cpb) {
  return (size_t)cpb * (NT * KMAX + 2) * sizeof(float2) + (size_t)NT * (KMAX / 4) * sizeof(unsigned);
}
template <int NT>
size_t lds_dx(int cpb) {
  return (size_t)(cpb * mrp::Tile<NT>::SZ + mrp::Tile<NT>::NTP) * sizeof(float);
}
template <int NT, int KMAX>
size_t lds_regular(int cpb) {
  return (size_t)(cpb * mrp::Tile<NT>::SZ + cpb * NT * KMAX + cpb * mrp::Tile<NT>::NTP + mrp::Tile<NT>::NTP) *
             sizeof(float) +
         2 * (size_t)NT * KMAX * sizeof(int);
}
// film_bwd_mfma: Wt/D + transpose tiles + S + slot table (cpb channels of npb nodes)
inline size_t lds_mfma(int cpb, int npb, int kmax) {
  const int cs = npb * (npb + 1) + (npb == 16 ? 4 : 2);  // film_bwd_mfma's CS, TR, SS
  return (size_t)(cpb * cs + 4 * 16 * 40 + cpb * (npb + 1)) * sizeof(float) + 2 * (size_t)npb * kmax * sizeof(int);
}
template <int NT>
size_t lds_bwd(int cpb, bool complete_logits, int lpc = 64) {
  // + the per-slot sigmoid values (float2) the COMPLETE epilogue reuses; one Gram partial per channel
  // group, or per wave when a plane spans several waves (lpc > 64)
  const int npg = lpc > 64 ? cpb * (lpc >> 6) : cpb;
  return (size_t)(cpb * mrp::Tile<NT>::SZ + npg * mrp::Tile<NT>::SZ + npg * mrp::Tile<NT>::SLS +
                  mrp::Tile<NT>::NTP) * sizeof(float) +
         (complete_logits ? (size_t)cpb * NT * NT * sizeof(float2) : 0);
}

#define MRP_LAUNCH(KERNEL, LDS) hipLaunchKernelGGL((KERNEL), dim3((unsigned)g.grid), dim3(g.threads), (LDS), st, a)


#define MRP_DISPATCH_NT(NTV, COMPLETE, FN, ...)                                        \
  switch (NTV) {                                                                       \
    case 1: return COMPLETE ? FN<1, true>(__VA_ARGS__) : FN<1, false>(__VA_ARGS__);    \
    case 2: return COMPLETE ? FN<2, true>(__VA_ARGS__) : FN<2, false>(__VA_ARGS__);    \
    case 3: return COMPLETE ? FN<3, true>(__VA_ARGS__) : FN<3, false>(__VA_ARGS__);    \
    case 4: return COMPLETE ? FN<4, true>(__VA_ARGS__) : FN<4, false>(__VA_ARGS__);    \
    case 5: return COMPLETE ? FN<5, true>(__VA_ARGS__) : FN<5, false>(__VA_ARGS__);    \
    case 6: return COMPLETE ? FN<6, true>(__VA_ARGS__) : FN<6, false>(__VA_ARGS__);    \
    case 7: return COMPLETE ? FN<7, true>(__VA_ARGS__) : FN<7, false>(__VA_ARGS__);    \
    case 8: return COMPLETE ? FN<8, true>(__VA_ARGS__) : FN<8, false>(__VA_ARGS__);    \
    case 9: return COMPLETE ? FN<9, true>(__VA_ARGS__) : FN<9, false>(__VA_ARGS__);    \
    case 10: return COMPLETE ? FN<10, true>(__VA_ARGS__) : FN<10, false>(__VA_ARGS__); \
    case 11: return COMPLETE ? FN<11, true>(__VA_ARGS__) : FN<11, false>(__VA_ARGS__); \
    case 12: return COMPLETE ? FN<12, true>(__VA_ARGS__) : FN<12, false>(__VA_ARGS__); \
    case 13: return COMPLETE ? FN<13, true>(__VA_ARGS__) : FN<13, false>(__VA_ARGS__); \
    case 14: return COMPLETE ? FN<14, true>(__VA_ARGS__) : FN<14, false>(__VA_ARGS__); \
    case 15: return COMPLETE ? FN<15, true>(__VA_ARGS__) : FN<15, false>(__VA_ARGS__); \
    case 16: return COMPLETE ? FN<16, true>(__VA_ARGS__) : FN<16, false>(__VA_ARGS__); \
    default: return hipErrorInvalidValue;                                              \
  }


inline bool common_args_ok(const int32_t* indptr, const int32_t* src, const int32_t* eid, const int32_t* graph_off,
                    int32_t num_graphs, int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                    int32_t C, int32_t P, int32_t mode) {
  if (num_graphs < 0 || num_nodes < 0 || num_edges < 0 || C < 0 || P < 0) return false;
  if (max_nodes < 0 || max_nodes > MRP_MAX_NODES) return false;
  if (mode < MRP_AGG_FILM_MEAN || mode > MRP_AGG_COPY_MEAN) return false;
  if (graph_kind == MRP_GRAPH_COMPLETE) {
    // every graph: exactly max_nodes nodes, all ordered pairs, numbered graph by graph
    if ((int64_t)num_graphs * max_nodes != num_nodes) return false;
    if ((int64_t)num_graphs * max_nodes * (max_nodes > 0 ? max_nodes - 1 : 0) != num_edges) return false;
    return true;
  }
  if (graph_kind != MRP_GRAPH_CSR && !MRP_GRAPH_IS_REGULAR(graph_kind)) return false;
  if (MRP_GRAPH_IS_REGULAR(graph_kind) && (MRP_GRAPH_REGULAR_K(graph_kind) < 1 ||
                                          (int64_t)MRP_GRAPH_REGULAR_K(graph_kind) * num_nodes != num_edges))
    return false;
  if (num_graphs > 0 && graph_off == nullptr) return false;
  if (num_nodes > 0 && indptr == nullptr) return false;
  if (num_edges > 0 && (src == nullptr || eid == nullptr)) return false;
  if ((int64_t)num_graphs * max_nodes < (int64_t)num_nodes) return false;
  return true;
}


}  // namespace mrp_host

// One case of a switch over the compile-time maximum graph size.
#define MRP_NT_CASE(N, COMPLETE, FN, ...) \
  case N: return COMPLETE ? FN<N, true>(__VA_ARGS__) : FN<N, false>(__VA_ARGS__);

namespace mrp_host {
// backward dispatch, split over translation units by graph size (they compile in parallel)
hipError_t dispatch_bwd_1_8(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st);
hipError_t dispatch_bwd_9_12(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st);
hipError_t dispatch_bwd_13_16(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st);
}  // namespace mrp_host

