// gcn_fused.hip — the no-grad GCN layer (edge encoder + FiLM-mean aggregation) in ONE launch, gfx950.
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:219-226, the eval path of
// dgl/eval.py:194-199 and dgl/training.py:225-240):
//     gamma, beta = edge_encoder(g.edata['pose'])      models.py:222  (Linear/ReLU/Linear/Sigmoid)
//     g.update_all(edge_udf, node_udf)                  models.py:223  (FiLM message, mailbox mean)
//
// Why one launch.  The aggregation streams 1.08 GB through HBM (film_fwd, ~174 us at the headline
// size) and leaves the matrix cores idle; the encoder (1.88 GFLOP, split-bf16 on the matrix cores)
// is ~20 us of its own launch in which HBM idles.  Here the first `nprod` workgroups of the grid
// ("producers") compute the encoder's logits z, graph by graph, while the remaining workgroups run
// the aggregation (film_fwd_body, unchanged arithmetic): each waits only for its own graph's rows.
//
// Producers.  Item = (four consecutive 32-edge halves, 32-column block cb): the halves of graphs are
// numbered graph-major (EPG = N(N-1) edges per graph in ceil(EPG/32) halves; an 8-node graph's second
// half holds 24 edges), so an item covers two 8-node graphs (four graphs of <= 6 nodes), and items run
// graph-major.  Wave w of a producer workgroup owns half w: per hidden block it computes X = relu(W1
// pose + b1) for its edges on the matrix cores, splits it, and accumulates z over the block's 32
// columns; the weight fragments of a hidden block (W1's and the column block's W2) are the same for the
// four waves and arrive once per workgroup by LDS-DMA (produce()).  The arithmetic, operand fragments
// and summation order are those of mrp_edge_encoder_fwd_split (encoder_split.hip, encoder2_body), so the
// logits are bit-identical to the two-launch path.
//
// Hand-off (cdna_hip_programming.md §6 Guideline 16; MI355X_MICROARCH.md § visibility).  Per item one
// 32-bit state word: 0 free, 1 claimed, 2 ready, zeroed by the launcher before every launch (a memset
// node).  A producer claims its items up front (agent-scope CAS), writes z with write-through (sc1)
// stores, drains them (s_waitcnt vmcnt(0) in every storing wave), passes a workgroup barrier and
// stores the item's word = ready (agent scope).  An aggregation workgroup polls the words of its
// graph's items with sc1 loads (requested before its first feature loads), and reads the rows with
// sc1 loads once every word is ready: no line of them is read by any CU before it was published in
// this launch, and the sc1 loads bypass L1.
//
// Progress under any dispatch order.  A consumer waits only on items some running workgroup claimed
// (a claimer never waits before publishing).  A consumer that finds an item still unclaimed after a
// bounded spin claims it and produces it itself (the same routine, same bits), so no placement or
// order of the workgroups can deadlock the grid; producers occupy the lowest workgroup indices, so in
// practice they claim everything first.  A claimed item that never turns ready (a fault) ends the
// wait after ~0.1 s with the launch's error word set, never a hang.

#include <cstring>

#include "encoder_split.hpp"
#include "film_mean_kernels.hpp"

namespace mrp_fused {

using mrp_x6::bf8;
using mrp_x6::f16v;
using mrp_x6::u4;
typedef __attribute__((address_space(1))) uint32_t gu32;

enum : uint32_t { kFree = 0u, kClaimed = 1u, kReady = 2u };
constexpr int kRing = 4;                          // producer: hidden blocks in the LDS-DMA ring
constexpr int kSlotsBytes = kRing * 9 * 64 * 16;  // ... of 9 KiB each (W1's 3 fragments, W2's 6)

struct FusedArgs {
  mrp::AggArgs agg;   // the aggregation (gb = z, logits)
  const float* pose;  // (E, 9)
  const u4* packed;   // mrp_edge_encoder_pack image of (W1, b1, W2)
  const float* b2;    // (2C) or null
  float* z;           // (E, 2C) logits, written by the producers
  uint32_t* state;    // one word per item (zeroed before every launch)
  uint32_t* err;      // set when a wait timed out (never expected)
  int32_t C, epg, halves, num_graphs;  // channels, edges per graph, 32-edge halves per graph, graphs
  int32_t nprod, nitems, kper;     // producer workgroups, items, items per producer
  int32_t lds_main;                // byte offset of the per-wave flag words past the main LDS region
  int32_t lab;                     // Tuning::fused_lab (0 in the product)
};

__device__ __forceinline__ uint32_t ld_state(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// uniform base + 32-bit byte offset (one address register instead of two)
__device__ __forceinline__ uint32_t ld_state_at(const uint32_t* base, uint32_t off) {
  return __hip_atomic_load((gu32*)(reinterpret_cast<const char*>(base) + off), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool claim(uint32_t* p) {
  uint32_t expected = kFree;
  return __hip_atomic_compare_exchange_strong((gu32*)p, &expected, kClaimed, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t image_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// s_waitcnt vmcnt(n) for a wave-uniform n in [0, 6]: the ring's own-DMA waits (the count is an immediate)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
  }
}

// One item (file header): z rows of the item's four 32-edge halves, columns of its 32-column block,
// published.  Called by all 256 threads (four waves); `lds` = the workgroup's LDS (the ring).
// Wave w owns edge half 4 ebg + w (graph b = half / halves): it computes X = relu(W1 pose + b1) of
// each hidden block for its own edges on the matrix cores and accumulates z += X^T W2^T for the block's
// 32 columns.  The four waves need the same weight fragments per hidden block — W1's (3 KiB) and the
// column block's W2 (6 KiB) — which arrive once per workgroup by LDS-DMA into a ring of kRing hidden
// blocks (kRing - 1 ahead), so a wave's weight bytes per MFMA are a quarter of a wave owning its own
// columns, and the fetch latency under the aggregation's HBM stream hides behind three blocks' work.
// lab bit 64 (Tuning::fused_lab): a timeline in the workspace past the hand-off words — per item its
// producer's start and publish times, per graph its first aggregation workgroup's wait window
// (s_memrealtime, 100 MHz).  Never set in the product.
__device__ __forceinline__ uint64_t* timeline(const FusedArgs& f) {
  return reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(f.err) + 256);
}

__device__ __forceinline__ void produce(const FusedArgs& f, int item, u4* lds) {
  using namespace mrp_x6;
  if ((f.lab & 64) && threadIdx.x == 0) timeline(f)[2 * item] = __builtin_amdgcn_s_memrealtime();
  const int C = f.C;
  const int HB = C / 32;
  const int ncolb = 2 * C / 32;
  const int cb = item % ncolb;
  const int ebg = item / ncolb;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int half = ebg * 4 + w;
  const int b = half / f.halves, h = half - (half / f.halves) * f.halves;
  const bool real = b < f.num_graphs;
  const int bb = real ? b : f.num_graphs - 1;  // a wave past the batch computes graph B-1 and stores nothing
  const int64_t e0 = (int64_t)bb * f.epg + h * 32;
  const int nval = real ? min(32, f.epg - h * 32) : 0;

  // pose fragment (B operand of X = W1' pose'^T): lane's edge, k = 8 hh + j; k = 9 is the 1.0 of b1
  bf8 pp[3];
  {
    const float* pr = f.pose + (e0 + min(r, max(nval, 1) - 1)) * kNin;
    float v[8];
    if (hh == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = pr[j];
    } else {
      v[0] = pr[8];
      v[1] = 1.f;
#pragma unroll
      for (int j = 2; j < 8; ++j) v[j] = 0.f;
    }
    split8(v, pp);
  }

  // ring slot of hidden block hb: [W1 parts 0..2 | W2 (s, p) 0..5], 1 KiB each (a wave's 64 lanes x 16 B);
  // chunk c of every slot is fetched by wave c % 4 (waves 0: 3 chunks, 1..3: 2)
  const __amdgpu_buffer_rsrc_t rs = image_rsrc(f.packed);
  const int nch = w == 0 ? 3 : 2;
  const uint32_t w1_bytes = (uint32_t)(w1_units(C) * 16);
  auto issue = [&](int hb) {
    u4* slot = lds + (hb % kRing) * 9 * 64;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int c = w + 4 * i;
      if (c >= 9) break;
      const uint32_t src = c < 3 ? (uint32_t)((hb * 3 + c) * 1024)
                                 : w1_bytes + (uint32_t)(((cb * HB + hb) * 6 + (c - 3)) * 1024);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, slot + c * 64, 16, (uint32_t)lane * 16u, src, 0, 0);
    }
  };
  f16v Z, ZL;
#pragma unroll
  for (int i = 0; i < 16; ++i) Z[i] = ZL[i] = 0.f;
  // the pose loads retire before the ring's (in order): the waits below cover them
#pragma unroll
  for (int hb = 0; hb < kRing - 1; ++hb)
    if (hb < HB) issue(hb);
#pragma unroll 1
  for (int hb = 0; hb < HB; ++hb) {
    wait_vmcnt(nch * min(kRing - 2, HB - 1 - hb));  // this wave's chunks of block hb have landed
    __syncthreads();  // everyone's chunks of hb landed; slot (hb - 1) % kRing read by every wave
    if (hb + kRing - 1 < HB) issue(hb + kRing - 1);
    const u4* slot = lds + (hb % kRing) * 9 * 64 + lane;
    bf8 wa[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) wa[p] = as_bf8(slot[p * 64]);
    f16v X;
#pragma unroll
    for (int i = 0; i < 16; ++i) X[i] = 0.f;
    X = mma6(wa, pp, X);
    // ReLU, split: X's accumulator layout is z's A operand (encoder_split.hip), s = 16-k half
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = relu(X[8 * s2 + j]);
      bf8 hp[3], wb[3];
      split8(hv, hp);
#pragma unroll
      for (int p = 0; p < 3; ++p) wb[p] = as_bf8(slot[(3 + 3 * s2 + p) * 64]);
      mma6_2(hp, wb, Z, ZL);
    }
  }
  // epilogue: accumulator register i of lane (r, hh) is row (i & 3) + 8 (i >> 2) + 4 hh, column r;
  // write-through stores (the hand-off's payload)
  const int N = 2 * C;
  const int col = cb * 32 + r;
  const float bias = f.b2 != nullptr ? f.b2[col] : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * hh;
    const float v = __fadd_rn(__fadd_rn(Z[i], ZL[i]), bias);
    if (row < nval && !(f.lab & 8))
      __hip_atomic_store((gu32*)(f.z + (e0 + row) * N + col), __float_as_uint(v), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the signal
  __syncthreads();  // (also: every wave is done with the ring before a next item refills it)
  if (threadIdx.x == 0) {
    __hip_atomic_store((gu32*)(f.state + item), kReady, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (f.lab & 64) timeline(f)[2 * item + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// A producer workgroup: claims its items (p, p + nprod, ...) in one round of CAS by wave 0, then
// produces the ones it won (an item a consumer already claimed is skipped).
__device__ __forceinline__ void producer(const FusedArgs& f, u4* slots, uint64_t* won_word) {
  const int p = blockIdx.x;
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    const int item = p + k * f.nprod;
    const bool won = k < f.kper && item < f.nitems && claim(f.state + item);
    const uint64_t m = __ballot(won);
    if (threadIdx.x == 0) *won_word = m;
  }
  __syncthreads();
  uint64_t m = *won_word;
  while (m != 0) {
    const int k = __builtin_ctzll(m);
    m &= m - 1;
    produce(f, p + k * f.nprod, slots);
  }
}

// The aggregation workgroups' side of the hand-off (film_fwd_body's Hook).  A workgroup's channels
// (a power of two <= 16 of them) lie in one 32-column block of z and its graph's edges in one group of
// four 32-edge halves: it waits on ONE item.
struct Consumer {
  static constexpr bool kFused = true;
  const FusedArgs& f;
  u4* slots;            // the workgroup's LDS (the fallback produces into it)
  uint32_t* wave_flag;  // 4 words past the main LDS region, then the fallback's two masks
  int item = 0;
  uint32_t v = kReady;  // lane 0: the item's state word

  __device__ Consumer(const FusedArgs& fa, u4* s, uint32_t* wf) : f(fa), slots(s), wave_flag(wf) {}

  __device__ void issue(int b, int c0) {
    b_ = b;
    c0_ = c0;
    // wave-uniform (a scalar register: it stays live across the fallback's producer routine)
    item = __builtin_amdgcn_readfirstlane((b * f.halves / 4) * (2 * f.C / 32) + (2 * c0) / 32);
    reload();
  }
  __device__ void reload() {
    if ((threadIdx.x & 63) == 0) v = ld_state_at(f.state, (uint32_t)item * 4u);
  }
  int b_ = 0, c0_ = 0;
  __device__ bool wait() {
    if (f.lab & 2) return true;
    const bool stamp = (f.lab & 64) && c0_ == 0 && threadIdx.x == 0;
    uint64_t t0 = stamp ? __builtin_amdgcn_s_memrealtime() : 0;
    const bool ok = spin();
    if (stamp) {
      uint64_t* tl = timeline(f) + 2 * f.nitems + 2 * b_;
      tl[0] = t0;
      tl[1] = __builtin_amdgcn_s_memrealtime();
    }
    return ok;
  }
  __device__ bool spin() {
    // relaxed sc1 polls by lane 0 with s_sleep; give up after a few ms (the caller's fallback)
    for (int spins = 0; !__all(v == kReady); ++spins) {
      if (spins >= 4096) return false;
      if (spins < 64)
        __builtin_amdgcn_s_sleep(2);
      else
        __builtin_amdgcn_s_sleep(32);
      reload();
    }
    return true;
  }
  // Workgroup-uniform: true when every wave saw its rows ready.
  __device__ bool all_ready(bool ready) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) wave_flag[w] = ready ? 1u : 0u;
    __syncthreads();
    return wave_flag[0] & wave_flag[1] & wave_flag[2] & wave_flag[3];
  }
  // After all_ready() said no (all 256 threads): wave 0 claims the item if it is still free (CAS),
  // the workgroup produces it if it won, else waits for it (claimed by a running workgroup), bounded at
  // ~0.1 s (then the launch's error word; never a hang).
  __device__ void fallback() {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    uint32_t* word = wave_flag + 4;
    for (int iter = 0;; ++iter) {
      __syncthreads();  // the word of the previous iteration read by every wave
      if (w == 0 && lane == 0) {
        const uint32_t s = ld_state(f.state + item);
        *word = s == kReady ? 0u : (s == kFree && claim(f.state + item)) ? 1u : 2u;
      }
      __syncthreads();
      const uint32_t what = *word;
      if (what == 1u) produce(f, item, slots);
      if (what <= 1u) return;
      if (iter >= 20000) {  // ~0.1 s: a claimed item never turned ready
        if (threadIdx.x == 0) __hip_atomic_store((gu32*)f.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(64);
    }
  }
};

// The second pass after a fallback: every row is published; read them past L1 as usual.
struct Published {
  static constexpr bool kFused = true;
  __device__ void issue(int, int) {}
  __device__ bool wait() { return true; }
  __device__ bool all_ready(bool) { return true; }
};


template <int NT>
__global__ void __launch_bounds__(256, 4) gcn_fused_fwd(FusedArgs f) {
  extern __shared__ float4 smem_fused[];
  u4* slots = reinterpret_cast<u4*>(smem_fused);
  uint32_t* flags = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(smem_fused) + f.lds_main);
  if ((int)blockIdx.x < f.nprod) {
    if (f.lab & 32) {  // lab: occupy the slot for ~40 us without touching memory
      for (int i = 0; i < 20000; ++i) __builtin_amdgcn_s_sleep(1);
      return;
    }
    if (!(f.lab & 4)) producer(f, slots, reinterpret_cast<uint64_t*>(flags + 4));
    return;
  }
  Consumer hook(f, slots, flags);
  const unsigned blk = blockIdx.x - (unsigned)f.nprod;
  if (!mrp::film_fwd_body<NT, 4, true, MRP_AGG_FILM_MEAN>(f.agg, blk, hook)) {
    hook.fallback();
    Published again;
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));  // the second pass recomputes its indices (nothing live across fallback)
    mrp::film_fwd_body<NT, 4, true, MRP_AGG_FILM_MEAN>(f.agg, blk, again, tid);
  }
}

}  // namespace mrp_fused

using namespace mrp_fused;

namespace {

// the fused launch's shapes: complete graphs of 2..8 nodes, C % 32 == 0, 16-byte slices, 256-thread
// aggregation workgroups of a power-of-two channel count (<= 16: one 32-column block of z)
struct FusedPlan {
  mrp_host::Geometry g;
  int32_t psplit, epg, halves, nitems;
};

bool fused_plan(int32_t num_graphs, int32_t N, int32_t C, int32_t P, FusedPlan& pl) {
  if (N < 2 || N > 8 || C <= 0 || C % 32 != 0 || P <= 0 || P % 4 != 0) return false;
  if ((mrp_x6::w1_units(C) + mrp_x6::w2_units(C)) * 16 >= ((int64_t)1 << 31)) return false;
  const mrp_host::Tuning& tu = mrp_host::tuning();
  pl.g = mrp_host::make_geometry(C, P, 4, tu.fwd_lo, tu.fwd_hi, tu.fwd_cap);
  if (pl.g.threads != 256 || 64 % pl.g.cpb != 0) return false;
  const int32_t pv = P / 4;
  pl.psplit = (pv + pl.g.lpc - 1) / pl.g.lpc;
  pl.epg = N * (N - 1);
  pl.halves = (pl.epg + 31) / 32;
  pl.nitems = (num_graphs * pl.halves + 3) / 4 * (2 * C / 32);  // (4 edge halves, 32 columns) items
  const int64_t grid = (int64_t)num_graphs * pl.g.ncb * pl.psplit;
  if (grid + 256 > 0x7fffffff || (int64_t)pl.nitems > 0x7fffffff / 2) return false;
  pl.g.grid = grid;
  return true;
}

int64_t state_bytes(int32_t nitems) { return ((int64_t)nitems * 4 + 255) / 256 * 256 + 256; }

}  // namespace

extern "C" {

int64_t mrp_gcn_fwd_fused_workspace_bytes(int32_t num_graphs, int32_t max_nodes, int32_t C, int32_t P) {
  FusedPlan pl;
  if (num_graphs <= 0 || !fused_plan(num_graphs, max_nodes, C, P, pl)) return 0;
  return state_bytes(pl.nitems);
}

int mrp_gcn_fwd_fused(const float* x, int64_t x_node_stride, const float* pose, const void* packed, const float* b2,
                      int32_t num_graphs, int32_t max_nodes, int32_t C, int32_t P, float* z, float* out,
                      int64_t out_node_stride, void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_graphs < 0 || max_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (num_graphs == 0 || C == 0 || P == 0) return hipSuccess;
  FusedPlan pl;
  if (!fused_plan(num_graphs, max_nodes, C, P, pl)) return hipErrorNotSupported;
  const int64_t plane = (int64_t)C * P;
  if (!x || !pose || !packed || !z || !out || !workspace) return hipErrorInvalidValue;
  if (x_node_stride < plane || out_node_stride < plane || x_node_stride % 4 != 0 || out_node_stride % 4 != 0 ||
      !mrp_host::aligned16(x) || !mrp_host::aligned16(out) || !mrp_host::aligned16(packed) ||
      !mrp_host::aligned16(workspace))
    return hipErrorInvalidValue;
  if (workspace_bytes < state_bytes(pl.nitems)) return hipErrorInvalidValue;
  // the aggregation reads z with 32-bit byte offsets
  if ((int64_t)num_graphs * pl.epg * 2 * C * 4 >= ((int64_t)1 << 31)) return hipErrorNotSupported;
  hipStream_t st = static_cast<hipStream_t>(stream);
  FusedArgs f = {};
  mrp::AggArgs& a = f.agg;
  a.x = x;
  a.xs = x_node_stride;
  a.gb = z;
  a.out = out;
  a.os = out_node_stride;
  a.C = C;
  a.P = P;
  a.PV = P / 4;
  a.mode = MRP_AGG_FILM_MEAN;
  a.lpc = pl.g.lpc;
  a.cpb = pl.g.cpb;
  a.ncb = pl.g.ncb;
  a.logits = 1;
  a.psplit = pl.psplit;
  a.agg_scale = 1.f;
  a.nmax = max_nodes;
  f.pose = pose;
  f.packed = static_cast<const u4*>(packed);
  f.b2 = b2;
  f.z = z;
  f.state = static_cast<uint32_t*>(workspace);
  f.err = reinterpret_cast<uint32_t*>(static_cast<char*>(workspace) + state_bytes(pl.nitems) - 256);
  f.C = C;
  f.epg = pl.epg;
  f.halves = pl.halves;
  f.num_graphs = num_graphs;
  f.nitems = pl.nitems;
  // 0 producers (lab/test knob): every item is produced by the aggregation workgroups' fallback
  const int knob = mrp_host::tuning().fused_producers;
  f.nprod = std::min(knob, pl.nitems);
  f.kper = 0;
  if (f.nprod > 0) {
    f.kper = (pl.nitems + f.nprod - 1) / f.nprod;
    if (f.kper > 64) {  // one CAS round by one wave claims a producer's items
      f.nprod = (pl.nitems + 63) / 64;
      f.kper = (pl.nitems + f.nprod - 1) / f.nprod;
    }
  }
  size_t lds_agg = 0;
  switch (max_nodes) {
#define MRP_FUSED_LDS(N) \
  case N: lds_agg = mrp_host::lds_fwd<N>(pl.g.cpb); break;
    MRP_FUSED_LDS(2) MRP_FUSED_LDS(3) MRP_FUSED_LDS(4) MRP_FUSED_LDS(5) MRP_FUSED_LDS(6) MRP_FUSED_LDS(7)
    MRP_FUSED_LDS(8)
#undef MRP_FUSED_LDS
  }
  f.lds_main = (int32_t)((std::max<size_t>(lds_agg, kSlotsBytes) + 15) / 16 * 16);
  const size_t lds = (size_t)f.lds_main + 32;  // + 4 wave flags + the fallback's two masks
  f.lab = mrp_host::tuning().fused_lab;
  if (!(f.lab & 1)) {
    hipError_t e = hipMemsetAsync(workspace, 0, (size_t)state_bytes(pl.nitems), st);
    if (e != hipSuccess) return e;
  }
  const dim3 grid((unsigned)(pl.g.grid + f.nprod));
  switch (max_nodes) {
#define MRP_FUSED_CASE(N) \
  case N: hipLaunchKernelGGL(gcn_fused_fwd<N>, grid, dim3(256), lds, st, f); break;
    MRP_FUSED_CASE(2) MRP_FUSED_CASE(3) MRP_FUSED_CASE(4) MRP_FUSED_CASE(5) MRP_FUSED_CASE(6)
    MRP_FUSED_CASE(7) MRP_FUSED_CASE(8)
#undef MRP_FUSED_CASE
  }
  return hipGetLastError();
}

}  // extern "C"
