// compress_fused.hip — the GCN layer's 1x1 compress convolution with the FiLM-mean aggregation
// fused into its operand producer, on the fp32 matrix cores of gfx950 (MI355X / CDNA4).
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:181-184):
//     g_h = self.gcn1(g)                       # update_all(edge_udf, node_udf), :207-211,223
//     h   = torch.cat((h, g_h), dim=1)          # (Nt, 2C, H, W)
//     h   = self.conv1(h)                       # nn.Conv2d(2C, C, 1): Y = W [x; agg] + b
// Here, per destination node v and pixel p:
//     Y[v, m, p] = sum_c W[m, c] x[v, c, p] + sum_c W[m, C + c] agg[v, c, p] + b[m]
// without the (Nt, 2C, P) concatenation buffer ever reaching HBM: each workgroup loads the slices of
// x of all nodes of ONE graph for a 16-pixel tile and a 16-channel stage, computes the aggregate of
// every node from those same registers (the reference's rounding: fl(fl(gamma x) + beta), sequential
// sum over in-edges by ascending source, true division), and feeds both halves to
// v_mfma_f32_16x16x4_f32 (f32 in, f32 accumulate: exact fp32 products, an fmaf chain per output).
//
// Work decomposition: workgroup = (graph b, 16-pixel tile, 128 output channels); 8 waves: 4 consumer
// waves (MFMA only) and 4 producer waves (loads, aggregate, LDS stores) — see the kernel.  The K loop
// runs over stages of 16 input channels: per stage every consumer wave issues 4 k-steps x 2 halves x
// 2 x N MFMAs (128 at N = 8) while the producers fill the other buffer with stage s+1.
//
// Supported: complete graphs (the reference topology, arithmetic edge ids) of N <= 8 nodes,
// P % 16 == 0, C % 128 == 0, mean/sum FiLM modes (gamma/beta as logits or post-sigmoid).  Anything
// else returns hipErrorNotSupported and the caller runs the unfused kernels (cat + library GEMM).
//
// Where the time goes (lab: tools/exp_cf_stamps.py, s_memtime around the barriers of one workgroup):
// an fp32 MFMA holds its SIMD's instruction issue for its whole 32 cycles, so the producers' VALU does
// not overlap the consumers' MFMAs — it is added to them.  A producer stage of 3.3k cycles alone took
// 10.9–11.4k beside the MFMAs (its aggregate phase 1.15k -> 7.3k: about one producer instruction per
// MFMA), against 9.0k cycles of MFMA-only stage.  Denser MFMA streams (b128 fragments for both
// operands) run the consumers alone faster (0.99 vs 1.02 ms) and the whole kernel slower (1.35 vs
// 1.26 ms at configs[1]).  Net: 1.19 ms against 1.24 ms for cat kernel + library GEMM at configs[1]
// (32x32 planes) and slower than it on 8x8 planes, where models.py keeps the unfused path.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fast_math.hpp"
#include "mrp_gnn.h"

#ifndef MRP_CF_WIDE_A
#define MRP_CF_WIDE_A 0
#endif

namespace mrp_cf {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kProducers = 4;  // load / aggregate / LDS-store waves
constexpr int TP = 16;         // pixels per workgroup
constexpr int KS = 16;         // input channels per stage (4 per producer wave)

// NC consumer (MFMA) waves, 32 output channels each: BM = 32 NC output channels per workgroup
template <int NC>
struct Geo {
  static constexpr int BM = 32 * NC;
  static constexpr int THREADS = 64 * (NC + kProducers);
  static constexpr int WF4 = 2 * KS * BM / 4 / (64 * kProducers);  // W float4 per producer lane per stage
};

// LDS stage layouts are "k4-packed": the 16 channels k = 4 k4 + lk of a stage are stored as [lk][...][k4],
// so the four values one MFMA lane (k row lk) needs for the stage's four k-steps are one 16-byte
// ds_read_b128 — 20 LDS reads per stage per consumer wave instead of 80 ds_read_b32.  A quarter-wave
// (16 lanes of one lk) reads 256 contiguous bytes: no bank conflicts without padding.
//   x / aggregate stage:  [node u][lk][pixel][k4]        (NT x 4 x 16 x 4 floats)
//   W stage:              [half h][lk][m (BM)][k4]       (2 x 4 x BM x 4 floats)
// The weight arrives pre-packed in HBM as [h][stage][lk][m (C)][k4] (mrp_compress_weight_pack), so a
// producer's float4 load is exactly one LDS float4.
// kPackB: the x / aggregate stages k4-packed too (one b128 per B fragment set) or plain [u][ch][pixel]
// (four ds_read_b32).  Packed makes the MFMA stream denser, which starves the producer waves more
// (an fp32 MFMA holds its SIMD's issue: lab stamps), so the plain layout is the faster combination.
constexpr bool kPackB = false;
// kWideA: the W fragments as one b128 per k4 set (1) or four ds_read_b32 from the same packed layout
// (0, default: 1.19 vs 1.23 ms at configs[1] for the same reason as kPackB)
constexpr bool kWideA = MRP_CF_WIDE_A;
__device__ __forceinline__ int xk4(int u, int ch, int px) {
  return kPackB ? ((u * 4 + (ch & 3)) * TP + px) * 4 + (ch >> 2) : (u * KS + ch) * TP + px;
}

struct Args {
  const float* x;
  int64_t xs;
  const float* gb;  // (E, C, 2)
  const float* wt;  // the conv weight packed by mrp_compress_weight_pack: [2][C/16][4][C][4]
  const float* bias;
  float* y;
  int64_t ys;
  int32_t C, P, ntiles_p, ntiles_m, mode, logits, remap;
  int32_t debug;  // kernel lab only: 1 = producers skip their work, 2 = consumers skip the MFMAs,
                  // 32 = no producer priority, 64 = BM 256 where C allows it
  long long* stamps;  // kernel lab only: s_memtime before/after the first 16 barriers of block 0, per wave
};

__device__ __forceinline__ float sigmoidf(float z) { return mrp_math::sigmoid(z); }  // the aggregation kernels' own

using mrp_math::div_fast;     // fast_math.hpp: the exact three-instruction x / (N - 1)
using mrp_math::div_fast_ok;

__device__ __forceinline__ const float* at_bytes(const float* base, uint32_t off) {
  return reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + off);
}

// DPP row_newbcast: every lane of a 16-lane row gets lane src's value of that row.  src must fold to a
// constant after unrolling (the DPP control is an immediate); the switch then folds away.  With full
// row/bank masks and bound_ctrl the compiler folds the move into the consuming v_mul / v_add (_dpp).
__device__ __forceinline__ float row_bcast(float v, int src) {
  const int i = __builtin_bit_cast(int, v);
  int r;
  switch (src) {
#define MRP_CF_BCAST(n) \
  case n: r = __builtin_amdgcn_update_dpp(0, i, 0x150 + n, 0xf, 0xf, true); break;
    MRP_CF_BCAST(0) MRP_CF_BCAST(1) MRP_CF_BCAST(2) MRP_CF_BCAST(3) MRP_CF_BCAST(4) MRP_CF_BCAST(5)
    MRP_CF_BCAST(6) MRP_CF_BCAST(7) MRP_CF_BCAST(8) MRP_CF_BCAST(9) MRP_CF_BCAST(10) MRP_CF_BCAST(11)
    MRP_CF_BCAST(12) MRP_CF_BCAST(13) MRP_CF_BCAST(14) default: r = __builtin_amdgcn_update_dpp(0, i, 0x15f, 0xf, 0xf, true);
#undef MRP_CF_BCAST
  }
  return __builtin_bit_cast(float, r);
}

template <int NT, int NC>
struct Lds {
  static constexpr int XS = NT * KS * TP;        // x stage  [node][lk][pix][k4]
  static constexpr int WS = 2 * KS * Geo<NC>::BM;  // W stage  [half][lk][m][k4]
  static constexpr int BUF = 2 * XS + WS;        // x, aggregate, W
  static constexpr int TOTAL = 2 * BUF;          // double buffer
};

// One K stage (16 input channels, both halves) of a consumer wave's 32 x (NT x 16) output block:
// W fragments from the k4-packed image (narrow or wide reads, kWideA), x / aggregate fragments from
// the [node][channel][pixel] images (kPackB: k4-packed instead).
template <int NT, int BM, bool WIDEA = kWideA>
__device__ __forceinline__ void consume_stage(f32x4 (&acc)[2][NT], const float* Xs, const float* As, const float* Ws,
                                              int w, int lk, int lc) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const f4* B4 = reinterpret_cast<const f4*>(h == 0 ? Xs : As);
    const f4* A4 = reinterpret_cast<const f4*>(Ws);
    f4 af[2], bf[NT];
    if (WIDEA) {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) af[mb] = A4[(h * 4 + lk) * BM + 32 * w + 16 * mb + lc];
    } else {
      const float* A1 = reinterpret_cast<const float*>(A4);
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) af[mb][k4] = A1[((h * 4 + lk) * BM + 32 * w + 16 * mb + lc) * 4 + k4];
    }
    if (kPackB) {
#pragma unroll
      for (int j = 0; j < NT; ++j) bf[j] = B4[(j * 4 + lk) * TP + lc];
    } else {
      const float* B1 = reinterpret_cast<const float*>(B4);
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) bf[j][k4] = B1[(j * KS + 4 * k4 + lk) * TP + lc];
    }
    // k-step k4 covers channels 4 k4 + (0..3) (lane row lk); consecutive MFMAs use different
    // accumulators, so no dependent issue back to back
#pragma unroll
    for (int k4 = 0; k4 < 4; ++k4)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int mb = 0; mb < 2; ++mb)
          acc[mb][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mb][k4], bf[j][k4], acc[mb][j], 0, 0, 0);
  }
}

// Epilogue: D[row = 4 (lane >> 4) + r][col = lane & 15] of block (mb, node j), + bias; nodes past
// nvalid (a partial node group) are not stored.
template <int NT, int BM>
__device__ __forceinline__ void store_tile(const f32x4 (&acc)[2][NT], float* y, int64_t ys, const float* bias, int P,
                                           int m0, int p0, int64_t node0, int nvalid, int w, int lk, int lc) {
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + 32 * w + 16 * mb + 4 * lk + r;
      const float bm = bias != nullptr ? bias[m] : 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if (j >= nvalid) break;
        float* yp = y + (node0 + j) * ys + (int64_t)m * P + p0 + lc;
        __builtin_nontemporal_store(__fadd_rn(acc[mb][j][r], bm), yp);
      }
    }
  }
}

// Roles (wave-uniform): waves 0..NC-1 are consumers — each owns output rows [32w, 32w + 32) x all N
// nodes x 16 pixels (2 x N accumulator blocks) and only reads LDS and issues MFMAs; the last 4 waves
// are producers — producer p fills channels [4p, 4p + 4) of the next stage: x slices of all N nodes,
// gamma/beta in registers (one edge per lane and slot), the aggregate from the same registers, and a
// quarter of the W stage.  Consumer and producer waves share each SIMD: the MFMA pipe and the
// VALU/memory work of the producer run concurrently (MI355X_MICROARCH.md, wave scheduling).  One
// workgroup barrier per stage hands the double-buffered stage over.  The aggregate of a (graph, pixel
// tile, stage) is recomputed by each of the C / BM workgroups of its output-channel column; the wider
// tile (NC = 8, BM = 256) halves that, but at one workgroup per CU it measured slower.
template <int NT, int NC, bool FILM, bool LOGITS, bool MEAN>
__global__ void __launch_bounds__(Geo<NC>::THREADS) compress_film_fwd(Args a) {
  using L = Lds<NT, NC>;
  constexpr int BM = Geo<NC>::BM, WF4 = Geo<NC>::WF4;
  extern __shared__ f4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);

  // block -> (graph, pixel tile, m tile); with remap, the m tiles of one (graph, pixel tile) are dealt
  // to the same XCD (blocks i and i + 8 share one), so their shared x slices hit that XCD's L2
  int id = blockIdx.x;
  if (a.remap) id = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const int mt = id % a.ntiles_m;
  const int rest = id / a.ntiles_m;
  const int pt = rest % a.ntiles_p;
  const int b = rest / a.ntiles_p;
  const int m0 = mt * BM, p0 = pt * TP;
  const int node0 = b * NT;
  const int64_t ebase = (int64_t)b * NT * (NT - 1);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nstages = a.C / KS;
  // lab stamps (a.stamps == nullptr in the product): shader-clock time around each barrier
  const bool stamping = a.stamps != nullptr && blockIdx.x == 0;
  int nbar = 0;
  auto sync = [&]() {
    if (stamping && nbar < 16 && lane == 0) a.stamps[w * 32 + 2 * nbar] = __builtin_amdgcn_s_memtime();
    __syncthreads();
    if (stamping && nbar < 16 && lane == 0) a.stamps[w * 32 + 2 * nbar + 1] = __builtin_amdgcn_s_memtime();
    ++nbar;
  };

  if (w >= NC) {
    // ------------------------------------------------------------------ producer
    // the producers' VALU would otherwise lose issue arbitration to the (older) consumer waves and
    // finish only after the consumers wait at the barrier (MI355X_MICROARCH.md, two waves per SIMD):
    // at high priority it fills the issue slots an MFMA leaves free (8 of its 32 cycles are held)
    if (!(a.debug & 32)) __builtin_amdgcn_s_setprio(2);
    const int pw = w - NC;                    // 0..3
    const int pt_id = pw * 64 + lane;         // 0..255 within the producers
    const int cl = lane >> 4, px = lane & 15;  // (channel within the wave's 4, pixel): one 16-lane DPP row per channel
    const int pch = 4 * pw + cl;              // channel within the stage
    constexpr int NE = NT * (NT - 1);          // edges of a graph
    constexpr int GI = (NE + 15) / 16;         // gamma/beta pairs per lane: lane px of a row holds edges px + 16 i
    // x (from HBM) is loaded two stages before it is stored to LDS, in two alternating register sets;
    // W and gamma/beta (L2-resident) one stage before, in one set — two sets of everything spilled at
    // BM = 256.  Issue order per stage: W + gamma/beta of the next stage, then x of the one after, so
    // waiting for the next stage's operands leaves the newest x loads in flight.
    struct XRegs {
      float xr[NT];
    };
    struct WRegs {
      f4 wr[WF4];
      float2 gr[GI];
    };
    XRegs X0, X1;
    WRegs WG;
    const int last = nstages - 1;
    // addressing: buffer loads — a wave-uniform resource per operand (x of this graph and pixel tile,
    // W of this m tile, gamma/beta of this graph), a per-lane 32-bit voffset fixed for the whole loop
    // and a wave-uniform soffset per stage (SGPR).  With flat pointers the compiler re-associated the
    // uniform and per-lane parts into 64-bit per-lane pointers (VGPR pairs + 64-bit adds per stage).
    // The host guarantees every byte offset fits in 31 bits.
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.x + (int64_t)node0 * a.xs + p0), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.wt + 4 * m0), 0, 0x7fffffff, 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.gb != nullptr ? a.gb + ebase * a.C * 2 : a.x), 0, 0x7fffffff, 0x00020000);
    const uint32_t x_off = (uint32_t)(pch * a.P + px) * 4u;
    // W float4 i of this lane: m = idx % BM, lk = (idx / BM) % 4, h = idx / (4 BM); in HBM at
    // [h][stage][lk][m0 + m][0..3], the stage part going into the per-stage soffset
    uint32_t w_off[WF4];
#pragma unroll
    for (int i = 0; i < WF4; ++i) {
      const int idx = pt_id + i * 256;
      const int m = idx % BM, lk = (idx / BM) % 4, h = idx / (4 * BM);
      w_off[i] = (uint32_t)(((h * (a.C / KS) * 4 + lk) * a.C + m) * 4) * 4u;
    }
    uint32_t g_off[GI];
#pragma unroll
    for (int i = 0; i < GI; ++i) g_off[i] = (uint32_t)((min(px + 16 * i, NE - 1) * a.C + pch) * 2) * 4u;
    auto issue_x = [&](XRegs& R, int s) {
      const int c0 = s * KS;
#pragma unroll
      for (int u = 0; u < NT; ++u)
        R.xr[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(xr, x_off, (c0 * a.P + u * (int)a.xs) * 4, 0));
    };
    auto issue_wg = [&](WRegs& R, int s) {
      const int c0 = s * KS;
#pragma unroll
      for (int i = 0; i < WF4; ++i)  // W stage: 2 halves x 16 k x BM m
        R.wr[i] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(wr, w_off[i], c0 * a.C * 4, 0));  // stage = 16 C floats
      // slots past the graph's NE edges reload the last edge (never read): no divergent branch around
      // the loads, so the compiler counts them exactly
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        if (FILM) {
          R.gr[i] = __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(gr, g_off[i], c0 * 2 * 4, 0));
        }
      }
    };
    auto produce = [&](const XRegs& X, const WRegs& R, int buf) {
      float* Xs = smem + buf * L::BUF;
      float* As = Xs + L::XS;
      float* Ws = As + L::XS;
#pragma unroll
      for (int u = 0; u < NT; ++u) Xs[xk4(u, pch, px)] = X.xr[u];
#pragma unroll
      for (int i = 0; i < WF4; ++i) {
        const int idx = pt_id + i * 256;
        const int m = idx % BM, lk = (idx / BM) % 4, h = idx / (4 * BM);
        *reinterpret_cast<f4*>(Ws + ((h * 4 + lk) * BM + m) * 4) = R.wr[i];
      }
      if (stamping && nbar < 16 && lane == 0) a.stamps[16 * 32 + w * 64 + 4 * nbar + 0] = __builtin_amdgcn_s_memtime();
      float gam[GI], bet[GI];
#pragma unroll
      for (int i = 0; i < GI; ++i) {
        gam[i] = LOGITS ? sigmoidf(R.gr[i].x) : R.gr[i].x;
        bet[i] = LOGITS ? sigmoidf(R.gr[i].y) : R.gr[i].y;
      }
      // agg[v] = sum over u != v, ascending, of fl(fl(gamma_uv x_u) + beta_uv): gamma/beta of edge
      // e = u -> v (i-major ids, dgl/dataloader.py:88-95) sit in lane e % 16 of this channel's row,
      // slot e / 16, and reach every pixel lane by a DPP row broadcast (no LDS round trip)
      // Under fp32 MFMA traffic a producer instruction that is not ready when the SIMD is free loses
      // the slot to a 32-cycle MFMA (lab stamps: a producer stage of 3.2k cycles alone took 11.4k
      // beside the MFMAs), so the stage is written for independent instructions back to back: the
      // destinations go in groups of four, all products, then all + beta, then the four running sums
      // interleaved (each sum still adds its terms in ascending source order).
      float sum[NT];
      float mn = __builtin_inff(), mx = 0.f;
      constexpr int VG = NT < 4 ? NT : 4;
#pragma unroll
      for (int v0 = 0; v0 < NT; v0 += VG) {
        float m[VG][NT];
#pragma unroll
        for (int vv = 0; vv < VG; ++vv) {
          const int v = v0 + vv;
#pragma unroll
          for (int u = 0; u < NT; ++u) {
            if (v >= NT || u == v) continue;
            m[vv][u] = X.xr[u];
            if (FILM) {
              const int e = u * (NT - 1) + (v < u ? v : v - 1);
              m[vv][u] = __fmul_rn(row_bcast(gam[e >> 4], e & 15), m[vv][u]);
            }
          }
        }
        if (FILM) {
#pragma unroll
          for (int vv = 0; vv < VG; ++vv) {
            const int v = v0 + vv;
#pragma unroll
            for (int u = 0; u < NT; ++u) {
              if (v >= NT || u == v) continue;
              const int e = u * (NT - 1) + (v < u ? v : v - 1);
              m[vv][u] = __fadd_rn(row_bcast(bet[e >> 4], e & 15), m[vv][u]);
            }
          }
        }
        float acc[VG];
#pragma unroll
        for (int vv = 0; vv < VG; ++vv) acc[vv] = 0.f;
#pragma unroll
        for (int u = 0; u < NT; ++u)
#pragma unroll
          for (int vv = 0; vv < VG; ++vv)
            if (v0 + vv < NT && u != v0 + vv) acc[vv] = __fadd_rn(acc[vv], m[vv][u]);
#pragma unroll
        for (int vv = 0; vv < VG; ++vv) {
          if (v0 + vv >= NT) continue;
          sum[v0 + vv] = acc[vv];
          if (MEAN && NT > 2) {
            mn = fminf(mn, __builtin_fabsf(acc[vv]));
            mx = fmaxf(mx, __builtin_fabsf(acc[vv]));
          }
        }
      }
      if (MEAN && NT > 2) {
        if (__builtin_expect(!div_fast_ok(mn, mx), 0)) {
#pragma unroll
          for (int v = 0; v < NT; ++v) sum[v] = sum[v] / (float)(NT - 1);
        } else {
#pragma unroll
          for (int v = 0; v < NT; ++v) sum[v] = div_fast<NT - 1>(sum[v]);
        }
      }
#pragma unroll
      for (int v = 0; v < NT; ++v) As[xk4(v, pch, px)] = sum[v];
      if (stamping && nbar < 16 && lane == 0) a.stamps[16 * 32 + w * 64 + 4 * nbar + 1] = __builtin_amdgcn_s_memtime();
    };
    // stage t: x in register set t & 1, LDS buffer t & 1.  nstages is a multiple of 8 (C % 128 == 0).
    // The loop body has no conditional loads (stage indices are clamped instead): with a path that
    // skipped them the compiler's wait counts would merge to "everything", draining the loads in
    // flight.
    issue_x(X0, 0);
    issue_wg(WG, 0);
    issue_x(X1, 1);
    produce(X0, WG, 0);
    issue_wg(WG, 1);
    issue_x(X0, min(2, last));
    if (a.debug & 1) {  // lab: consumers only
      for (int s = 0; s < nstages; ++s) sync();
      return;
    }
    for (int s = 0; s < nstages - 2; s += 2) {
      sync();  // barrier #s: stage s complete in LDS, stage s-1 consumed
      produce(X1, WG, 1);  // stage s+1
      issue_wg(WG, s + 2);
      issue_x(X1, s + 3);
      sync();  // barrier #(s+1)
      produce(X0, WG, 0);  // stage s+2
      issue_wg(WG, min(s + 3, last));
      issue_x(X0, min(s + 4, last));
    }
    sync();  // barrier #(nstages-2)
    produce(X1, WG, 1);  // the last stage
    sync();  // barrier #(nstages-1)
    return;
  }

  // -------------------------------------------------------------------- consumer
  f32x4 acc[2][NT];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lk = lane >> 4, lc = lane & 15;
  for (int s = 0; s < nstages; ++s) {
    sync();  // stage s is in LDS; the producers now fill stage s+1 in the other buffer
    const float* Xs = smem + (s & 1) * L::BUF;
    const float* As = Xs + L::XS;
    const float* Ws = As + L::XS;
    if (a.debug & 2) continue;  // lab: producers only
    consume_stage<NT, BM>(acc, Xs, As, Ws, w, lk, lc);
  }

  store_tile<NT, BM>(acc, a.y, a.ys, a.bias, a.P, m0, p0, node0, NT, w, lk, lc);
}

// ---------------------------------------------------------------------------------------------
// Two-source form: y = W[:, :C] x + W[:, C:] agg + b with agg already in HBM (mrp_film_mean_fwd's
// output), i.e. the compress of models.py:181-184 without the (N, 2C, P) concatenation.  Same tiles
// and consumer waves as the fused kernel; the producers only move operands, by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, no VALU, 1 KiB per instruction) — 32 per stage per
// workgroup, 8 per producer wave: x of 8 nodes, agg of 8 nodes, the W stage's 16 KiB.  One stage
// ahead: stage s+1 is issued right after barrier #s (its buffer was consumed before that barrier)
// and retired by the producers' explicit vmcnt(0) ahead of barrier #(s+1).  Nodes are taken in groups of 8
// (any node count: a partial last group re-loads its last node and stores only its own nodes).
// ---------------------------------------------------------------------------------------------
struct DualArgs {
  const float* x;
  int64_t xs;
  const float* g;  // aggregate
  int64_t gs;
  const float* wt;  // packed weight (mrp_compress_weight_pack)
  const float* bias;
  float* y;
  int64_t ys;
  int32_t C, P, num_nodes, ntiles_p, ntiles_m, remap;
};

template <bool WIDEA>
__global__ void __launch_bounds__(Geo<4>::THREADS) compress_dual_fwd(DualArgs a) {
  constexpr int NT = 8, NC = 4;
  using L = Lds<NT, NC>;
  constexpr int BM = Geo<NC>::BM;
  extern __shared__ f4 smem_f4[];
  float* smem = reinterpret_cast<float*>(smem_f4);
  int id = blockIdx.x;
  if (a.remap) id = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
  const int mt = id % a.ntiles_m;
  const int rest = id / a.ntiles_m;
  const int pt = rest % a.ntiles_p;
  const int grp = rest / a.ntiles_p;
  const int m0 = mt * BM, p0 = pt * TP;
  const int64_t node0 = (int64_t)grp * NT;
  const int nvalid = (int)min((int64_t)NT, (int64_t)a.num_nodes - node0);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nstages = a.C / KS;

  if (w >= NC) {
    const int pw = w - NC;  // 0: x, 1: agg, 2 / 3: W halves 0 / 1
    const int r = lane >> 2, q = lane & 3;  // x / agg: channel row within the stage, 16-byte chunk
    // LDS destinations as float4 indices into the __shared__ array itself (the builtin needs an
    // LDS-typed pointer; the wave's 64 lanes land at dst + lane)
    auto issue = [&](int s) {
      const int buf4 = (s & 1) * L::BUF / 4;
      const int c0 = s * KS;
      if (pw < 2) {
        const float* src = pw == 0 ? a.x : a.g;
        const int64_t ss = pw == 0 ? a.xs : a.gs;
        const int dst4 = buf4 + pw * L::XS / 4;
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int64_t node = node0 + min(u, nvalid - 1);
          const float* gp = src + node * ss + (int64_t)(c0 + r) * a.P + p0 + 4 * q;
          __builtin_amdgcn_global_load_lds(gp, &smem_f4[dst4 + u * KS * TP / 4], 16, 0, 0);
        }
      } else {
        const int h = pw - 2;
        const int dst4 = buf4 + 2 * L::XS / 4;
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // (lk, half) of this W half: 2 KiB per lk
          const int lk = i >> 1, half = i & 1;
          const float* gp = a.wt + ((((int64_t)h * (a.C / KS) + s) * 4 + lk) * a.C + m0 + 64 * half + lane) * 4;
          __builtin_amdgcn_global_load_lds(gp, &smem_f4[dst4 + (h * 4 + lk) * BM + 64 * half], 16, 0, 0);
        }
      }
    };
    issue(0);
    for (int s = 0; s < nstages; ++s) {
      // LDS-DMA writes are tracked by the issuing wave's vmcnt only: the compiler's workgroup fence
      // waits for LDS (lgkmcnt) but not for them, so without this wait the consumers could read a
      // stage that has not landed (tools/exp_determinism.py caught it: NaN / run-to-run differences)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // barrier #s: stage s landed; stage s-1's buffer is free
      if (s + 1 < nstages) issue(s + 1);
    }
    return;
  }

  f32x4 acc[2][NT];
#pragma unroll
  for (int mb = 0; mb < 2; ++mb)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[mb][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int lk = lane >> 4, lc = lane & 15;
  for (int s = 0; s < nstages; ++s) {
    __syncthreads();
    const float* Xs = smem + (s & 1) * L::BUF;
    consume_stage<NT, BM, WIDEA>(acc, Xs, Xs + L::XS, Xs + 2 * L::XS, w, lk, lc);
  }
  store_tile<NT, BM>(acc, a.y, a.ys, a.bias, a.P, m0, p0, node0, nvalid, w, lk, lc);
}

// gamma/beta = sigmoid(z), the aggregation kernels' own expression (fast_math.hpp):
// the fused kernel then reads post-sigmoid pairs instead of evaluating 2 x NE sigmoids per channel in
// every workgroup of a (graph, channel) column
__global__ void __launch_bounds__(256) film_gate(const float4* __restrict__ z, float4* __restrict__ g, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = z[i];
    g[i] = make_float4(sigmoidf(v.x), sigmoidf(v.y), sigmoidf(v.z), sigmoidf(v.w));
  }
}

// wp[h][s][lk][m][k4] = w[m][h C + 16 s + 4 k4 + lk]: the (C, 2C) conv weight in the k4-packed stage
// layout above.  One thread per output float4.
__global__ void __launch_bounds__(256) weight_pack(const float* __restrict__ w, f4* __restrict__ wp, int32_t C) {
  const int64_t n4 = (int64_t)2 * C * C / 4;  // float4 of wp
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int64_t m = i % C;
    const int64_t rest = i / C;  // (h, s, lk)
    const int lk = (int)(rest % 4);
    const int64_t hs = rest / 4;  // h * (C / 16) + s
    const int64_t h = hs / (C / KS), st = hs % (C / KS);
    const float* src = w + m * 2 * C + h * C + st * KS + lk;
    wp[i] = f4{src[0], src[4], src[8], src[12]};
  }
}

}  // namespace mrp_cf

namespace {

int mrp_cf_debug = 0;
long long* mrp_cf_stamps = nullptr;

template <int NT, int NC, bool FILM, bool LOGITS, bool MEAN>
hipError_t launch_mode(const mrp_cf::Args& a, int64_t grid, hipStream_t st) {
  const size_t lds = (size_t)mrp_cf::Lds<NT, NC>::TOTAL * sizeof(float);  // N = 8: 68 KB (NC 4), 101 KB (NC 8)
  auto* kern = &mrp_cf::compress_film_fwd<NT, NC, FILM, LOGITS, MEAN>;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(mrp_cf::Geo<NC>::THREADS), lds, st, a);
  return hipGetLastError();
}

// the FiLM mode is a template parameter: evaluated per edge term at run time it left the producers'
// inner loops full of branches
template <int NT, int NC>
hipError_t launch_nc(const mrp_cf::Args& a, int64_t grid, hipStream_t st) {
  if (a.mode == MRP_AGG_COPY_MEAN) return launch_mode<NT, NC, false, false, true>(a, grid, st);
  const bool mean = a.mode == MRP_AGG_FILM_MEAN;
  if (a.logits)
    return mean ? launch_mode<NT, NC, true, true, true>(a, grid, st) : launch_mode<NT, NC, true, true, false>(a, grid, st);
  return mean ? launch_mode<NT, NC, true, false, true>(a, grid, st) : launch_mode<NT, NC, true, false, false>(a, grid, st);
}

// BM = 128 output channels per workgroup (two workgroups per CU); BM = 256 (one per CU, half the
// redundant aggregation per MFMA) only through the lab hook: 1.25 vs 1.19 ms at configs[1]
template <int NT>
hipError_t launch(mrp_cf::Args a, int32_t num_graphs, hipStream_t st) {
  const int nc = (a.C % 256 == 0 && (a.debug & 64)) ? 8 : 4;
  a.ntiles_m = a.C / (32 * nc);
  const int64_t grid = (int64_t)num_graphs * a.ntiles_p * a.ntiles_m;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  a.remap = grid % 8 == 0 ? 1 : 0;
  return nc == 8 ? launch_nc<NT, 8>(a, grid, st) : launch_nc<NT, 4>(a, grid, st);
}

}  // namespace

extern "C" int mrp_compress_weight_pack(const float* w, float* wp, int32_t C, void* stream) {
  if (C <= 0 || C % mrp_cf::KS != 0 || w == nullptr || wp == nullptr || (reinterpret_cast<uintptr_t>(wp) & 15))
    return hipErrorInvalidValue;
  const int64_t n4 = (int64_t)2 * C * C / 4;
  const int64_t blocks = (n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096;
  hipLaunchKernelGGL(mrp_cf::weight_pack, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), w,
                     reinterpret_cast<mrp_cf::f4*>(wp), C);
  return hipGetLastError();
}

extern "C" int mrp_film_gate(const float* z, float* gb, int64_t n, void* stream) {
  if (n < 0 || n % 4 != 0) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  if (z == nullptr || gb == nullptr || (reinterpret_cast<uintptr_t>(z) & 15) || (reinterpret_cast<uintptr_t>(gb) & 15))
    return hipErrorInvalidValue;
  const int64_t n4 = n / 4;
  const int64_t blocks = (n4 + 255) / 256 < 4096 ? (n4 + 255) / 256 : 4096;
  hipLaunchKernelGGL(mrp_cf::film_gate, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     reinterpret_cast<const float4*>(z), reinterpret_cast<float4*>(gb), n4);
  return hipGetLastError();
}

// kernel-lab hook (tools/exp_compress_fused.py): not part of the ABI header
extern "C" void mrp_compress_film_debug(int mode) { mrp_cf_debug = mode; }
extern "C" void mrp_compress_film_debug_stamps(long long* device_buffer) { mrp_cf_stamps = device_buffer; }

extern "C" int mrp_compress_dual_fwd(const float* x, int64_t x_node_stride, const float* agg, int64_t agg_node_stride,
                                     int32_t num_nodes, int32_t C, int32_t P, const float* wt, const float* bias, float* y,
                                     int64_t y_node_stride, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (C % 128 != 0 || P % mrp_cf::TP != 0 || C == 0) return hipErrorNotSupported;
  if (num_nodes == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (!x || !agg || !y || !wt || x_node_stride < plane || agg_node_stride < plane || y_node_stride < plane)
    return hipErrorInvalidValue;
  // 16-byte LDS-DMA pieces: every row start 16-byte aligned
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(agg) & 15) ||
      (reinterpret_cast<uintptr_t>(wt) & 15) || (x_node_stride & 3) || (agg_node_stride & 3) || (P & 3))
    return hipErrorNotSupported;
  mrp_cf::DualArgs a;
  a.x = x;
  a.xs = x_node_stride;
  a.g = agg;
  a.gs = agg_node_stride;
  a.wt = wt;
  a.bias = bias;
  a.y = y;
  a.ys = y_node_stride;
  a.C = C;
  a.P = P;
  a.num_nodes = num_nodes;
  a.ntiles_p = P / mrp_cf::TP;
  a.ntiles_m = C / mrp_cf::Geo<4>::BM;
  const int64_t groups = ((int64_t)num_nodes + 7) / 8;
  const int64_t grid = groups * a.ntiles_p * a.ntiles_m;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  a.remap = grid % 8 == 0 ? 1 : 0;
  const size_t lds = (size_t)mrp_cf::Lds<8, 4>::TOTAL * sizeof(float);
  // W fragments as four ds_read_b32 (default) or, lab hook bit 128, one ds_read_b128 per k4 set:
  // 1056 vs 1049 us at configs[1] and 0.5-1 % slower at every other config (tools/exp_compress_dual.py)
  const bool wide = (mrp_cf_debug & 128) != 0;
  auto* kern = wide ? &mrp_cf::compress_dual_fwd<true> : &mrp_cf::compress_dual_fwd<false>;
  static const hipError_t attr_w = hipFuncSetAttribute(reinterpret_cast<const void*>(&mrp_cf::compress_dual_fwd<true>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  static const hipError_t attr_n = hipFuncSetAttribute(reinterpret_cast<const void*>(&mrp_cf::compress_dual_fwd<false>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_w != hipSuccess) return attr_w;
  if (attr_n != hipSuccess) return attr_n;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(mrp_cf::Geo<4>::THREADS), lds, static_cast<hipStream_t>(stream), a);
  return hipGetLastError();
}

extern "C" int mrp_compress_film_fwd(const float* x, int64_t x_node_stride, const float* gb, int32_t num_graphs,
                                     int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges,
                                     int32_t C, int32_t P, int32_t mode_flags, const float* wt, const float* bias,
                                     float* y, int64_t y_node_stride, void* stream) {
  const int32_t logits = (mode_flags & MRP_AGG_GB_LOGITS) ? 1 : 0;
  const int32_t mode = mode_flags & ~MRP_AGG_GB_LOGITS;
  if (num_graphs < 0 || C < 0 || P < 0 || mode < MRP_AGG_FILM_MEAN || mode > MRP_AGG_COPY_MEAN)
    return hipErrorInvalidValue;
  if (graph_kind != MRP_GRAPH_COMPLETE || max_nodes < 2 || max_nodes > 8 || P % mrp_cf::TP != 0 ||
      C % 128 != 0 || C == 0)
    return hipErrorNotSupported;
  if ((int64_t)num_graphs * max_nodes != num_nodes ||
      (int64_t)num_graphs * max_nodes * (max_nodes - 1) != num_edges)
    return hipErrorInvalidValue;
  if (num_graphs == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (x == nullptr || y == nullptr || wt == nullptr || x_node_stride < plane || y_node_stride < plane)
    return hipErrorInvalidValue;
  if (mode != MRP_AGG_COPY_MEAN && gb == nullptr) return hipErrorInvalidValue;
  if ((reinterpret_cast<uintptr_t>(wt) & 15) != 0) return hipErrorInvalidValue;  // float4 W loads
  // buffer-load byte offsets are 31-bit: x of one graph, the (2C, C) weight
  if ((int64_t)(max_nodes - 1) * x_node_stride * 4 + plane * 4 >= (1LL << 31) || (int64_t)2 * C * C * 4 >= (1LL << 31))
    return hipErrorNotSupported;
  mrp_cf::Args a;
  a.x = x;
  a.xs = x_node_stride;
  a.gb = gb;
  a.wt = wt;
  a.bias = bias;
  a.y = y;
  a.ys = y_node_stride;
  a.C = C;
  a.P = P;
  a.ntiles_p = P / mrp_cf::TP;
  a.mode = mode;
  a.logits = logits;
  a.debug = mrp_cf_debug;
  a.stamps = mrp_cf_stamps;
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (max_nodes) {
    case 2: return launch<2>(a, num_graphs, st);
    case 3: return launch<3>(a, num_graphs, st);
    case 4: return launch<4>(a, num_graphs, st);
    case 5: return launch<5>(a, num_graphs, st);
    case 6: return launch<6>(a, num_graphs, st);
    case 7: return launch<7>(a, num_graphs, st);
    case 8: return launch<8>(a, num_graphs, st);
    default: return hipErrorNotSupported;
  }
}
