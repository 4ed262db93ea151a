// compress_gemm.hip — the GCN layer's 1x1 compress convolution and both of its gradients as fp32
// matrix-core GEMMs over the node-major feature layout, gfx950 (MI355X / CDNA4).
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:163-165,181-184,186-189):
//     h = torch.cat((h, g_h), dim=1)          # (Nt, 2C, H, W)
//     h = self.conv1(h)                        # nn.Conv2d(2C, C, kernel_size=1)
// trained through autograd (dgl/training.py:208-210).  With x = h, a = g_h (the aggregate), W the
// (C, 2C) weight and P = H W pixels per node, the three products are
//     forward      y[n]  = W [x[n]; a[n]] + b                      M = C,  K = 2C, columns = Nt P
//     data grad    [dx[n]; da[n]] = W^T dy[n]                      M = 2C, K = C,  columns = Nt P
//     weight grad  dW = sum_n dy[n] [x[n]; a[n]]^T, db = sum dy    M = C,  N = 2C, K = Nt P
// The concatenation is never formed: the forward reads its K rows from two tensors (x, a) and the data
// gradient writes its M rows to two tensors (dx, da), each with its own node stride — so the cat
// buffer's halves, separate tensors, or any node-strided views all work.
//
// Kernel family (template Cfg<MF, BK, NBUF, WM, WN>): a workgroup of WM x WN waves owns a
// (64 WM) x (64 WN) output tile, each wave 64 x 64, accumulated over K stages of BK on fp32 MFMAs
// (MF = 16: v_mfma_f32_16x16x4_f32, 4 x 4 blocks per wave; MF = 32: v_mfma_f32_32x32x2_f32, 2 x 2
// blocks) — f32 in, f32 accumulate: exact fp32 products, an fmaf chain per output.  Operands are
// staged HBM -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPRs, one instruction per KiB) into
// NBUF LDS buffers, NBUF - 1 stages in flight while one is multiplied.  The LDS images are
// lane-linear (what LDS-DMA writes); the bank swizzle is applied to the per-lane SOURCE address
// instead (cdna_hip_programming.md §5, glds caveat):
//   A image  [row][k (BK)]       16-byte chunk c of row r stored at c ^ swz(r): (r >> 1) & 7 at BK 32,
//                                r & 15 at BK 64
//   B image  NN: [k (BK)][col]   chunk c of row k stored at c ^ (((k >> 2) & 3) << 2)
//            NT: [col][k (BK)]   like the A image
// so the fragment reads (ds_read_b128 of a lane's consecutive k, ds_read_b32 of consecutive columns)
// meet every bank once per lane group (MI355X_MICROARCH.md §LDS).  A lane's k-steps within a 16-k
// group use k = 4q + t (MF 16, q = lane >> 4) or 8h + t (MF 32, h = lane >> 5): the same permutation
// on both operands, so each MFMA still sums matching k and a lane's A values are 16-byte reads.
//
// Weight gradient: K = Nt P is long and the output small, so it is split over K (ranges of whole
// stages) into a workspace of per-split partial tiles, summed in a fixed order by a second kernel
// (deterministic, no atomics); db is the row sum of the dy operand, accumulated from the A fragments
// by the waves of the first column tile.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mrp_gnn.h"
#include "tuning.hpp"

namespace mrp_cg {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

template <int MF_, int BK_, int NBUF_, int WM_, int WN_, int WT_ = 64>
struct Cfg {
  static constexpr int MF = MF_, BK = BK_, NBUF = NBUF_, WM = WM_, WN = WN_;
  static constexpr int WT = WT_;  // wave tile WT x WT (64, or 32 for small products)
  static constexpr int TM = WT * WM, TN = WT * WN;
  static constexpr int NW = WM * WN, THREADS = 64 * NW;
  static constexpr int A_FLOATS = TM * BK, B_FLOATS = BK * TN, BUF = A_FLOATS + B_FLOATS;
  static constexpr int LDS = NBUF * BUF * 4;
  static constexpr int WG_PER_CU = LDS <= 80 * 1024 ? 2 : 1;
  static constexpr int A_PIECES = A_FLOATS / 256, B_PIECES = B_FLOATS / 256;  // 1 KiB LDS-DMA pieces
  static constexpr int PA = A_PIECES / NW, PB = B_PIECES / NW;                  // per wave per stage
  static constexpr int CPR = BK / 4;                                           // 16-B chunks per A-image row
  static constexpr int RPP = 64 / CPR;                                         // A-image rows per piece
  static constexpr int CPRB = TN / 4;                                          // chunks per NN-B row
  static constexpr int RPPB = 64 / CPRB;                                       // NN-B rows per piece
  static constexpr int FB = WT / MF;                                           // fragment blocks per wave side
  static constexpr int T = MF == 16 ? 4 : 8;                                   // k-steps per 16-k group
  static constexpr int CH = MF == 16 ? 1 : 2;                                  // 16-B A reads per group
  static_assert(A_PIECES % NW == 0 && B_PIECES % NW == 0, "pieces must divide over the waves");
  static_assert(BK == 32 || BK == 64, "BK");
  static_assert(RPPB >= 1, "TN");
};

// the product configuration: 128 x 128 workgroup tiles of 2 x 2 waves on 32x32x2 MFMAs, BK 32, two
// LDS buffers (64 KiB: two workgroups per CU).  Round 3's other configurations (16x16x4 MFMAs, three
// or four buffers, 256 x 128 tiles) measured within 1-2 % of it or behind (tools/exp_gemm.py) and
// are no longer built.
using V1 = Cfg<32, 32, 2, 2, 2>;

// Buffer resource over `base` (raw, offsets in bytes; the range check is never reached: every lane
// offset is clamped into its tensor on the host side of the kernel)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}

// One 1 KiB LDS-DMA piece: lane l's 16 bytes from base + voff + soff land at lds + 16 l.  The
// per-lane part (voff) is fixed for the whole K loop, the per-stage advance is the scalar soff.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, f4* lds, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, lds, 16, voff, soff, 0, 0);
}

// Bijective block -> work-item remap: blocks orig, orig + 8, ... run on the same XCD (the dispatcher
// deals blocks round-robin over the 8 XCDs) and get consecutive ids, so tiles that share an operand
// share that XCD's L2 (cdna_hip_programming.md, XCD swizzle).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

template <int BK>
__device__ __forceinline__ int swz_a(int row) {
  return BK == 32 ? (row >> 1) & 7 : row & 15;
}

// The K loop, two LDS buffers, software-pipelined across the barrier.  Per stage s (buffer s & 1) the
// fragments of group g + 1 are read before the MFMAs of group g; before the last group's MFMAs the
// wave retires its LDS-DMA pieces of stage s + 1 (vmcnt: the barrier's fence does not count DMA
// writes) and passes the barrier that (a) publishes stage s + 1 to every wave and (b) certifies that
// every wave holds its stage-s fragments in registers, so stage s + 2 may be DMA'd into buffer s & 1;
// then stage s + 1's first fragments are read under stage s's last MFMA group.  One barrier per
// stage and no LDS latency exposed after it.  The loop is unrolled by 2 so every LDS offset is an
// immediate.  issue(stage, buf), read(buf, g, frags), mma(frags).
// Stages in flight: the prologue issues stages 0 .. NBUF-1 (one per buffer); at stage s's barrier
// buffer s % NBUF has been read by every wave, so stage s + NBUF is issued into it.  The wait before
// a barrier retires the stage it publishes and leaves the younger ones outstanding (counted vmcnt),
// and the barrier is the raw s_barrier (__syncthreads() would wait vmcnt(0) and drain them).
template <class G>
__device__ __forceinline__ void stage_barrier(int younger) {  // younger: stages issued after the one waited for
  constexpr int PS = G::PA + G::PB;  // LDS-DMA pieces per wave per stage
  if (younger >= 3)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PS) : "memory");
  else if (younger == 2)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PS) : "memory");
  else if (younger == 1)
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PS) : "memory");
  else
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

// PRE_ISSUED: the caller has already issued stages 0 .. min(NBUF, nst) - 1 (the encoder overlaps
// their latency with its own prologue).
template <class G, bool PRE_ISSUED = false, class Issue, class Read, class Mma>
__device__ __forceinline__ void kloop(int nst, Issue&& issue, Read&& read, Mma&& mma) {
  constexpr int NB = G::NBUF;
  static_assert(NB >= 2 && NB <= 4, "kloop: 2 to 4 LDS buffers");
  constexpr int NG = G::BK / 16;
  typedef float Frag[2][G::FB][G::T];  // [A | B][block][k-step]
  Frag f[2];
  if (nst <= 0) return;
  if constexpr (!PRE_ISSUED) {
#pragma unroll
    for (int p = 0; p < NB; ++p)
      if (p < nst) issue(p, p);
  }
  stage_barrier<G>(min(NB - 1, nst - 1));  // stage 0 landed; stages 1 .. NB-1 may still be in flight
  read(0, 0, f[0]);
  for (int s0 = 0; s0 < nst; s0 += NB) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int s = s0 + b;
      if (s < nst) {
#pragma unroll
        for (int g = 0; g < NG; ++g) {
          if (g + 1 < NG) {
            read(b, g + 1, f[(g + 1) & 1]);
          } else if (s + 1 < nst) {
            stage_barrier<G>(min(NB - 2, nst - 2 - s));  // stage s + 1 landed; s + 2 .. s + NB - 1 in flight
            if (s + NB < nst) issue(s + NB, b);  // into the buffer stage s just vacated
            read((b + 1) % NB, 0, f[(g + 1) & 1]);
          }
          mma(f[g & 1]);
        }
      }
    }
  }
}

template <int MF>
struct Acc;
template <>
struct Acc<16> {
  typedef f4 T;
  static constexpr int R = 4;
  __device__ static T mfma(float a, float b, T c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
  // accumulator register r of lane l: row 4 (l >> 4) + r, col l & 15
  __device__ static int row(int lane, int r) { return 4 * (lane >> 4) + r; }
  __device__ static int col(int lane) { return lane & 15; }
};
template <>
struct Acc<32> {
  typedef f16v T;
  static constexpr int R = 16;
  __device__ static T mfma(float a, float b, T c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }
  // accumulator register r of lane l: row 8 (r >> 2) + (r & 3) + 4 (l >> 5), col l & 31
  __device__ static int row(int lane, int r) { return 8 * (r >> 2) + (r & 3) + 4 * (lane >> 5); }
  __device__ static int col(int lane) { return lane & 31; }
};

// Per-lane float offsets of the fragment reads within one stage buffer.  The swizzle of an A-type
// row depends only on the row's low bits, i.e. on the lane, so block mb of the wave is the same
// offset + mb MF BK (an immediate), and group g of the NN-B image is + 16 g TN.
//   A-type image (rows r = rbase + lane's row, k chunk per group g and read e):
//     MF 16: chunk 4g + q;  MF 32: chunk 4g + 2h + e
template <class G>
__device__ __forceinline__ void a_offsets(int rbase, int lane, int (&off)[G::BK / 16][G::CH]) {
  const int row = rbase + Acc<G::MF>::col(lane);
  const int sw = swz_a<G::BK>(row);
#pragma unroll
  for (int g = 0; g < G::BK / 16; ++g)
#pragma unroll
    for (int e = 0; e < G::CH; ++e) {
      const int ch = G::MF == 16 ? 4 * g + (lane >> 4) : 4 * g + 2 * (lane >> 5) + e;
      off[g][e] = row * G::BK + 4 * (ch ^ sw);
    }
}
//   NN-B image [k][TN]: lane's k for step t of group g: MF 16: 16g + 4q + t; MF 32: 16g + 8h + t.
//   off[nb][t >> 2] is the offset at g = 0, t & 3 = 0; step (g, t) adds (16 g + (t & 3)) TN.
template <class G>
__device__ __forceinline__ void bnn_offsets(int cbase, int lane, int (&off)[G::FB][G::CH]) {
#pragma unroll
  for (int nb = 0; nb < G::FB; ++nb)
#pragma unroll
    for (int tb = 0; tb < G::CH; ++tb) {
      const int col = cbase + nb * G::MF + Acc<G::MF>::col(lane);
      const int k = G::MF == 16 ? 4 * (lane >> 4) : 8 * (lane >> 5) + 4 * tb;
      off[nb][tb] = k * G::TN + 4 * ((col >> 2) ^ (((k >> 2) & 3) << 2)) + (col & 3);
    }
}

template <class G>
__device__ __forceinline__ void read_a(const float* buf, const int (&off)[G::BK / 16][G::CH], int g, int mb,
                                       float (&v)[G::T]) {
#pragma unroll
  for (int e = 0; e < G::CH; ++e) {
    const f4 x = *reinterpret_cast<const f4*>(buf + off[g][e] + mb * G::MF * G::BK);
    v[4 * e] = x.x, v[4 * e + 1] = x.y, v[4 * e + 2] = x.z, v[4 * e + 3] = x.w;
  }
}

template <class G>
__device__ __forceinline__ void read_bnn(const float* buf, const int (&off)[G::FB][G::CH], int g, int nb,
                                         float (&v)[G::T]) {
#pragma unroll
  for (int t = 0; t < G::T; ++t) v[t] = buf[off[nb][t >> 2] + (16 * g + (t & 3)) * G::TN];
}

template <class G, class AT>
__device__ __forceinline__ void mma_group(AT (&acc)[G::FB][G::FB], const float (&af)[G::FB][G::T],
                                          const float (&bf)[G::FB][G::T]) {
#pragma unroll
  for (int t = 0; t < G::T; ++t)
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb)
#pragma unroll
      for (int nb = 0; nb < G::FB; ++nb) acc[mb][nb] = Acc<G::MF>::mfma(af[mb][t], bf[nb][t], acc[mb][nb]);
}

// ------------------------------------------------------------------------------------------------
// NN: out[n] (M x P) = A (M x K, row-major) . B[n] (K x P), K rows of B from two node-major tensors
// (rows [0, k0) from b0, [k0, K) from b1; k0 % BK == 0, K % BK == 0), M rows of out to two (rows
// [0, m0) to c0, [m0, M) to c1).  Columns are the flattened (node, pixel) index, so a tile may span
// nodes (P < TN) or be part of one.
// ------------------------------------------------------------------------------------------------
struct NNArgs {
  const float* a;
  int64_t lda;
  const float* b0;
  int64_t b0s;
  const float* b1;
  int64_t b1s;
  float* c0;
  int64_t c0s;
  float* c1;
  int64_t c1s;
  const float* bias;  // (M) or null
  int64_t ncols;      // nodes * P
  int32_t M, K, k0, m0, P, mtiles;
};

template <class G>
__global__ void __launch_bounds__(G::THREADS, G::WG_PER_CU) gemm_nn(NNArgs a) {
  using AC = Acc<G::MF>;
  extern __shared__ f4 smem4[];
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = id % a.mtiles, nt = id / a.mtiles;  // the m tiles of one column tile share an XCD
  const int mbase = mt * G::TM;
  const int64_t nbase = (int64_t)nt * G::TN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // ---- LDS-DMA pieces (per stage A_PIECES + B_PIECES of 1 KiB; wave w issues pieces w, w + NW, ...)
  // A piece j: image rows RPP j .. (lane -> row RPP j + lane / CPR, stored chunk lane % CPR)
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.a + (int64_t)mbase * a.lda);
  uint32_t va[G::PA];
#pragma unroll
  for (int jj = 0; jj < G::PA; ++jj) {
    const int row = G::RPP * (w + jj * G::NW) + lane / G::CPR;
    const int c = (lane % G::CPR) ^ swz_a<G::BK>(row);
    const int r = min(row, a.M - 1 - mbase);  // rows past M: any valid data, never stored
    va[jj] = (uint32_t)(((int64_t)r * a.lda + 4 * c) * 4);
  }
  // B piece j: k rows RPPB j .. (lane -> row RPPB j + lane / CPRB); a lane's column (node, pixel) is
  // fixed, relative to the tile's first node
  const int64_t nfirst = nbase / a.P;
  const __amdgpu_buffer_rsrc_t rb0 = rsrc(a.b0 + nfirst * a.b0s), rb1 = rsrc(a.b1 + nfirst * a.b1s);
  uint32_t vb0[G::PB], vb1[G::PB];
#pragma unroll
  for (int jj = 0; jj < G::PB; ++jj) {
    const int row = G::RPPB * (w + jj * G::NW) + lane / G::CPRB;
    const int c = (lane % G::CPRB) ^ (((row >> 2) & 3) << 2);
    int64_t col = nbase + 4 * c;
    if (col > a.ncols - 4) col = a.ncols - 4;  // columns past the end: any valid data, never stored
    const int64_t node = col / a.P;
    const int64_t p = col - node * a.P;
    vb0[jj] = (uint32_t)(((node - nfirst) * a.b0s + p + (int64_t)row * a.P) * 4);
    vb1[jj] = (uint32_t)(((node - nfirst) * a.b1s + p + (int64_t)row * a.P) * 4);
  }
  const int ks0 = a.k0 / G::BK;
  const uint32_t bstage = (uint32_t)(G::BK * a.P * 4);
  auto issue = [&](int s, int buf) {
#pragma unroll
    for (int jj = 0; jj < G::PA; ++jj)
      dma16(ra, &smem4[(buf * G::BUF + (w + jj * G::NW) * 256) / 4], va[jj], (uint32_t)(s * G::BK * 4));
    if (s < ks0) {
#pragma unroll
      for (int jj = 0; jj < G::PB; ++jj)
        dma16(rb0, &smem4[(buf * G::BUF + G::A_FLOATS + (w + jj * G::NW) * 256) / 4], vb0[jj], s * bstage);
    } else {
#pragma unroll
      for (int jj = 0; jj < G::PB; ++jj)
        dma16(rb1, &smem4[(buf * G::BUF + G::A_FLOATS + (w + jj * G::NW) * 256) / 4], vb1[jj], (s - ks0) * bstage);
    }
  };

  const int wm = w / G::WN, wn = w % G::WN;
  int aoff[G::BK / 16][G::CH], boff[G::FB][G::CH];
  a_offsets<G>(wm * G::WT, lane, aoff);
  bnn_offsets<G>(wn * G::WT, lane, boff);
  typename AC::T acc[G::FB][G::FB];
#pragma unroll
  for (int mb = 0; mb < G::FB; ++mb)
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb)
#pragma unroll
      for (int r = 0; r < AC::R; ++r) acc[mb][nb][r] = 0.f;

  const float* smem = reinterpret_cast<const float*>(smem4);
  auto read = [&](int buf, int g, float (&fr)[2][G::FB][G::T]) {
    const float* As = smem + buf * G::BUF;
    const float* Bs = As + G::A_FLOATS;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb) read_a<G>(As, aoff, g, mb, fr[0][mb]);
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb) read_bnn<G>(Bs, boff, g, nb, fr[1][nb]);
  };
  auto mma = [&](const float (&fr)[2][G::FB][G::T]) { mma_group<G>(acc, fr[0], fr[1]); };
  kloop<G>(a.K / G::BK, issue, read, mma);

  // ---- epilogue: accumulator (row, col) of each block, + bias, to the row's destination
#pragma unroll
  for (int nb = 0; nb < G::FB; ++nb) {
    const int64_t col = nbase + wn * G::WT + nb * G::MF + AC::col(lane);
    if (col >= a.ncols) continue;
    const int64_t node = col / a.P;
    const int64_t p = col - node * a.P;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb) {
#pragma unroll
      for (int r = 0; r < AC::R; ++r) {
        const int row = mbase + wm * G::WT + mb * G::MF + AC::row(lane, r);
        if (row >= a.M) continue;
        float v = acc[mb][nb][r];
        if (a.bias != nullptr) v = __fadd_rn(v, a.bias[row]);
        float* dst = row < a.m0 ? a.c0 + node * a.c0s + (int64_t)row * a.P + p
                                : a.c1 + node * a.c1s + (int64_t)(row - a.m0) * a.P + p;
        *dst = v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// NT: partial[split] (M x N) = sum over k in the split's range of A[m][k] B[n][k], with k the flattened
// (node, pixel) index: A = dy (nodes, M, P); B rows [0, n0) from s0 (nodes, n0, P), [n0, N) from s1
// (n0 % 8 == 0).  P % BK == 0, so a stage lies in one node.  Row sums of A (db) by the waves of column
// tile 0 when outb != null.
// ------------------------------------------------------------------------------------------------
struct NTArgs {
  const float* g;
  int64_t gs;
  const float* s0;
  int64_t s0s;
  const float* s1;
  int64_t s1s;
  float* out;      // [split][M][N]
  float* outb;     // [split][M] or null
  const float* colbias;  // (N) added to out (one split only), or null
  int64_t ktot;    // nodes * P
  int64_t kchunk;  // k per split, a multiple of BK
  int32_t M, N, n0, P, mtiles, ntiles;
};

template <class G>
__global__ void __launch_bounds__(G::THREADS, G::WG_PER_CU) gemm_nt(NTArgs a) {
  using AC = Acc<G::MF>;
  extern __shared__ f4 smem4[];
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles = a.mtiles * a.ntiles;
  const int split = id / tiles;
  const int tid = id - split * tiles;
  const int mt = tid % a.mtiles, nt = tid / a.mtiles;
  const int mbase = mt * G::TM, nbase = nt * G::TN;
  const int64_t kbeg = (int64_t)split * a.kchunk;
  const int64_t kend = kbeg + a.kchunk < a.ktot ? kbeg + a.kchunk : a.ktot;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  // operands relative to the split's first node; a piece's rows RPP j .. RPP j + RPP - 1 (lane ->
  // row RPP j + lane / CPR, stored chunk lane % CPR); a B piece's rows all come from one tensor
  const int64_t node0 = kbeg / a.P;
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.g + node0 * a.gs + (int64_t)mbase * a.P);
  const __amdgpu_buffer_rsrc_t rx = rsrc(a.s0 + node0 * a.s0s), rg = rsrc(a.s1 + node0 * a.s1s);
  uint32_t va[G::PA], vb[G::PB];
#pragma unroll
  for (int jj = 0; jj < G::PA; ++jj) {
    const int row = G::RPP * (w + jj * G::NW) + lane / G::CPR;
    const int c = (lane % G::CPR) ^ swz_a<G::BK>(row);
    va[jj] = (uint32_t)(((int64_t)min(row, a.M - 1 - mbase) * a.P + 4 * c) * 4);
  }
  bool bhi[G::PB];
#pragma unroll
  for (int jj = 0; jj < G::PB; ++jj) {
    const int row = G::RPP * (w + jj * G::NW) + lane / G::CPR;
    const int c = (lane % G::CPR) ^ swz_a<G::BK>(row);
    bhi[jj] = nbase + G::RPP * (w + jj * G::NW) >= a.n0;  // wave-uniform
    const int n = min(nbase + row, a.N - 1);
    vb[jj] = (uint32_t)(((int64_t)(bhi[jj] ? n - a.n0 : n) * a.P + 4 * c) * 4);
  }
  // stage position (node relative to node0, pixel) of the next stage to issue: scalar bookkeeping
  int st_node = 0, st_p = (int)(kbeg - node0 * a.P);
  auto issue = [&](int, int buf) {  // stages are issued in order: the position advances per call
    const uint32_t sa = (uint32_t)(((int64_t)st_node * a.gs + st_p) * 4);
    const uint32_t sx = (uint32_t)(((int64_t)st_node * a.s0s + st_p) * 4);
    const uint32_t sg = (uint32_t)(((int64_t)st_node * a.s1s + st_p) * 4);
#pragma unroll
    for (int jj = 0; jj < G::PA; ++jj) dma16(ra, &smem4[(buf * G::BUF + (w + jj * G::NW) * 256) / 4], va[jj], sa);
#pragma unroll
    for (int jj = 0; jj < G::PB; ++jj) {
      f4* dst = &smem4[(buf * G::BUF + G::A_FLOATS + (w + jj * G::NW) * 256) / 4];
      if (bhi[jj])
        dma16(rg, dst, vb[jj], sg);
      else
        dma16(rx, dst, vb[jj], sx);
    }
    st_p += G::BK;
    if (st_p == a.P) {
      st_p = 0;
      ++st_node;
    }
  };

  const int wm = w / G::WN, wn = w % G::WN;
  const bool do_db = a.outb != nullptr && nt == 0 && wn == 0;  // wave-uniform
  int aoff[G::BK / 16][G::CH], boff[G::BK / 16][G::CH];
  a_offsets<G>(wm * G::WT, lane, aoff);
  a_offsets<G>(wn * G::WT, lane, boff);
  typename AC::T acc[G::FB][G::FB];
  float dbs[G::FB];
#pragma unroll
  for (int mb = 0; mb < G::FB; ++mb) {
    dbs[mb] = 0.f;
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb)
#pragma unroll
      for (int r = 0; r < AC::R; ++r) acc[mb][nb][r] = 0.f;
  }

  const float* smem = reinterpret_cast<const float*>(smem4);
  auto read = [&](int buf, int g, float (&fr)[2][G::FB][G::T]) {
    const float* As = smem + buf * G::BUF;
    const float* Bs = As + G::A_FLOATS;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb) read_a<G>(As, aoff, g, mb, fr[0][mb]);
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb) read_a<G>(Bs, boff, g, nb, fr[1][nb]);
  };
  auto mma = [&](const float (&fr)[2][G::FB][G::T]) {
    if (do_db) {
#pragma unroll
      for (int mb = 0; mb < G::FB; ++mb) {
        float s4 = 0.f;
#pragma unroll
        for (int t = 0; t < G::T; ++t) s4 += fr[0][mb][t];
        dbs[mb] += s4;
      }
    }
    mma_group<G>(acc, fr[0], fr[1]);
  };
  kloop<G>(kend > kbeg ? (int)((kend - kbeg) / G::BK) : 0, issue, read, mma);

  float* out = a.out + (int64_t)split * a.M * a.N;
#pragma unroll
  for (int nb = 0; nb < G::FB; ++nb) {
    const int col = nbase + wn * G::WT + nb * G::MF + AC::col(lane);
    if (col >= a.N) continue;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb)
#pragma unroll
      for (int r = 0; r < AC::R; ++r) {
        const int row = mbase + wm * G::WT + mb * G::MF + AC::row(lane, r);
        if (row < a.M) out[(int64_t)row * a.N + col] = a.colbias ? __fadd_rn(acc[mb][nb][r], a.colbias[col]) : acc[mb][nb][r];
      }
  }
  if (do_db) {
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb) {
      // a row's k values are spread over the lane groups that share its row index
      float v = dbs[mb];
      if (G::MF == 16) v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int row = mbase + wm * G::WT + mb * G::MF + AC::col(lane);
      if ((G::MF == 16 ? (lane >> 4) : (lane >> 5)) == 0 && row < a.M) a.outb[(int64_t)split * a.M + row] = v;
    }
  }
}

__global__ void __launch_bounds__(256) split_sum(const f4* __restrict__ part, int nsplit, int64_t n4, f4* __restrict__ out,
                                                 const float* __restrict__ partb, int32_t M, float* __restrict__ outb) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t e = tid; e < n4; e += stride) {
    f4 v = part[e];
    for (int s = 1; s < nsplit; ++s) v += part[(int64_t)s * n4 + e];
    out[e] = v;
  }
  if (outb != nullptr)
    for (int64_t m = tid; m < M; m += stride) {
      float v = partb[m];
      for (int s = 1; s < nsplit; ++s) v += partb[(int64_t)s * M + m];
      outb[m] = v;
    }
}

// wt (cols x rows) = w^T for w (rows x cols), 32 x 32 tiles through LDS
__global__ void __launch_bounds__(256) transpose(const float* __restrict__ w, float* __restrict__ wt, int32_t rows, int32_t cols) {
  __shared__ float tile[32][33];
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  const int c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int r = r0 + ty + k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + k][tx] = w[(int64_t)r * cols + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const int c = c0 + ty + k, r = r0 + tx;
    if (r < rows && c < cols) wt[(int64_t)c * rows + r] = tile[tx][ty + k];
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

constexpr int kCUs = 256;
constexpr int64_t kOffMax = (int64_t)1 << 31;  // buffer offsets are 32-bit; keep every one below 2^31

template <class G>
hipError_t launch_nn_cfg(NNArgs a, hipStream_t st) {
  if (a.K % G::BK != 0 || a.k0 % G::BK != 0) return hipErrorNotSupported;
  const int64_t bs = a.b0s > a.b1s ? a.b0s : a.b1s;
  if (((int64_t)G::TM * a.lda + a.K) * 4 >= kOffMax || ((G::TN / a.P + 2) * bs + (int64_t)a.K * a.P) * 4 >= kOffMax)
    return hipErrorNotSupported;
  a.mtiles = (a.M + G::TM - 1) / G::TM;
  const int64_t grid = (int64_t)a.mtiles * ((a.ncols + G::TN - 1) / G::TN);
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nn<G>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(gemm_nn<G>, dim3((unsigned)grid), dim3(G::THREADS), G::LDS, st, a);
  return hipGetLastError();
}

hipError_t launch_nn(const NNArgs& a, hipStream_t st) { return launch_nn_cfg<V1>(a, st); }

// Splits of the weight gradient's K = Nt P: the count that minimises (rounds of resident workgroups)
// x (stages per split), plus the partial-tile traffic of the final sum.  A split spans at most
// max_stages stages (its node range must stay within 32-bit buffer offsets).
struct SplitPlan {
  int nsplit;
  int64_t kchunk;
};

SplitPlan plan_splits(int64_t tiles, int64_t ktot, int64_t M, int64_t N, int bk, int slots, double stage_us,
                      int64_t max_stages) {
  const int64_t stages = ktot / bk;
  SplitPlan best{0, 0};
  double best_cost = 1e300;
  for (int s = 1; s <= 256; ++s) {
    const int64_t per = (stages + s - 1) / s;
    const int64_t used = (stages + per - 1) / per;  // splits actually non-empty
    if (used != s || per > max_stages) continue;
    const int64_t rounds = (tiles * s + slots - 1) / slots;
    // the split sum reads s partial tiles: M N 4 s bytes at ~4 TB/s, plus a launch
    const double cost = (double)rounds * per * stage_us + (s > 1 ? (double)M * N * 4.0 * (s + 1) / 4.0e6 + 4.0 : 0.0);
    if (cost < best_cost) {
      best_cost = cost;
      best = SplitPlan{s, per * bk};
    }
  }
  return best;  // nsplit 0: no plan within the offset limit
}

template <class G>
SplitPlan plan_nt(int64_t M, int64_t N, int64_t ktot, int32_t P, int64_t max_stride) {
  if (P % G::BK != 0 || ktot == 0) return SplitPlan{0, 0};
  const int64_t tiles = ((M + G::TM - 1) / G::TM) * ((N + G::TN - 1) / G::TN);
  // one stage of one workgroup: 2 TM TN BK flops at 1/(256 WG_PER_CU) of ~150 TF/s
  const double stage_us = 2.0 * G::TM * G::TN * G::BK / (150e6 / (kCUs * G::WG_PER_CU));
  // a split's node range (+ 1 for a partial first node) times the largest node stride < 2^31 bytes
  const int64_t max_nodes = kOffMax / (4 * max_stride) - 2;
  if (max_nodes < 1) return SplitPlan{0, 0};
  const int64_t max_stages = max_nodes * P / G::BK;
  return plan_splits(tiles, ktot, M, N, G::BK, kCUs * G::WG_PER_CU, stage_us, max_stages);
}

SplitPlan plan_nt_any(int64_t M, int64_t N, int64_t ktot, int32_t P, int64_t max_stride) {
  return plan_nt<V1>(M, N, ktot, P, max_stride);
}

template <class G>
hipError_t launch_nt_cfg(NTArgs a, int nsplit, hipStream_t st) {
  if ((int64_t)G::TM * a.P * 4 >= kOffMax) return hipErrorNotSupported;
  a.mtiles = (a.M + G::TM - 1) / G::TM;
  a.ntiles = (a.N + G::TN - 1) / G::TN;
  const int64_t grid = (int64_t)a.mtiles * a.ntiles * nsplit;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt<G>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(gemm_nt<G>, dim3((unsigned)grid), dim3(G::THREADS), G::LDS, st, a);
  return hipGetLastError();
}

hipError_t launch_nt(const NTArgs& a, int nsplit, hipStream_t st) { return launch_nt_cfg<V1>(a, nsplit, st); }

}  // namespace mrp_cg

using namespace mrp_cg;

extern "C" int mrp_compress_fwd(const float* x, int64_t x_node_stride, const float* agg, int64_t agg_node_stride,
                                int32_t num_nodes, int32_t C, int32_t P, const float* w, const float* bias, float* y,
                                int64_t y_node_stride, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (num_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (!x || !agg || !w || !y || x_node_stride < plane || agg_node_stride < plane || y_node_stride < plane)
    return hipErrorInvalidValue;
  // 16-byte LDS-DMA pieces: pixel rows and weight rows start on 16-byte boundaries
  if (C % 4 != 0 || P % 4 != 0 || (x_node_stride & 3) || (agg_node_stride & 3) || !aligned16(x) || !aligned16(agg) ||
      !aligned16(w))
    return hipErrorNotSupported;
  NNArgs a;
  a.a = w;
  a.lda = 2 * (int64_t)C;
  a.b0 = x;
  a.b0s = x_node_stride;
  a.b1 = agg;
  a.b1s = agg_node_stride;
  a.c0 = y;
  a.c0s = y_node_stride;
  a.c1 = y;
  a.c1s = y_node_stride;
  a.bias = bias;
  a.ncols = (int64_t)num_nodes * P;
  a.M = C;
  a.K = 2 * C;
  a.k0 = C;
  a.m0 = C;
  a.P = P;
  return launch_nn(a, static_cast<hipStream_t>(stream));
}

extern "C" int mrp_compress_weight_transpose(const float* w, float* wt, int32_t C, void* stream) {
  if (C < 0) return hipErrorInvalidValue;
  if (C == 0) return hipSuccess;
  if (!w || !wt) return hipErrorInvalidValue;
  const int rows = C, cols = 2 * C;
  hipLaunchKernelGGL(transpose, dim3((cols + 31) / 32, (rows + 31) / 32), dim3(256), 0, static_cast<hipStream_t>(stream),
                     w, wt, rows, cols);
  return hipGetLastError();
}

extern "C" int mrp_compress_bwd_data(const float* gy, int64_t gy_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                                     const float* wt, float* gx, int64_t gx_node_stride, float* gagg,
                                     int64_t gagg_node_stride, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (num_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (!gy || !wt || !gx || !gagg || gy_node_stride < plane || gx_node_stride < plane || gagg_node_stride < plane)
    return hipErrorInvalidValue;
  if (C % 4 != 0 || P % 4 != 0 || (gy_node_stride & 3) || !aligned16(gy) || !aligned16(wt)) return hipErrorNotSupported;
  NNArgs a;
  a.a = wt;
  a.lda = C;
  a.b0 = gy;
  a.b0s = gy_node_stride;
  a.b1 = gy;
  a.b1s = gy_node_stride;
  a.c0 = gx;
  a.c0s = gx_node_stride;
  a.c1 = gagg;
  a.c1s = gagg_node_stride;
  a.bias = nullptr;
  a.ncols = (int64_t)num_nodes * P;
  a.M = 2 * C;
  a.K = C;
  a.k0 = C;
  a.m0 = C;
  a.P = P;
  return launch_nn(a, static_cast<hipStream_t>(stream));
}

namespace {
int64_t max3(int64_t a, int64_t b, int64_t c) { return a > b ? (a > c ? a : c) : (b > c ? b : c); }
}  // namespace

extern "C" int64_t mrp_compress_bwd_weight_workspace(int32_t num_nodes, int32_t C, int32_t P, int64_t max_node_stride) {
  if (num_nodes <= 0 || C <= 0 || P <= 0) return 0;
  const int64_t M = C, N = 2 * (int64_t)C;
  const int64_t stride = max_node_stride > (int64_t)C * P ? max_node_stride : (int64_t)C * P;
  const SplitPlan sp = plan_nt_any(M, N, (int64_t)num_nodes * P, P, stride);
  if (sp.nsplit <= 1) return 0;
  return ((int64_t)sp.nsplit * M * N + (int64_t)sp.nsplit * M) * 4;
}

extern "C" int mrp_compress_bwd_weight(const float* gy, int64_t gy_node_stride, const float* x, int64_t x_node_stride,
                                       const float* agg, int64_t agg_node_stride, int32_t num_nodes, int32_t C, int32_t P,
                                       float* gw, float* gbias, void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (C == 0) return hipSuccess;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t M = C, N = 2 * (int64_t)C;
  if (gw == nullptr && gbias == nullptr) return hipSuccess;
  if (num_nodes == 0 || P == 0) {  // empty sum
    if (gw && hipMemsetAsync(gw, 0, M * N * 4, st) != hipSuccess) return hipErrorUnknown;
    if (gbias && hipMemsetAsync(gbias, 0, M * 4, st) != hipSuccess) return hipErrorUnknown;
    return hipSuccess;
  }
  const int64_t plane = (int64_t)C * P;
  if (!gy || !x || !agg || !gw || gy_node_stride < plane || x_node_stride < plane || agg_node_stride < plane)
    return hipErrorInvalidValue;
  if (C % 8 != 0 || P % 4 != 0 || (gy_node_stride & 3) || (x_node_stride & 3) || (agg_node_stride & 3) ||
      !aligned16(gy) || !aligned16(x) || !aligned16(agg) || !aligned16(gw))
    return hipErrorNotSupported;
  const int64_t ktot = (int64_t)num_nodes * P;
  const SplitPlan sp = plan_nt_any(M, N, ktot, P, max3(gy_node_stride, x_node_stride, agg_node_stride));
  if (sp.nsplit == 0) return hipErrorNotSupported;  // P % BK, or node strides beyond 32-bit offsets
  const int64_t need = sp.nsplit == 1 ? 0 : ((int64_t)sp.nsplit * M * N + (int64_t)sp.nsplit * M) * 4;
  if (need > 0 && (workspace == nullptr || workspace_bytes < need || !aligned16(workspace))) return hipErrorInvalidValue;
  float* ws = static_cast<float*>(workspace);
  NTArgs a = {};
  a.g = gy;
  a.gs = gy_node_stride;
  a.s0 = x;
  a.s0s = x_node_stride;
  a.s1 = agg;
  a.s1s = agg_node_stride;
  a.out = sp.nsplit == 1 ? gw : ws;
  a.outb = gbias == nullptr ? nullptr : (sp.nsplit == 1 ? gbias : ws + sp.nsplit * M * N);
  a.ktot = ktot;
  a.kchunk = sp.kchunk;
  a.M = (int32_t)M;
  a.N = (int32_t)N;
  a.n0 = C;
  a.P = P;
  hipError_t e = launch_nt(a, sp.nsplit, st);
  if (e != hipSuccess || sp.nsplit == 1) return e;
  const int64_t n4 = M * N / 4;  // N = 2C, C % 4 == 0
  const int64_t blocks = (n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048;
  hipLaunchKernelGGL(split_sum, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<const f4*>(ws), sp.nsplit, n4,
                     reinterpret_cast<f4*>(gw), a.outb, (int32_t)M, gbias);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Edge encoder, second Linear (dgl/model/models.py:146-149): z = h W2^T + b2 for h (E, C), W2 (2C, C)
// (nn.Linear weight layout), b2 (2C) -> z (E, 2C).  Both operands are K-contiguous (the NT product of
// the weight gradient with one "node" of P = C pixels): 64 x 64 workgroup tiles of four 32 x 32
// waves give E/64 x 2C/64 workgroups (448 at the headline: 1792 edges, C = 512) with the whole
// K = C per workgroup — no split, no partial sums; the bias is added in the epilogue.
// ------------------------------------------------------------------------------------------------
namespace mrp_cg {
using VE1 = Cfg<32, 32, 2, 2, 2, 32>;  // (the 16x16x4 form measured no faster and is no longer built)
}  // namespace mrp_cg

extern "C" int mrp_edge_logits_fwd(const float* h, int32_t num_edges, int32_t C, const float* w2, const float* b2,
                                   float* z, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (!h || !w2 || !z) return hipErrorInvalidValue;
  if (C % VE1::BK != 0 || !aligned16(h) || !aligned16(w2)) return hipErrorNotSupported;
  if ((int64_t)num_edges * C * 4 >= kOffMax || (int64_t)2 * C * C * 4 >= kOffMax) return hipErrorNotSupported;
  NTArgs a = {};
  a.g = h;
  a.gs = (int64_t)num_edges * C;  // one "node": rows m = edges, k = the C hidden units
  a.s0 = w2;
  a.s0s = (int64_t)2 * C * C;
  a.s1 = w2;
  a.s1s = a.s0s;
  a.out = z;
  a.outb = nullptr;
  a.colbias = b2;
  a.ktot = C;
  a.kchunk = C;
  a.M = num_edges;
  a.N = 2 * C;
  a.n0 = 2 * C;  // every B row from w2
  a.P = C;
  hipStream_t st = static_cast<hipStream_t>(stream);
  return launch_nt_cfg<VE1>(a, 1, st);
}
