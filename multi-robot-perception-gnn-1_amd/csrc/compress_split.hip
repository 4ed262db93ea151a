// compress_split.hip — the GCN layer's 1x1 compress convolution (forward and data gradient) on the
// bf16 matrix cores at fp32 accuracy, gfx950 (MI355X / CDNA4).
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:163-165,181-184,186-189):
//     h = self.conv1(torch.cat((h, g_h), dim=1))       # nn.Conv2d(2C, C, kernel_size=1), fp32
// and its input gradient in training (dgl/training.py:208-210).  Per node n, with P = H W pixels:
//     forward      y[n] = W [x[n]; a[n]] + b          M = C,  K = 2C (rows from x, then a)
//     data grad    [dx[n]; da[n]] = W^T dy[n]         M = 2C, K = C  (rows to dx, then da)
// the same NN product as compress_gemm.hip's gemm_nn (which runs it on the fp32 MFMA), here on
// v_mfma_f32_32x32x16_bf16 with the exact three-way bf16 split of encoder_split.hip: every fp32 operand
// x = x0 + x1 + x2 (+ < 2^-24 |x|), each product the sum of the six partial products a_i b_j with
// i + j <= 2, exact in the MFMA and summed in fp32 — as accurate as an fp32 GEMM (the omitted terms are
// below 2^-25 of the product; 6 roundings per 16 k against the fp32 MFMA's 16), at 192 MFMA cycles per
// 16 k instead of 512.
//
// Operands.  A (the weight, M x K) is split and laid out once per weight version by
// mrp_compress_split_pack in per-lane fragment order (16-byte unit ((mb KS + ks) 3 + p) 64 + lane holds
// lane (r, h)'s eight k = 16 ks + 8 h + j of row 32 mb + r, part p) and arrives by LDS-DMA.  B (the
// activations) is node-major NCHW: k = channel rows of P contiguous pixels, i.e. k-strided for the
// MFMA, which wants eight consecutive k per lane.  Each thread loads 16-byte row pieces of the next
// stage into registers, splits them, and stores the three bf16 parts row-major into LDS ([k][column],
// 256-byte rows, 16-byte chunks XOR-swizzled by the row: cdna_hip_programming.md T10 layout (b)); the
// MFMA fragments come back with ds_read_b64_tr_b16, which delivers four k of one column per lane
// (conflict-free on that layout).
//
// Workgroup: a (64 WMW) x 128 output tile of WMW x 2 waves of 64 x 64; K in stages of 32, two LDS
// buffers (A 12 WMW KiB + B 3 x 8 KiB each): stage s + 1's A is DMA'd and its B loaded into registers
// while stage s is multiplied; one barrier per stage.  Product forms: WMW = 4 (8 waves, two per SIMD,
// each B stage split once for 256 rows) on v_mfma_f32_16x16x32_bf16 (4 x 4 tiles of 16 x 16 per wave)
// where M % 256 == 0 — every reference configuration — else WMW = 2 on 32x32x16 (2 x 2 blocks of
// 32 x 32).  The weight gradient (below) runs the same structure on two activation operands, and with
// its dy operand split once (gemm_nt_psa).  Round 4's other forms are lab forms (tools/lab_forms.hip).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <functional>
#include <map>
#include <mutex>
#include <vector>

#include "mrp_gnn.h"
#include "tuning.hpp"

namespace mrp_cs {

typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2 __attribute__((ext_vector_type(2)));

constexpr int TN = 128, BK = 32;
constexpr int B_PART_BYTES = BK * TN * 2;  // one bf16 part of the B stage: 8 KiB

// Workgroup geometry: WMW x 2 waves of 64 x 64, TM = 64 WMW rows.
template <int WMW>
struct Geo {
  static constexpr int TM = 64 * WMW, NW = 2 * WMW, THREADS = 64 * NW;
  static constexpr int A_PIECES = (TM / 32) * (BK / 16) * 3;  // 1 KiB pieces per stage (6 per wave)
  static constexpr int A_BYTES = A_PIECES * 1024;
  static constexpr int BUF_BYTES = A_BYTES + 3 * B_PART_BYTES;
  static constexpr int LDS_BYTES = 2 * BUF_BYTES;  // 96 KiB (WMW 2), 144 KiB (WMW 4)
  static constexpr int BJ = BK * TN / 4 / THREADS;  // 16-byte B pieces per thread per stage
  static constexpr int KR = THREADS / 32;           // B rows per pass
};

__device__ __forceinline__ uint32_t cvt2(f2 x) { return __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf2)); }
__device__ __forceinline__ f2 widen2(uint32_t p) {
  f2 r;
  r.x = __uint_as_float(p << 16);
  r.y = __uint_as_float(p & 0xffff0000u);
  return r;
}

// exact three-way split of two fp32 values: one dword (two bf16) per part
__device__ __forceinline__ void split2(f2 x, uint32_t& a, uint32_t& b, uint32_t& c) {
  a = cvt2(x);
  const f2 r1 = x - widen2(a);
  b = cvt2(r1);
  const f2 r2 = r1 - widen2(b);
  c = cvt2(r2);
}

// The six partial products of one 16-k step into two accumulators: the five small ones (at most 2^-8
// of the product) into `lo`, a0 b0 into `hi`, summed once in the epilogue.  The bf16 MFMA rounds its
// sum into the accumulator to nearest, but where the accumulator is large against the products the
// low-order bits it drops are biased (tools/exp_split_dgrad.py: pixel sums of the data gradient 6x
// the fp32 GEMM's error with one accumulator); with a0 b0 alone in `hi` the long accumulator sees a
// sixth of the additions and the others happen 2^8 lower, and the bias falls to the fp32 GEMM's level.
struct Acc2 {
  f16v hi, lo;
};
__device__ __forceinline__ void mma6(const bf8 (&a)[3], const bf8 (&b)[3], Acc2& acc) {
  acc.lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc.lo, 0, 0, 0);
  acc.hi = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc.hi, 0, 0, 0);
}

// 16x16x32 form of the six partial products (four accumulator registers per 16 x 16 tile)
typedef float f4acc __attribute__((ext_vector_type(4)));
struct Acc2s {
  f4acc hi, lo;
};
__device__ __forceinline__ void mma6_16(const bf8 (&a)[3], const bf8 (&b)[3], Acc2s& acc) {
  acc.lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc.lo, 0, 0, 0);
  acc.lo = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc.lo, 0, 0, 0);
  acc.hi = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc.hi, 0, 0, 0);
}

// byte offset of 16-byte chunk ch (8 columns) of row `row` in a [BK][TN] bf16 image
__device__ __forceinline__ uint32_t boff(int row, int ch) {
  return (uint32_t)(256 * row + 16 * (ch ^ (((row & 3) << 2) | ((row >> 2) & 3))));
}

// A (M x K) = w (row-major, M x K, stride lda) or w^T (w: K x M row-major, stride lda) -> packed parts
__global__ void __launch_bounds__(256) pack(const float* __restrict__ w, int64_t lda, int trans, int M, int K,
                                            u4* __restrict__ out) {
  const int KS = K / 16;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)(M / 32) * KS * 64) return;
  const int lane = (int)(t & 63);
  const int64_t g = t >> 6;  // mb * KS + ks
  const int ks = (int)(g % KS), mb = (int)(g / KS);
  const int m = 32 * mb + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = trans ? w[(int64_t)(k0 + j) * lda + m] : w[(int64_t)m * lda + k0 + j];
  u4 p0, p1, p2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f2 x;
    x.x = v[2 * i];
    x.y = v[2 * i + 1];
    uint32_t e0, e1, e2;
    split2(x, e0, e1, e2);
    p0[i] = e0, p1[i] = e1, p2[i] = e2;
  }
  out[(g * 3 + 0) * 64 + lane] = p0;
  out[(g * 3 + 1) * 64 + lane] = p1;
  out[(g * 3 + 2) * 64 + lane] = p2;
}

struct Args {
  const u4* ap;  // packed A
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
  int32_t group;  // tile order (tile_of)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// Tile t of an mtiles x ntiles grid, in runs of `group` m-tiles walked m fastest (group <= 0: all of
// them, round 4's order).  An XCD runs ~32 consecutive tiles at once (the XCD-aware remap gives it a
// contiguous range), and they share its L2: with group 4 that window is 4 m-tiles x 8 column tiles,
// so the L2 misses per window are 4 row blocks of the packed operand plus 8 column blocks of the
// streamed one — at configs[3] (8 m-tiles x 32 column tiles) 42 MB per XCD against 59 MB for 8 x 4,
// and for its data gradient (16 m-tiles) 21 against 52 MB.
__device__ __forceinline__ void tile_of(int t, int mtiles, int ntiles, int group, int& mt, int& nt) {
  const int gmax = group > 0 && group < mtiles ? group : mtiles;
  const int run = gmax * ntiles;
  const int g = t / run, first = g * gmax;
  const int gm = mtiles - first < gmax ? mtiles - first : gmax;
  const int rem = t - g * run;
  mt = first + rem % gm;
  nt = rem / gm;
}

template <int WMW, bool MF16 = false>
__device__ __forceinline__ void gemm_nn_split_body(const Args& a) {
  using G = Geo<WMW>;
  constexpr int TM = G::TM, NW = G::NW, A_PIECES = G::A_PIECES, A_BYTES = G::A_BYTES, BUF_BYTES = G::BUF_BYTES;
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  // XCD-aware tile order: the m tiles of one column tile run on one XCD and share its L2 (B is read
  // once from HBM per column tile)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  int mt, nt;
  tile_of(id, a.mtiles, nwg / a.mtiles, a.group, mt, nt);
  const int64_t nbase = (int64_t)nt * TN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int KS = a.K / 16, nst = a.K / BK, ks0 = a.k0 / BK, MB = a.M / 32;

  // ---- A: LDS-DMA pieces pc = (mbl 2 + ksl) 3 + p (local m block, 16-k step, part), pc = w + NW i
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.ap);
  uint32_t va[A_PIECES / NW];
#pragma unroll
  for (int i = 0; i < A_PIECES / NW; ++i) {
    const int pc = w + NW * i;
    const int mbl = pc / 6, kp = pc % 6;  // kp = 3 ksl + p
    const int mb = min(mt * (TM / 32) + mbl, MB - 1);  // blocks past M: any valid data, never stored
    va[i] = (uint32_t)((((int64_t)mb * KS * 3 + kp) * 64 + lane) * 16);
  }
  auto issue_a = [&](int s, int buf) {
#pragma unroll
    for (int i = 0; i < A_PIECES / NW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, lds + (buf * BUF_BYTES + (w + NW * i) * 1024) / 16, 16, va[i],
                                               (uint32_t)s * 6 * 1024, 0, 0);
  };

  // ---- B: thread t loads the 16-byte pieces (row (t >> 5) + KR j, columns 4 (t & 31) ..) of a stage
  const int fc = threadIdx.x & 31, kr = threadIdx.x >> 5;
  int64_t col = nbase + 4 * fc;
  if (col > a.ncols - 4) col = a.ncols - 4;  // columns past the end: any valid data, never stored
  const int64_t node = col / a.P, pix = col - node * a.P;
  const float* bp0 = a.b0 + node * a.b0s + pix + (int64_t)kr * a.P;
  const float* bp1 = a.b1 + node * a.b1s + pix + (int64_t)kr * a.P;
  f4 breg[G::BJ];
  auto load_b = [&](int s) {
    const float* p = s < ks0 ? bp0 + (int64_t)s * BK * a.P : bp1 + (int64_t)(s - ks0) * BK * a.P;
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) breg[j] = *reinterpret_cast<const f4*>(p + (int64_t)G::KR * j * a.P);
  };
  auto store_b = [&](int buf) {  // split the registers' stage into the buffer's three part images
    char* bimg = ldsb + buf * BUF_BYTES + A_BYTES;
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) {
      u2 p0, p1, p2;
      f2 lo, hi;
      lo.x = breg[j].x, lo.y = breg[j].y, hi.x = breg[j].z, hi.y = breg[j].w;
      uint32_t l0, l1, l2, h0, h1, h2;
      split2(lo, l0, l1, l2);
      split2(hi, h0, h1, h2);
      p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
      const uint32_t o = boff(kr + G::KR * j, fc >> 1) + 8 * (fc & 1);
      *reinterpret_cast<u2*>(bimg + o) = p0;
      *reinterpret_cast<u2*>(bimg + B_PART_BYTES + o) = p1;
      *reinterpret_cast<u2*>(bimg + 2 * B_PART_BYTES + o) = p2;
    }
  };

  // ---- fragment reads of one 16-k step: A by row pieces (ds_read_b128), B by ds_read_b64_tr_b16
  const int g16 = lane >> 4, i16 = lane & 15, hh = lane >> 5;
  // tr read: lane 4q + p of its 16-lane group reads row r0 + q, columns c0 + 4p .. (c0 = 16 (g16 & 1))
  const int trq = i16 >> 2, trp = i16 & 3;
  auto read_step = [&](int buf, int ksl, bf8 (&af)[2][3], bf8 (&bf)[2][3]) {
    const char* base = ldsb + buf * BUF_BYTES;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int pc = ((2 * wm + mi) * 2 + ksl) * 3 + p;
        af[mi][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + pc * 1024 + lane * 16));
      }
    const char* bimg = base + A_BYTES;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        s4 v[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int row = 16 * ksl + 8 * hh + 4 * t + trq;
          const int ch = (64 * wn + 32 * ni + 16 * (g16 & 1)) / 8 + (trp >> 1);
          const char* addr = bimg + p * B_PART_BYTES + boff(row, ch) + 8 * (trp & 1);
          v[t] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (__attribute__((address_space(3))) s4*)(reinterpret_cast<uintptr_t>(addr)));
        }
        u4 u;
        u.x = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[0], v[0], 0, 1));
        u.y = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[0], v[0], 2, 3));
        u.z = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[1], v[1], 0, 1));
        u.w = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[1], v[1], 2, 3));
        bf[ni][p] = __builtin_bit_cast(bf8, u);
      }
  };

  if constexpr (MF16) {
    // 16x16x32 products over the whole 32-k stage: lane (r16, qq) of a 16 x 16 tile holds k = 8 qq ..
    // 8 qq + 7.  A: 16-row block mi of the wave is half (mi & 1) of 32-row block 2 wm + (mi >> 1); the
    // packed image holds 16-k steps in the 32 x 32 x 16 lane order (lane r + 32 hh: row r, k 8 hh ..),
    // so the lane reads step qq >> 1, slot 16 (mi & 1) + r16 + 32 (qq & 1).  B: the transposing reads of
    // rows 8 qq + 4 t .. + 3 (t = 0, 1), columns 64 wn + 16 ni ...
    const int r16 = lane & 15, qq = lane >> 4;
    uint32_t tr16[4][2];  // byte address of read (ni, t) in buffer 0, part 0
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int t = 0; t < 2; ++t)
        tr16[ni][t] = (uint32_t)reinterpret_cast<uintptr_t>(
            ldsb + A_BYTES + boff(8 * qq + 4 * t + trq, (64 * wn + 16 * ni) / 8 + (trp >> 1)) + 8 * (trp & 1));
    const int aslot = (r16 + 32 * (qq & 1)) * 16;
    const uint32_t abase0 =
        (uint32_t)reinterpret_cast<uintptr_t>(ldsb + aslot + ((4 * wm + (qq >> 1)) * 3) * 1024);
    Acc2s acc[4][4];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;
    issue_a(0, 0);
    load_b(0);
#pragma unroll 1
    for (int s = 0; s < nst; ++s) {
      const int buf = s & 1;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      store_b(buf);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      {  // (scope of the stage's fragments)
        // every fragment read by inline asm (the transposing-read builtin carries no memory operand, so
        // hipcc would wait for the LDS-DMA issued below, which fills the other buffer) with counted
        // waits, in the order the MFMAs need them: A row 0, B columns 0..3, then A row mi + 1 under row
        // mi's MFMAs (lgkmcnt holds at most 15).  2-3 % over one wait for all of them.
        const uint32_t ab = abase0 + (uint32_t)(buf * BUF_BYTES);
        u4 ar[2][3];
        s4 v[4][3][2];
        auto read_a16 = [&](int mi, u4 (&r)[3]) {
#pragma unroll
          for (int p = 0; p < 3; ++p)
            asm volatile("ds_read_b128 %0, %1 offset:%2"
                         : "=v"(r[p])
                         : "v"(ab), "i"((mi >> 1) * 6144 + p * 1024 + 256 * (mi & 1)));
        };
        read_a16(0, ar[0]);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int t = 0; t < 2; ++t)
              asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
                           : "=v"(v[ni][p][t])
                           : "v"(tr16[ni][t] + (uint32_t)(buf * BUF_BYTES)), "i"(p * B_PART_BYTES));
        if (s + 1 < nst) {
          issue_a(s + 1, buf ^ 1);
          load_b(s + 1);
        }
        bf8 bf[4][3];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          u4 (&cur)[3] = ar[mi & 1];
          if (mi < 3) read_a16(mi + 1, ar[(mi + 1) & 1]);
          if (mi > 0) {
            if (mi < 3)
              asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
            else
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            asm volatile("" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]));
          }
#pragma unroll
          for (int ni = 0; ni < 4; ++ni) {
            if (mi == 0) {
              // A row 0 and B columns 0..ni landed: younger are 6 (3 - ni) B reads and A row 1's 3
              if (ni < 2)
                asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory");
              else if (ni == 2)
                asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
              else
                asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
              if (ni == 0) asm volatile("" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]));
#pragma unroll
              for (int p = 0; p < 3; ++p) {
                asm volatile("" : "+v"(v[ni][p][0]), "+v"(v[ni][p][1]));
                u4 u;
                u.x = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[ni][p][0], v[ni][p][0], 0, 1));
                u.y = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[ni][p][0], v[ni][p][0], 2, 3));
                u.z = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[ni][p][1], v[ni][p][1], 0, 1));
                u.w = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[ni][p][1], v[ni][p][1], 2, 3));
                bf[ni][p] = __builtin_bit_cast(bf8, u);
              }
            }
            const bf8 af[3] = {__builtin_bit_cast(bf8, cur[0]), __builtin_bit_cast(bf8, cur[1]),
                               __builtin_bit_cast(bf8, cur[2])};
            mma6_16(af, bf[ni], acc[mi][ni]);
            if (mi == 0 || ni == 3) __builtin_amdgcn_sched_barrier(0);  // keep each wait before its MFMAs
          }
        }
      }
    }
    // Epilogue.  Accumulator register r of lane (r16, qq) of tile (mi, ni): row 16 mi + 4 qq + r, column
    // 16 ni + r16.  Each store is one buffer_store_dword: the lane's byte offset (node, pixel, 4 qq rows)
    // is fixed per ni and the row's part (16 mi + r rows) is a scalar offset; a 16-row block lies on one
    // side of m0 (the launch requires m0 % 64 == 0), so its output tensor is picked per block.  Round 4's
    // per-element 64-bit addressing (an int64 division per column, a bias load and the side select per
    // element: ~1,800 VALU instructions per wave) cost 3-11 % of the kernel (tools/ab_gemm.py).
    const int mb0 = mt * TM + 64 * wm;
    uint32_t vo0[4], vo1[4];  // per ni: byte offset of (node, pixel, row 4 qq) in c0 / c1
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int64_t n = nbase + 64 * wn + 16 * ni + r16;
      const bool live = n < a.ncols;
      const uint32_t nn = (uint32_t)(live ? n : 0);  // the launch requires ncols < 2^31
      const uint32_t nd = nn / (uint32_t)a.P, px = nn - nd * (uint32_t)a.P;
      // columns past the end: an offset past the buffer's 2^31 - 1 bytes, so the store is dropped
      // (the range check covers the lane offset, not the scalar one)
      vo0[ni] = live ? 4u * ((uint32_t)((int64_t)nd * a.c0s) + px + (uint32_t)(4 * qq * a.P)) : 0x80000000u;
      vo1[ni] = live ? 4u * ((uint32_t)((int64_t)nd * a.c1s) + px + (uint32_t)(4 * qq * a.P)) : 0x80000000u;
    }
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      const int mrow = mb0 + 16 * mi;  // the block's first row (wave-uniform)
      const bool side1 = mrow >= a.m0;
      const uint32_t srow = (uint32_t)(side1 ? mrow - a.m0 : mrow);
      const __amdgpu_buffer_rsrc_t rc = rsrc(side1 ? a.c1 : a.c0);
      f4 bv = {0.f, 0.f, 0.f, 0.f};
      if (a.bias != nullptr) {
        const float* bp = a.bias + mrow + 4 * qq;
        bv = {bp[0], bp[1], bp[2], bp[3]};
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t so = 4u * (srow + (uint32_t)r) * (uint32_t)a.P;
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          float v = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
          if (a.bias != nullptr) v = __fadd_rn(v, bv[r]);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, side1 ? vo1[ni] : vo0[ni], so, 0);
        }
      }
    }
    return;
  }

  Acc2 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;

  issue_a(0, 0);
  load_b(0);
#pragma unroll 1
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    // stage s's B registers and A pieces (own) landed; its buffer was last read in stage s - 2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store_b(buf);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage s visible to every wave; every wave is past stage s - 1's reads
    if (s + 1 < nst) {
      issue_a(s + 1, buf ^ 1);
      load_b(s + 1);
    }
#pragma unroll
    for (int ksl = 0; ksl < 2; ++ksl) {
      bf8 af[2][3], bf[2][3];
      read_step(buf, ksl, af, bf);
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) mma6(af[mi], bf[ni], acc[mi][ni]);
    }
  }

  // ---- epilogue: accumulator register r of lane (column l & 31, half hh) is row (r & 3) + 8 (r >> 2) + 4 hh
  const int mbase = mt * TM + 64 * wm;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int64_t n = nbase + 64 * wn + 32 * ni + (lane & 31);
    if (n >= a.ncols) continue;
    const int64_t nd = n / a.P, px = n - nd * a.P;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mbase + 32 * mi + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m >= a.M) continue;
        float v = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
        if (a.bias != nullptr) v = __fadd_rn(v, a.bias[m]);
        float* dst = m < a.m0 ? a.c0 + nd * a.c0s + (int64_t)m * a.P + px
                              : a.c1 + nd * a.c1s + (int64_t)(m - a.m0) * a.P + px;
        *dst = v;
      }
  }
}

__global__ void __launch_bounds__(256, 1) gemm_nn_split_w2(Args a) { gemm_nn_split_body<2>(a); }
__global__ void __launch_bounds__(512, 1) gemm_nn_split_w4_mf16(Args a) { gemm_nn_split_body<4, true>(a); }

constexpr int64_t kOffMax = (int64_t)1 << 31;

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// one instantiation per kernel, so each kernel's LDS attribute is set (once) for that kernel
template <int WMW, void (*K)(Args)>
hipError_t launch_w(Args a, hipStream_t st) {
  using G = Geo<WMW>;
  a.mtiles = (a.M + G::TM - 1) / G::TM;
  const int64_t grid = (int64_t)a.mtiles * ((a.ncols + TN - 1) / TN);
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(K), hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
  if (attr != hipSuccess) return attr;
  a.group = mrp_host::tuning().gemm_group;
  hipLaunchKernelGGL(K, dim3((unsigned)grid), dim3(G::THREADS), G::LDS_BYTES, st, a);
  return hipGetLastError();
}

// the 16x16x32 form's epilogue: 16-row blocks on one side of m0, 32-bit buffer offsets into c0 / c1
bool mf16_ok(const Args& a) {
  if (a.M % 256 != 0 || a.m0 % 64 != 0 || a.ncols >= kOffMax) return false;
  const int64_t nodes = a.ncols / a.P;
  const int64_t r0 = a.m0 < a.M ? a.m0 : a.M, r1 = a.M - r0;
  const int64_t e0 = ((nodes - 1) * a.c0s + r0 * a.P) * 4;
  const int64_t e1 = r1 > 0 ? ((nodes - 1) * a.c1s + r1 * a.P) * 4 : 0;
  return e0 < kOffMax && e1 < kOffMax;
}

hipError_t launch(Args a, hipStream_t st) {
  if (a.K % BK != 0 || a.k0 % BK != 0 || a.M % 32 != 0 || a.P % 4 != 0) return hipErrorNotSupported;
  if ((int64_t)a.M * a.K * 6 >= kOffMax) return hipErrorNotSupported;
  // 256-row workgroups of 8 waves on 16x16x32 MFMAs (each B stage split once for 256 rows) when M is a
  // multiple of 256 (gemm_split 7), else 128-row workgroups of 4 waves on 32x32x16 MFMAs (2).  Round 4's
  // other forms — the 256-row 32x32x16 kernel and the pipelined 16-k-stage ones, 7-12 % slower than 7
  // at every config shape (the smaller MFMA holds a higher clock under the power limit) — are lab forms
  // now (tools/lab_forms.hip).
  int v = mrp_host::tuning().gemm_split;
  const bool mf16 = mf16_ok(a);
  if (v < 0) v = mf16 ? 7 : 2;
  if (v == 7 && mf16) return launch_w<4, gemm_nn_split_w4_mf16>(a, st);
  return launch_w<2, gemm_nn_split_w2>(a, st);
}

// ------------------------------------------------------------------------------------------------
// Weight gradient  dW[m][n] = sum_k dy[m][k] S[n][k],  db[m] = sum_k dy[m][k],  k = (node, pixel):
// both operands are k-contiguous rows (a channel's P pixels of one node), so no transposing read is
// needed — each thread loads 16-byte row pieces of a stage (A = dy: TMW rows, B = [x; agg]: 128 rows,
// 32 pixels of one node), splits them and stores the three bf16 parts as [row][32 k] 64-byte rows (the
// row's four 16-byte chunks rotated by (row >> 2) & 3, so the fragment reads meet every bank once),
// from which a lane's eight consecutive k are one ds_read_b128.  K = Nt P is split over workgroups
// (whole stages, each within one node) into per-split partial tiles summed in a fixed order by
// split_sum_nt (deterministic); db from the fp32 dy pieces as loaded, per split.
// ------------------------------------------------------------------------------------------------
struct NTArgs {
  const float* g;  // dy (nodes, M, P), node stride gs
  int64_t gs;
  const float* s0;  // rows [0, n0) of B: x (nodes, n0, P)
  int64_t s0s;
  const float* s1;  // rows [n0, N): agg
  int64_t s1s;
  float* out;   // [split][M][N]
  float* outb;  // [split][M] or null
  int64_t ktot, kchunk;
  int32_t M, N, n0, P, mtiles, ntiles;
  const u4* ap;  // gemm_nt_psa: the pre-split image of g (split_rows), KS = ktot / 16 16-k steps per row block
  int32_t group;  // tile order (tile_of)
};

template <int WMW>
struct NTGeo {
  static constexpr int TM = 64 * WMW, NW = 2 * WMW, THREADS = 64 * NW;
  static constexpr int ROWB = BK * 2;                                  // bytes per [row][32 k] bf16 row
  static constexpr int A_PART = TM * ROWB, B_PART = TN * ROWB;
  static constexpr int BUF_BYTES = 3 * (A_PART + B_PART);
  static constexpr int LDS_BYTES = 2 * BUF_BYTES;                      // 144 KiB at WMW 4
  static constexpr int RPP = THREADS / 8;                              // rows per load pass (8 pieces a row)
  static constexpr int AJ = TM / RPP, BJ = TN / RPP;                   // A / B pieces per thread per stage
};

__device__ __forceinline__ uint32_t rowoff(int row, int chunk) {  // [row][4 chunks of 16 B], rotated
  return (uint32_t)(64 * row + 16 * (chunk ^ ((row >> 2) & 3)));
}


// The products on v_mfma_f32_16x16x32_bf16 (the wave's 64 x 64 as 4 x 4 tiles of 16 x 16, one MFMA per
// 32 k), which holds a higher clock than the 32x32x16 shape under the chip's power limit
// (MI355X_MICROARCH.md, DVFS give-back item 7); the 32x32x16 forms are lab forms (tools/lab_forms.hip)
template <int WMW>
__device__ __forceinline__ void gemm_nt_split_body(const NTArgs& a, int orig, int nwg) {
  using G = NTGeo<WMW>;
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int q8 = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + orig / 8;
  const int tiles = a.mtiles * a.ntiles;
  const int split = id / tiles, tid = id - split * tiles;
  int mt, nt;
  tile_of(tid, a.mtiles, a.ntiles, a.group, mt, nt);
  const int mbase = mt * G::TM, nbase = nt * TN;
  const int64_t kbeg = (int64_t)split * a.kchunk;
  const int64_t kend = kbeg + a.kchunk < a.ktot ? kbeg + a.kchunk : a.ktot;
  const int nst = kend > kbeg ? (int)((kend - kbeg) / BK) : 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;

  // ---- loads: thread t -> piece (t & 7) (4 pixels) of rows (t >> 3) + RPP j
  const int pc4 = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  int64_t aoff[G::AJ], boffs[G::BJ];  // row offsets within a node (elements), fixed
  bool bhi[G::BJ];
#pragma unroll
  for (int j = 0; j < G::AJ; ++j) aoff[j] = (int64_t)min(mbase + r0 + G::RPP * j, a.M - 1) * a.P + 4 * pc4;
#pragma unroll
  for (int j = 0; j < G::BJ; ++j) {
    const int n = min(nbase + r0 + G::RPP * j, a.N - 1);
    bhi[j] = n >= a.n0;
    boffs[j] = (int64_t)(bhi[j] ? n - a.n0 : n) * a.P + 4 * pc4;
  }
  f4 areg[G::AJ], breg[G::BJ];
  float rsum[G::AJ];
#pragma unroll
  for (int j = 0; j < G::AJ; ++j) rsum[j] = 0.f;
  // stages in order, k = (node ind, pixel ipx) advanced per stage (P % BK == 0: a stage never straddles
  // two nodes) — an int64 division per stage put ~80 scalar instructions between the barrier and the
  // stage's loads
  int64_t ind = kbeg / a.P;
  int ipx = (int)(kbeg - ind * a.P);
  auto load = [&]() {
    const float* gp = a.g + ind * a.gs + ipx;
    const float* xp = a.s0 + ind * a.s0s + ipx;
    const float* ap = a.s1 + ind * a.s1s + ipx;
#pragma unroll
    for (int j = 0; j < G::AJ; ++j) areg[j] = *reinterpret_cast<const f4*>(gp + aoff[j]);
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) breg[j] = *reinterpret_cast<const f4*>((bhi[j] ? ap : xp) + boffs[j]);
    ipx += BK;
    if (ipx == a.P) {
      ipx = 0;
      ++ind;
    }
  };
  auto store = [&](int buf) {
    char* base = ldsb + buf * G::BUF_BYTES;
    auto put = [&](char* img, int part_bytes, int row, const f4& v) {
      u2 p0, p1, p2;
      f2 lo, hi;
      lo.x = v.x, lo.y = v.y, hi.x = v.z, hi.y = v.w;
      uint32_t l0, l1, l2, h0, h1, h2;
      split2(lo, l0, l1, l2);
      split2(hi, h0, h1, h2);
      p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
      const uint32_t o = rowoff(row, pc4 >> 1) + 8 * (pc4 & 1);
      *reinterpret_cast<u2*>(img + o) = p0;
      *reinterpret_cast<u2*>(img + part_bytes + o) = p1;
      *reinterpret_cast<u2*>(img + 2 * part_bytes + o) = p2;
    };
#pragma unroll
    for (int j = 0; j < G::AJ; ++j) {
      rsum[j] += (areg[j].x + areg[j].y) + (areg[j].z + areg[j].w);
      put(base, G::A_PART, r0 + G::RPP * j, areg[j]);
    }
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) put(base + 3 * G::A_PART, G::B_PART, r0 + G::RPP * j, breg[j]);
  };
  // lane (r16, q) reads k = 8 q .. 8 q + 7 (chunk q) of row r16 of a 16-row block
  const int r16 = lane & 15, q = lane >> 4;
  Acc2s acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;
  if (nst > 0) load();
#pragma unroll 1
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store(buf);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nst) load();
    const char* base = ldsb + buf * G::BUF_BYTES;
    const char* bb = base + 3 * G::A_PART;
    bf8 bf[4][3];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bf[ni][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(bb + p * G::B_PART +
                                                                          rowoff(64 * wn + 16 * ni + r16, q)));
#pragma unroll
    for (int mi = 0; mi < 4; ++mi) {
      bf8 af[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        af[p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + p * G::A_PART +
                                                                      rowoff(64 * wm + 16 * mi + r16, q)));
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) mma6_16(af, bf[ni], acc[mi][ni]);
    }
  }
  float* out = a.out + (int64_t)split * a.M * a.N;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = nbase + 64 * wn + 16 * ni + r16;
    if (n >= a.N) continue;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mbase + 64 * wm + 16 * mi + 4 * q + r;
        if (m < a.M) out[(int64_t)m * a.N + n] = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
      }
  }
  if (a.outb != nullptr && nt == 0) {  // the column-tile-0 workgroups write the split's row sums
#pragma unroll
    for (int j = 0; j < G::AJ; ++j) {
      float v = rsum[j];  // the 8 threads of a row are 8 consecutive lanes (t & 7)
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      v += __shfl_xor(v, 4, 64);
      const int m = mbase + r0 + G::RPP * j;
      if (pc4 == 0 && m < a.M) a.outb[(int64_t)split * a.M + m] = v;
    }
  }
}

__global__ void __launch_bounds__(512, 1) gemm_nt_split_w4_mf16(NTArgs a) {
  gemm_nt_split_body<4>(a, blockIdx.x, gridDim.x);
}

// ------------------------------------------------------------------------------------------------
// Weight gradient with a pre-split A (round 5; split_nt 4, the default where C >= 1024).  The kernel
// above splits BOTH operands in every workgroup: A = dy (M = C rows) is re-split by every column tile
// (2C / 128 of them: 32 at configs[3]) and B = [x; agg] by every row tile (C / 256), three times the
// NN kernel's split work per MFMA (PMC r04: 1.59x its VALU instructions, MFMA busy 0.55 vs 0.66).
// Here dy is split ONCE, by split_rows, into `pack`'s fragment-ordered image (4 bytes read and 6
// written per element, plus the row sums db in fixed-order groups), and arrives by LDS-DMA exactly as
// the NN kernel's weight does; B is split in-kernel as before.  Per output the products and their
// order are gemm_nt_split_body<4, true>'s, so at the same split dW is bit-identical to it.
// ------------------------------------------------------------------------------------------------

// g (nodes, M, P), node stride gs -> the packed A image of the M x K matrix, k = node P + pixel
// (P % 16 == 0): unit ((mb KS + ks) 3 + p) 64 + lane holds lane (r = lane & 31, h = lane >> 5)'s
// k = 16 ks + 8 h .. + 7 of row 32 mb + r, part p — `pack`'s layout.  One wave per (row block mb,
// group of G 16-k steps); its row sums over the group go to rsum[m][group] (null: none), the two lanes
// of a row added in one fixed order.
__global__ void __launch_bounds__(256) split_rows(const float* __restrict__ g, int64_t gs, int32_t M, int32_t P,
                                                  int64_t KS, int32_t G, int32_t ngroups, u4* __restrict__ out,
                                                  float* __restrict__ rsum) {
  const int lane = threadIdx.x & 63;
  const int64_t wv = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  const int MB = M / 32;
  if (wv >= (int64_t)MB * ngroups) return;
  const int mb = (int)(wv % MB), grp = (int)(wv / MB);
  const int r = lane & 31, h = lane >> 5;
  const int64_t ks0 = (int64_t)grp * G;
  const int64_t ks1 = ks0 + G < KS ? ks0 + G : KS;
  int64_t nd = 16 * ks0 / P;  // the step's node and first pixel (P % 16 == 0: a step is within a node)
  int px = (int)(16 * ks0 - nd * P);
  const float* row = g + (int64_t)(32 * mb + r) * P + 8 * h;
  u4* o = out + ((int64_t)mb * KS * 3) * 64 + lane;
  float sum = 0.f;
#pragma unroll 2
  for (int64_t ks = ks0; ks < ks1; ++ks) {
    const float* src = row + nd * gs + px;
    const f4 v0 = *reinterpret_cast<const f4*>(src), v1 = *reinterpret_cast<const f4*>(src + 4);
    sum += ((v0.x + v0.y) + (v0.z + v0.w)) + ((v1.x + v1.y) + (v1.z + v1.w));
    u4 p0, p1, p2;
    const f2 x[4] = {{v0.x, v0.y}, {v0.z, v0.w}, {v1.x, v1.y}, {v1.z, v1.w}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t e0, e1, e2;
      split2(x[i], e0, e1, e2);
      p0[i] = e0, p1[i] = e1, p2[i] = e2;
    }
    u4* d = o + ks * 3 * 64;
    __builtin_nontemporal_store(p0, d);
    __builtin_nontemporal_store(p1, d + 64);
    __builtin_nontemporal_store(p2, d + 128);
    px += 16;
    if (px == P) {
      px = 0;
      ++nd;
    }
  }
  if (rsum != nullptr) {
    const float other = __shfl_xor(sum, 32, 64);
    const float tot = h == 0 ? sum + other : other + sum;
    if (h == 0) rsum[(int64_t)(32 * mb + r) * ngroups + grp] = tot;  // [m][group]: a row's partials contiguous
  }
}

// out[m] = the sum of part[m][0 .. n) in a fixed order: one wave per row, lane l adding partials
// l, l + 64, .. in order, then a fixed xor butterfly (every lane ends with the same value)
__global__ void __launch_bounds__(64) row_sums(const float* __restrict__ part, int32_t n, int32_t M,
                                               float* __restrict__ out) {
  const int m = blockIdx.x, lane = threadIdx.x;
  if (m >= M) return;
  const float* p = part + (int64_t)m * n;
  float v = 0.f;
  for (int i = lane; i < n; i += 64) v += p[i];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) out[m] = v;
}

__device__ __forceinline__ void gemm_nt_psa_body(const NTArgs& a, int orig, int nwg) {
  using G = NTGeo<4>;
  constexpr int A_BYTES = 48 * 1024;  // 256 rows x 32 k x 3 parts: 48 1-KiB pieces, 6 per wave
  constexpr int BP = G::B_PART, BUF = A_BYTES + 3 * BP;  // 72 KiB per buffer, two buffers
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int q8 = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q8 + 1) : rr * (q8 + 1) + (xcd - rr) * q8) + orig / 8;
  const int tiles = a.mtiles * a.ntiles;
  const int split = id / tiles, tid = id - split * tiles;
  int mt, nt;
  tile_of(tid, a.mtiles, a.ntiles, a.group, mt, nt);
  const int mbase = mt * G::TM, nbase = nt * TN;
  const int64_t kbeg = (int64_t)split * a.kchunk;
  const int64_t kend = kbeg + a.kchunk < a.ktot ? kbeg + a.kchunk : a.ktot;
  const int nst = kend > kbeg ? (int)((kend - kbeg) / BK) : 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int64_t KS = a.ktot / 16;
  const int MB = a.M / 32;

  // ---- A: LDS-DMA pieces pc = (mbl 2 + ksl) 3 + p of the stage, pc = w + 8 i
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.ap);
  uint32_t va[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const int pc = w + 8 * i;
    const int mbl = pc / 6, kp = pc % 6;
    const int mb = min(mt * 8 + mbl, MB - 1);  // blocks past M: any valid data, never stored
    va[i] = (uint32_t)((((int64_t)mb * KS + kbeg / 16) * 3 + kp) * 64 + lane) * 16;
  }
  auto issue_a = [&](int s, int buf) {
#pragma unroll
    for (int i = 0; i < 6; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, lds + (buf * BUF + (w + 8 * i) * 1024) / 16, 16, va[i],
                                               (uint32_t)s * 6 * 1024, 0, 0);
  };

  // ---- B: thread t -> piece (t & 7) (4 pixels) of rows (t >> 3) + 64 j of the stage
  const int pc4 = threadIdx.x & 7, r0 = threadIdx.x >> 3;
  int64_t boffs[G::BJ];
  bool bhi[G::BJ];
#pragma unroll
  for (int j = 0; j < G::BJ; ++j) {
    const int n = min(nbase + r0 + G::RPP * j, a.N - 1);
    bhi[j] = n >= a.n0;
    boffs[j] = (int64_t)(bhi[j] ? n - a.n0 : n) * a.P + 4 * pc4;
  }
  f4 breg[G::BJ];
  int64_t ind = kbeg / a.P;
  int ipx = (int)(kbeg - ind * a.P);
  auto load_b = [&]() {
    const float* xp = a.s0 + ind * a.s0s + ipx;
    const float* ap = a.s1 + ind * a.s1s + ipx;
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) breg[j] = *reinterpret_cast<const f4*>((bhi[j] ? ap : xp) + boffs[j]);
    ipx += BK;
    if (ipx == a.P) {
      ipx = 0;
      ++ind;
    }
  };
  auto store_b = [&](int buf) {
    char* img = ldsb + buf * BUF + A_BYTES;
#pragma unroll
    for (int j = 0; j < G::BJ; ++j) {
      u2 p0, p1, p2;
      f2 lo, hi;
      lo.x = breg[j].x, lo.y = breg[j].y, hi.x = breg[j].z, hi.y = breg[j].w;
      uint32_t l0, l1, l2, h0, h1, h2;
      split2(lo, l0, l1, l2);
      split2(hi, h0, h1, h2);
      p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
      const uint32_t o = rowoff(r0 + G::RPP * j, pc4 >> 1) + 8 * (pc4 & 1);
      *reinterpret_cast<u2*>(img + o) = p0;
      *reinterpret_cast<u2*>(img + BP + o) = p1;
      *reinterpret_cast<u2*>(img + 2 * BP + o) = p2;
    }
  };

  // fragments: lane (r16, qq) holds k = 8 qq .. 8 qq + 7 of row r16 of a 16-row block.  A: 16-row block mi
  // of the wave is half (mi & 1) of 32-row block 2 wm + (mi >> 1); the packed image holds 16-k steps in the
  // 32 x 32 x 16 lane order, so the lane reads step qq >> 1, slot 16 (mi & 1) + r16 + 32 (qq & 1) (the NN
  // kernel's A reads).  B: chunk qq of row 64 wn + 16 ni + r16 of the [row][32 k] images.
  const int r16 = lane & 15, qq = lane >> 4;
  const uint32_t abase0 = (uint32_t)reinterpret_cast<uintptr_t>(ldsb + (r16 + 32 * (qq & 1)) * 16 +
                                                                 ((4 * wm + (qq >> 1)) * 3) * 1024);
  uint32_t bro[4];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni)
    bro[ni] = (uint32_t)reinterpret_cast<uintptr_t>(ldsb + A_BYTES + rowoff(64 * wn + 16 * ni + r16, qq));
  Acc2s acc[4][4];
#pragma unroll
  for (int mi = 0; mi < 4; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;
  if (nst > 0) {
    issue_a(0, 0);
    load_b();
  }
#pragma unroll 1
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage s's B registers and own A pieces landed
    store_b(buf);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // stage s complete for every wave; every wave is past stage s - 1's reads
    {
      // every fragment read by inline asm with counted waits (a C++ LDS read beside the LDS-DMA issued
      // below would make hipcc wait for the DMA): A row 0, B columns 0..3, then A row mi + 1 under row
      // mi's MFMAs
      const uint32_t ab = abase0 + (uint32_t)(buf * BUF);
      u4 ar[2][3], br[4][3];
      auto read_a16 = [&](int mi, u4 (&rg)[3]) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(rg[p])
                       : "v"(ab), "i"((mi >> 1) * 6144 + p * 1024 + 256 * (mi & 1)));
      };
      read_a16(0, ar[0]);
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          asm volatile("ds_read_b128 %0, %1 offset:%2"
                       : "=v"(br[ni][p])
                       : "v"(bro[ni] + (uint32_t)(buf * BUF)), "i"(p * BP));
      if (s + 1 < nst) {
        issue_a(s + 1, buf ^ 1);
        load_b();
      }
#pragma unroll
      for (int mi = 0; mi < 4; ++mi) {
        u4 (&cur)[3] = ar[mi & 1];
        if (mi < 3) read_a16(mi + 1, ar[(mi + 1) & 1]);
        if (mi > 0) {
          if (mi < 3)
            asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
          else
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          asm volatile("" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]));
        }
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          if (mi == 0) {
            // A row 0 and B columns 0..ni landed: younger are 3 (3 - ni) B reads and A row 1's 3
            if (ni == 0)
              asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
            else if (ni == 1)
              asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
            else if (ni == 2)
              asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
            else
              asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
            if (ni == 0) asm volatile("" : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]));
            asm volatile("" : "+v"(br[ni][0]), "+v"(br[ni][1]), "+v"(br[ni][2]));
          }
          const bf8 af[3] = {__builtin_bit_cast(bf8, cur[0]), __builtin_bit_cast(bf8, cur[1]),
                             __builtin_bit_cast(bf8, cur[2])};
          const bf8 bfr[3] = {__builtin_bit_cast(bf8, br[ni][0]), __builtin_bit_cast(bf8, br[ni][1]),
                              __builtin_bit_cast(bf8, br[ni][2])};
          mma6_16(af, bfr, acc[mi][ni]);
          if (mi == 0 || ni == 3) __builtin_amdgcn_sched_barrier(0);  // keep each wait before its MFMAs
        }
      }
    }
  }
  float* out = a.out + (int64_t)split * a.M * a.N;
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = nbase + 64 * wn + 16 * ni + r16;
    if (n >= a.N) continue;
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = mbase + 64 * wm + 16 * mi + 4 * qq + r;
        if (m < a.M) out[(int64_t)m * a.N + n] = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
      }
  }
}

__global__ void __launch_bounds__(512, 1) gemm_nt_psa(NTArgs a) { gemm_nt_psa_body(a, blockIdx.x, gridDim.x); }

// the same with the first product's A operand pre-split (gemm_nt_psa_body: the edge encoder's W2^T,
// packed once per weight version) — the split body re-split it once per column tile and call
__global__ void __launch_bounds__(512, 1) gemm_nt_dual_psa1(NTArgs a1, NTArgs a2, int grid1) {
  if ((int)blockIdx.x < grid1)
    gemm_nt_psa_body(a1, blockIdx.x, grid1);
  else
    gemm_nt_split_body<4>(a2, blockIdx.x - grid1, gridDim.x - grid1);
}

// two independent NT products in one launch (the edge encoder's backward), on the default (16x16x32)
// form: workgroups [0, grid1) run a1, the rest a2, each product with its own XCD-aware tile order
__global__ void __launch_bounds__(512, 1) gemm_nt_dual_mf16(NTArgs a1, NTArgs a2, int grid1) {
  if ((int)blockIdx.x < grid1)
    gemm_nt_split_body<4>(a1, blockIdx.x, grid1);
  else
    gemm_nt_split_body<4>(a2, blockIdx.x - grid1, gridDim.x - grid1);
}

// out = sum over the splits of part (fixed order); outb = the same over nsplitb row-sum partials
__global__ void __launch_bounds__(256) split_sum_nt(const f4* __restrict__ part, int nsplit, int64_t n4,
                                                    f4* __restrict__ out, const float* __restrict__ partb,
                                                    int nsplitb, int32_t M, float* __restrict__ outb) {
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
      for (int s = 1; s < nsplitb; ++s) v += partb[(int64_t)s * M + m];
      outb[m] = v;
    }
}

// Splits of K = Nt P (whole stages): the count minimising (rounds of one-per-CU workgroups) x
// (stages per split) plus the partial-tile traffic of the final sum.
int nt_splits(int64_t tiles, int64_t ktot, int64_t M, int64_t N, int64_t* kchunk) {
  const int64_t stages = ktot / BK;
  int best = 1;
  double best_cost = 1e300;
  for (int s = 1; s <= 256; ++s) {
    const int64_t per = (stages + s - 1) / s;
    if ((stages + per - 1) / per != s) continue;  // some split would be empty
    const int64_t rounds = (tiles * s + 255) / 256;
    // one 32-k stage of a 256 x 128 workgroup (12.6 MFLOP of bf16 products on one CU, ~1.3 us at the
    // CU's peak) takes ~1.6 us; the split sum streams the partial tiles at ~4 TB/s plus a launch
    const double cost = (double)rounds * per * 1.6 + (s > 1 ? (double)M * N * 4.0 * (s + 1) / 4.0e6 + 4.0 : 0.0);
    if (cost < best_cost) {
      best_cost = cost;
      best = s;
    }
  }
  *kchunk = ((stages + best - 1) / best) * BK;
  return best;
}

}  // namespace mrp_cs

using namespace mrp_cs;

extern "C" int64_t mrp_compress_split_pack_bytes(int32_t M, int32_t K) {
  if (M <= 0 || K <= 0 || M % 32 != 0 || K % 16 != 0) return 0;
  return (int64_t)M * K * 6;
}

extern "C" int mrp_compress_split_pack(const float* w, int64_t ld, int32_t transpose, int32_t M, int32_t K,
                                       void* packed, void* stream) {
  if (M <= 0 || K <= 0 || ld <= 0) return hipErrorInvalidValue;
  if (M % 32 != 0 || K % 16 != 0) return hipErrorNotSupported;
  if (!w || !packed || !aligned16(packed)) return hipErrorInvalidValue;
  const int64_t threads = (int64_t)(M / 32) * (K / 16) * 64;
  hipLaunchKernelGGL(pack, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream), w,
                     ld, transpose ? 1 : 0, M, K, static_cast<u4*>(packed));
  return hipGetLastError();
}

extern "C" int mrp_compress_fwd_split(const float* x, int64_t x_node_stride, const float* agg, int64_t agg_node_stride,
                                      int32_t num_nodes, int32_t C, int32_t P, const void* packed_w, const float* bias,
                                      float* y, int64_t y_node_stride, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (num_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (!x || !agg || !packed_w || !y || x_node_stride < plane || agg_node_stride < plane || y_node_stride < plane)
    return hipErrorInvalidValue;
  if (C % 32 != 0 || P % 4 != 0 || (x_node_stride & 3) || (agg_node_stride & 3) || !aligned16(x) || !aligned16(agg) ||
      !aligned16(packed_w))
    return hipErrorNotSupported;
  Args a = {};
  a.ap = static_cast<const u4*>(packed_w);
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
  return launch(a, static_cast<hipStream_t>(stream));
}

extern "C" int mrp_compress_bwd_data_split(const float* gy, int64_t gy_node_stride, int32_t num_nodes, int32_t C,
                                           int32_t P, const void* packed_wt, float* gx, int64_t gx_node_stride,
                                           float* gagg, int64_t gagg_node_stride, void* stream) {
  if (num_nodes < 0 || C < 0 || P < 0) return hipErrorInvalidValue;
  if (num_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (!gy || !packed_wt || !gx || !gagg || gy_node_stride < plane || gx_node_stride < plane ||
      gagg_node_stride < plane)
    return hipErrorInvalidValue;
  if (C % 32 != 0 || P % 4 != 0 || (gy_node_stride & 3) || !aligned16(gy) || !aligned16(packed_wt))
    return hipErrorNotSupported;
  Args a = {};
  a.ap = static_cast<const u4*>(packed_wt);
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
  return launch(a, static_cast<hipStream_t>(stream));
}

namespace {
bool nt_split_ok(int32_t num_nodes, int32_t C, int32_t P) {
  return num_nodes > 0 && C > 0 && C % 64 == 0 && P % BK == 0;
}

// workspace bytes of one NT product (split-K partial tiles, and row sums when wanted)
int64_t nt_workspace(int64_t M, int64_t N, int64_t ktot) {
  const int64_t tiles = ((M + NTGeo<4>::TM - 1) / NTGeo<4>::TM) * ((N + TN - 1) / TN);
  int64_t kchunk;
  const int ns = nt_splits(tiles, ktot, M, N, &kchunk);
  return ns <= 1 ? 0 : ((int64_t)ns * M * N + (int64_t)ns * M) * 4;
}

// out (M x N) = sum_k g[m][k] s[n][k] (+ row sums of g into outb), k = (node, pixel) over `nodes` nodes of
// P pixels; a.g/gs, a.s0/s0s, a.s1/s1s, a.n0, a.P set by the caller
hipError_t nt_run(NTArgs a, int64_t M, int64_t N, int32_t nodes, float* out, float* outb, void* workspace,
                  int64_t workspace_bytes, hipStream_t st) {
  using G = NTGeo<4>;
  a.mtiles = (int32_t)((M + G::TM - 1) / G::TM);
  a.ntiles = (int32_t)((N + TN - 1) / TN);
  a.ktot = (int64_t)nodes * a.P;
  const int ns = nt_splits((int64_t)a.mtiles * a.ntiles, a.ktot, M, N, &a.kchunk);
  const int64_t need = ns == 1 ? 0 : ((int64_t)ns * M * N + (int64_t)ns * M) * 4;
  if (need > 0 && (workspace == nullptr || workspace_bytes < need || !aligned16(workspace))) return hipErrorInvalidValue;
  float* ws = static_cast<float*>(workspace);
  a.out = ns == 1 ? out : ws;
  a.outb = outb == nullptr ? nullptr : (ns == 1 ? outb : ws + (int64_t)ns * M * N);
  a.M = (int32_t)M;
  a.N = (int32_t)N;
  const int64_t grid = (int64_t)a.mtiles * a.ntiles * ns;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  // the 32-k-stage form on 16x16x32 MFMAs (split_nt 3; the compress weight gradient takes nt_run_psa
  // instead at 4, and at -1 where C >= 1024).  Round 4's 32x32x16 forms (the 32-k-stage one and the
  // pipelined 16-k-stage one), 4-5 % slower at every config shape, are lab forms (tools/lab_forms.hip).
  static const hipError_t attr16 = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_split_w4_mf16),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
  if (attr16 != hipSuccess) return attr16;
  a.group = mrp_host::tuning().nt_group;
  hipLaunchKernelGGL(gemm_nt_split_w4_mf16, dim3((unsigned)grid), dim3(G::THREADS), G::LDS_BYTES, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || ns == 1) return e;
  const int64_t n4 = M * N / 4;
  const int64_t blocks = (n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048;
  hipLaunchKernelGGL(split_sum_nt, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<const f4*>(ws), ns, n4,
                     reinterpret_cast<f4*>(out), a.outb, ns, (int32_t)M, outb);
  return hipGetLastError();
}

// The pre-split-A weight gradient (split_rows + gemm_nt_psa): workspace = [partial tiles (splits > 1)]
// [dy's packed image, M K 6 bytes][row-sum group partials].  The default (split_nt -1) where C >= 1024
// and the image is addressable with 32-bit buffer offsets; forced by split_nt 4.  The GEMM alone runs
// 15-20 % faster than gemm_nt_split_w4_mf16 at every config shape (configs[3]: 281 vs 333 us,
// 244 TF/s); behind the data gradient in a training step (tools/exp_dy_image.py, HIP graph, the chip at
// its power limit) the pair gains 3 % at C = 1024 / 2048 (configs[4] 1278 vs 1320 us, [3] 626 vs
// 648), 1 % at C = 1280 and loses 4 % at C = 512 (the split pass moves 10 bytes per element of dy
// for a re-split factor of only 2C / 128 = 8 there).
struct PsaPlan {
  int ns, G, ngroups;
  int64_t kchunk, img_off, rs_off, bytes;
};

bool psa_ok(int64_t M, int64_t ktot) {
  const int v = mrp_host::tuning().split_nt;
  return ((v < 0 && M >= 1024) || v == 4) && M % 32 == 0 && ktot % BK == 0 && M * ktot * 6 < kOffMax;
}

PsaPlan psa_plan(int64_t M, int64_t N, int64_t ktot) {
  PsaPlan q{};
  const int64_t tiles = ((M + NTGeo<4>::TM - 1) / NTGeo<4>::TM) * ((N + TN - 1) / TN);
  q.ns = nt_splits(tiles, ktot, M, N, &q.kchunk);
  // split_rows: one wave per (32-row block, group of G 16-k steps), ~8192 waves
  const int64_t KS = ktot / 16, MB = M / 32;
  int64_t G = (KS * MB + 8191) / 8192;
  if (G < 1) G = 1;
  q.G = (int)G;
  q.ngroups = (int)((KS + G - 1) / G);
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  q.img_off = al(q.ns > 1 ? (int64_t)q.ns * M * N * 4 : 0);
  q.rs_off = al(q.img_off + M * ktot * 6);
  q.bytes = q.rs_off + (int64_t)q.ngroups * M * 4;
  return q;
}

// The pre-split-A GEMM proper: dW (+ db from rparts row-sum partials [M][nparts]) from dy's packed
// image `img` (split_rows' layout, or written by the data gradient: mrp_compress_bwd_data_split_img);
// the workspace holds the partial tiles when the plan splits K
hipError_t psa_gemm(NTArgs a, int64_t M, int64_t N, const u4* img, const float* rparts, int nparts, float* out,
                    float* outb, void* tiles_ws, hipStream_t st) {
  using G = NTGeo<4>;
  const PsaPlan q = psa_plan(M, N, a.ktot);
  a.ap = img;
  a.mtiles = (int32_t)((M + G::TM - 1) / G::TM);
  a.ntiles = (int32_t)((N + TN - 1) / TN);
  a.kchunk = q.kchunk;
  a.out = q.ns == 1 ? out : static_cast<float*>(tiles_ws);
  a.outb = nullptr;
  a.M = (int32_t)M;
  a.N = (int32_t)N;
  const int64_t grid = (int64_t)a.mtiles * a.ntiles * q.ns;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_psa),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
  if (attr != hipSuccess) return attr;
  a.group = mrp_host::tuning().nt_group;
  hipLaunchKernelGGL(gemm_nt_psa, dim3((unsigned)grid), dim3(G::THREADS), G::LDS_BYTES, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (outb != nullptr) {
    hipLaunchKernelGGL(row_sums, dim3((unsigned)M), dim3(64), 0, st, rparts, nparts, (int32_t)M, outb);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (q.ns == 1) return hipSuccess;
  const int64_t n4 = M * N / 4;
  const int64_t blocks = (n4 + 255) / 256 < 2048 ? (n4 + 255) / 256 : 2048;
  hipLaunchKernelGGL(split_sum_nt, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<const f4*>(tiles_ws), q.ns,
                     n4, reinterpret_cast<f4*>(out), nullptr, 0, (int32_t)M, nullptr);
  return hipGetLastError();
}

hipError_t nt_run_psa(NTArgs a, int64_t M, int64_t N, int32_t nodes, float* out, float* outb, void* workspace,
                      int64_t workspace_bytes, hipStream_t st) {
  a.ktot = (int64_t)nodes * a.P;
  const PsaPlan q = psa_plan(M, N, a.ktot);
  if (workspace == nullptr || workspace_bytes < q.bytes || !aligned16(workspace)) return hipErrorInvalidValue;
  char* ws = static_cast<char*>(workspace);
  u4* img = reinterpret_cast<u4*>(ws + q.img_off);
  float* rs = reinterpret_cast<float*>(ws + q.rs_off);
  const int64_t waves = (M / 32) * q.ngroups;
  hipLaunchKernelGGL(split_rows, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, a.g, a.gs, (int32_t)M, a.P,
                     a.ktot / 16, q.G, q.ngroups, img, outb != nullptr ? rs : nullptr);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return psa_gemm(a, M, N, img, rs, q.ngroups, out, outb, ws, st);
}

}  // namespace

extern "C" int64_t mrp_compress_bwd_weight_split_workspace(int32_t num_nodes, int32_t C, int32_t P) {
  if (!nt_split_ok(num_nodes, C, P)) return 0;
  const int64_t ktot = (int64_t)num_nodes * P;
  if (psa_ok(C, ktot)) return psa_plan(C, 2 * (int64_t)C, ktot).bytes;
  return nt_workspace(C, 2 * (int64_t)C, ktot);
}

extern "C" int mrp_compress_bwd_weight_split(const float* gy, int64_t gy_node_stride, const float* x,
                                             int64_t x_node_stride, const float* agg, int64_t agg_node_stride,
                                             int32_t num_nodes, int32_t C, int32_t P, float* gw, float* gbias,
                                             void* workspace, int64_t workspace_bytes, void* stream) {
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
  if (!nt_split_ok(num_nodes, C, P) || (gy_node_stride & 3) || (x_node_stride & 3) || (agg_node_stride & 3) ||
      !aligned16(gy) || !aligned16(x) || !aligned16(agg) || !aligned16(gw))
    return hipErrorNotSupported;
  NTArgs a = {};
  a.g = gy;
  a.gs = gy_node_stride;
  a.s0 = x;
  a.s0s = x_node_stride;
  a.s1 = agg;
  a.s1s = agg_node_stride;
  a.n0 = C;
  a.P = P;
  if (psa_ok(M, (int64_t)num_nodes * P))
    return nt_run_psa(a, M, N, num_nodes, gw, gbias, workspace, workspace_bytes, st);
  return nt_run(a, M, N, num_nodes, gw, gbias, workspace, workspace_bytes, st);
}

// The edge encoder's backward GEMMs on the same kernel (training path, encoder.py): operands are rows
// with k contiguous, i.e. one "node" of K pixels:
//   dh^T (C x E)  = W2^T (C x 2C) . dz^T     (k = j: rows of W2^T and of dz)
//   dW2 (2C x C)  = dz^T (2C x E) . h         (k = e: rows of dz^T and of h^T; db2 = its row sums of dz^T)
extern "C" int64_t mrp_edge_encoder_bwd_split_workspace(int32_t num_edges, int32_t C) {
  if (num_edges <= 0 || C <= 0 || num_edges % BK != 0 || C % 32 != 0) return 0;
  const int64_t a = nt_workspace(C, num_edges, 2 * (int64_t)C), b = nt_workspace(2 * (int64_t)C, C, num_edges);
  return a > b ? a : b;
}

extern "C" int mrp_edge_encoder_bwd_split(const float* dz, const float* dzT, const float* w2T, const float* hT,
                                          int32_t num_edges, int32_t C, float* dhT, float* dw2, float* db2,
                                          void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (db2 != nullptr && dw2 == nullptr) return hipErrorInvalidValue;  // db2 rides on the dW2 product
  if (num_edges == 0 || C == 0 || (dhT == nullptr && dw2 == nullptr)) return hipSuccess;
  if (num_edges % BK != 0 || C % 32 != 0) return hipErrorNotSupported;
  if ((dhT && (!dz || !w2T || !aligned16(dz) || !aligned16(w2T) || !aligned16(dhT))) ||
      (dw2 && (!dzT || !hT || !aligned16(dzT) || !aligned16(hT) || !aligned16(dw2))))
    return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t E = num_edges, C2 = 2 * (int64_t)C;
  if (dhT) {
    NTArgs a = {};
    a.g = w2T;  // rows u, k = j
    a.gs = C * C2;
    a.s0 = dz;  // rows e, k = j
    a.s0s = E * C2;
    a.s1 = dz;
    a.s1s = E * C2;
    a.n0 = (int32_t)E;
    a.P = (int32_t)C2;
    const hipError_t e = nt_run(a, C, E, 1, dhT, nullptr, workspace, workspace_bytes, st);
    if (e != hipSuccess) return e;
  }
  if (dw2) {
    NTArgs a = {};
    a.g = dzT;  // rows j, k = e
    a.gs = C2 * E;
    a.s0 = hT;  // rows u, k = e
    a.s0s = (int64_t)C * E;
    a.s1 = hT;
    a.s1s = (int64_t)C * E;
    a.n0 = C;
    a.P = (int32_t)E;
    return nt_run(a, C2, C, 1, dw2, db2, workspace, workspace_bytes, st);  // row sums of dz^T = db2
  }
  return hipSuccess;
}

// ------------------------------------------------------------------------------------------------
// The edge encoder's whole backward in three launches on one stream (training path, encoder.py):
//   1. dz^T                                     (mrp_edge_encoder_bwd_prep)
//   2. dh^T = W2^T dz^T and dW2 = dz^T h        one launch of both split-K NT products, splits chosen
//                                               jointly so the two fill one round of the chip
//   3. encoder_bwd_reduce: dW2 and db2 = the fixed-order sums of their partial tiles / row sums; and,
//      per hidden unit (one workgroup over all edges), dh^T summed from its partial tiles, masked by
//      [h^T > 0] (ReLU) and reduced against the pose rows into dW1 / db1 — dh^T never written.
//      (Round 4 first reduced per (4 units, 256 edges) into partials summed by a fourth launch: the
//      whole backward 46.2 -> 42.8 us at E = 1792, C = 512, tools/exp_enc_bwd.py.)
// ------------------------------------------------------------------------------------------------
namespace mrp_cs {

constexpr int kNin = 9;

// dz (E x N2, row-major) -> the packed split image of dz^T (N2 x E, k = the edges; `pack`'s layout, the
// dW2 product's A operand, read by LDS-DMA) and db2's partials csum[eb][j] = sum of dz[e][j] over the
// 64-edge block eb in edge order (summed over the blocks in order by encoder_bwd_reduce).  64 x 64 tile
// through LDS as dz_transpose; lane -> (row j0 + (u & 63), edges 8 (u >> 6) ..): a wave's 32-row halves
// store 512 contiguous bytes per part.  E % 16 == 0.
__global__ void __launch_bounds__(256) dzT_pack(const float* __restrict__ dz, int E, int N2, u4* __restrict__ img,
                                                float* __restrict__ csum) {
  __shared__ float tile[64][65];
  const int j0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  const int c4 = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  f4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = e0 + r0 + 16 * i, j = j0 + 4 * c4;
    v[i] = (e < E && j < N2) ? *reinterpret_cast<const f4*>(dz + (int64_t)e * N2 + j) : f4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[r0 + 16 * i][4 * c4 + q] = v[i][q];
  __syncthreads();
  if (threadIdx.x < 64 && j0 + (int)threadIdx.x < N2) {
    float sum = 0.f;
    for (int e = 0; e < 64; ++e) sum += tile[e][threadIdx.x];
    csum[(int64_t)blockIdx.y * N2 + j0 + threadIdx.x] = sum;
  }
  const int64_t KS = E / 16;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int u = threadIdx.x + 256 * i;
    const int jl = u & 63, g8 = u >> 6;
    const int j = j0 + jl, e = e0 + 8 * g8;
    if (j >= N2 || e >= E) continue;
    u4 p0, p1, p2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f2 x;
      x.x = tile[8 * g8 + 2 * q][jl];
      x.y = tile[8 * g8 + 2 * q + 1][jl];
      uint32_t a0, a1, a2;
      split2(x, a0, a1, a2);
      p0[q] = a0, p1[q] = a1, p2[q] = a2;
    }
    const int64_t base = (((int64_t)(j >> 5) * KS + (e >> 4)) * 3) * 64 + (j & 31) + 32 * ((e >> 3) & 1);
    img[base] = p0;
    img[base + 64] = p1;
    img[base + 128] = p2;
  }
}

// both products with a pre-split A: W2^T's packed image and dz^T's (dzT_pack)
__global__ void __launch_bounds__(512, 1) gemm_nt_dual_psa2(NTArgs a1, NTArgs a2, int grid1) {
  if ((int)blockIdx.x < grid1)
    gemm_nt_psa_body(a1, blockIdx.x, grid1);
  else
    gemm_nt_psa_body(a2, blockIdx.x - grid1, gridDim.x - grid1);
}

struct EncPlan {
  int s1, s2;
  int64_t kc1, kc2;
  int t1, t2;  // tiles of each product
  int64_t off_dzT, off_p1, off_p2, off_p2b, bytes;
};

EncPlan enc_plan(int64_t E, int64_t C) {
  EncPlan pl{};
  const int64_t C2 = 2 * C;
  pl.t1 = (int)(((C + NTGeo<4>::TM - 1) / NTGeo<4>::TM) * ((E + TN - 1) / TN));       // dh^T: M = C, N = E
  pl.t2 = (int)(((C2 + NTGeo<4>::TM - 1) / NTGeo<4>::TM) * ((C + TN - 1) / TN));      // dW2: M = 2C, N = C
  const int64_t st1 = C2 / BK, st2 = E / BK;                                // 32-k split granules
  // Split counts: the makespan of the launch's workgroups dispatched in order (the a t1 units of the
  // first product, p1 stages each, then the b t2 of the second) onto 256 CUs one at a time (~2.8 us per
  // 32-k stage), plus the partial tiles written and read back at ~4 TB/s.  Round 4's estimate (rounds x
  // the longer split) missed that the second product's units start as soon as the first's free their CU:
  // round 5 (tools/ab_enc_splits.py) configs[2] (3, 3) 136.9 vs its (2, 1) 141.7 us, configs[1] (8, 7)
  // 30.0 vs (5, 4) 33.8, configs[3] (4, 1) 101.4 vs (8, 1) 106.2; the headline and configs[4] unchanged.
  // Memoised per shape (at most kMemo shapes; a full memo starts over).  A pair whose lower bound — its
  // first product's rounds, or all its work spread evenly over the CUs, plus its traffic — is no better
  // than the best found is not simulated: the full search is up to 32 x 32 pairs of b t2 heap steps
  // each (~5e5 at C = 2048), the pruned one a few percent of that.
  constexpr size_t kMemo = 64;
  static std::mutex mu;
  static std::map<std::pair<int64_t, int64_t>, std::pair<int, int>> memo;
  {
    std::lock_guard<std::mutex> lock(mu);
    auto it = memo.find({E, C});
    if (it != memo.end()) {
      pl.s1 = it->second.first;
      pl.s2 = it->second.second;
    } else {
      double best = 1e300;
      pl.s1 = pl.s2 = 1;
      std::vector<int64_t> slot(256);
      for (int a = 1; a <= 32; ++a)
        for (int b = 1; b <= 32; ++b) {
          const int64_t p1 = (st1 + a - 1) / a, p2 = (st2 + b - 1) / b;
          if ((st1 + p1 - 1) / p1 != a || (st2 + p2 - 1) / p2 != b) continue;  // no empty split
          const int64_t n1 = (int64_t)a * pl.t1, n2 = (int64_t)b * pl.t2;
          const int64_t q = n1 / 256, r = n1 % 256;
          const double traffic = ((double)a * C * E + (double)b * C2 * C) * 8.0 / 4.0e6;
          const int64_t lb = std::max<int64_t>((q + (r ? 1 : 0)) * p1, (n1 * p1 + n2 * p2 + 255) / 256);
          if ((double)lb * 2.8 + traffic >= best) continue;  // cannot beat the best: skip the simulation
          for (int i = 0; i < 256; ++i) slot[i] = (q + (i < r ? 1 : 0)) * p1;  // the first product round robin
          std::make_heap(slot.begin(), slot.end(), std::greater<int64_t>());
          int64_t span = (q + (r ? 1 : 0)) * p1;
          for (int64_t i = 0; i < n2; ++i) {  // the second product onto the earliest free CU
            std::pop_heap(slot.begin(), slot.end(), std::greater<int64_t>());
            slot.back() += p2;
            span = slot.back() > span ? slot.back() : span;
            std::push_heap(slot.begin(), slot.end(), std::greater<int64_t>());
          }
          const double cost = (double)span * 2.8 + traffic;
          if (cost < best) {
            best = cost;
            pl.s1 = a;
            pl.s2 = b;
          }
        }
      if (memo.size() >= kMemo) memo.clear();
      memo[{E, C}] = {pl.s1, pl.s2};
    }
  }
  // lab knobs enc_s1 / enc_s2 (0: the planner's): force a split count (the chunks cover K, none empty)
  if (mrp_host::tuning().enc_s1 > 0) pl.s1 = (int)(mrp_host::tuning().enc_s1 < st1 ? mrp_host::tuning().enc_s1 : st1);
  if (mrp_host::tuning().enc_s2 > 0) pl.s2 = (int)(mrp_host::tuning().enc_s2 < st2 ? mrp_host::tuning().enc_s2 : st2);
  pl.kc1 = ((st1 + pl.s1 - 1) / pl.s1) * BK;
  pl.kc2 = ((st2 + pl.s2 - 1) / pl.s2) * BK;
  pl.s1 = (int)((st1 * BK + pl.kc1 - 1) / pl.kc1);  // the splits the chunks give (no empty one)
  pl.s2 = (int)((st2 * BK + pl.kc2 - 1) / pl.kc2);
  auto al = [](int64_t v) { return (v + 63) / 64 * 64; };  // 256-byte segments
  int64_t o = 0;
  pl.off_dzT = o;
  o += al(C2 * E * 3 / 2);  // dz^T in fp32, or its packed split image (6 bytes per element)
  pl.off_p1 = o;
  o += al((int64_t)pl.s1 * C * E);
  pl.off_p2 = o;
  o += al((int64_t)pl.s2 * C2 * C);
  pl.off_p2b = o;
  const int64_t nb2 = (int64_t)pl.s2 > (E + 63) / 64 ? pl.s2 : (E + 63) / 64;  // db2 partials: splits or edge blocks
  o += al(nb2 * C2);
  pl.bytes = o * 4;
  return pl;
}

// blocks [0, nb1): one hidden unit each -> dW1 / db1; blocks [nb1, ...): 1024
// outputs of dW2 each (and, in the first 2C / 256 of them, 256 of db2)
__global__ void __launch_bounds__(256) encoder_bwd_reduce(const float* __restrict__ p1, int s1,
                                                          const float* __restrict__ hT, const float* __restrict__ pose,
                                                          int E, int C, float* __restrict__ dw1,
                                                          float* __restrict__ db1, int nb1,
                                                          const f4* __restrict__ p2, const float* __restrict__ p2b,
                                                          int s2, int s2b, f4* __restrict__ dw2, float* __restrict__ db2) {
  if ((int)blockIdx.x < nb1) {
    // one workgroup per hidden unit u: wave w's lanes walk edges 64 w + lane + 256 k, summing the dh^T
    // partials in split order, masking by the ReLU and accumulating d pose^T and d in registers; a
    // fixed lane butterfly per wave, the four waves' sums added in wave order, and dW1[u] / db1[u]
    // written directly (no per-edge-block partials, no final launch)
    __shared__ float wsum[4][kNin + 1];
    const int u = blockIdx.x, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t plane = (int64_t)C * E;
    const float* p1u = p1 + (int64_t)u * E;
    const float* hTu = hT + (int64_t)u * E;
    float acc[kNin + 1];
#pragma unroll
    for (int i = 0; i <= kNin; ++i) acc[i] = 0.f;
#pragma unroll 2
    for (int e = threadIdx.x; e < E; e += 256) {
      float dh;
      if (s1 <= 8) {  // every partial's load issued before the sums (clamped index, no branch per load)
        float pv[8];
#pragma unroll
        for (int sp = 0; sp < 8; ++sp) pv[sp] = p1u[(int64_t)(sp < s1 ? sp : s1 - 1) * plane + e];
        dh = pv[0];
#pragma unroll
        for (int sp = 1; sp < 8; ++sp) dh = sp < s1 ? dh + pv[sp] : dh;
      } else {
        dh = p1u[e];
        for (int sp = 1; sp < s1; ++sp) dh += p1u[(int64_t)sp * plane + e];
      }
      const float d = hTu[e] > 0.f ? dh : 0.f;
      const float* pr = pose + (int64_t)e * kNin;
#pragma unroll
      for (int i = 0; i < kNin; ++i) acc[i] = fmaf(d, pr[i], acc[i]);
      acc[kNin] += d;
    }
#pragma unroll
    for (int i = 0; i <= kNin; ++i)
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) acc[i] += __shfl_xor(acc[i], o, 64);
    if (lane <= kNin) {
      float v = acc[0];
#pragma unroll
      for (int i = 1; i <= kNin; ++i) v = lane == i ? acc[i] : v;
      wsum[w][lane] = v;
    }
    __syncthreads();
    if (threadIdx.x <= kNin) {
      const float v = ((wsum[0][threadIdx.x] + wsum[1][threadIdx.x]) + wsum[2][threadIdx.x]) + wsum[3][threadIdx.x];
      if (threadIdx.x < kNin)
        dw1[(int64_t)u * kNin + threadIdx.x] = v;
      else
        db1[u] = v;
    }
    return;
  }
  const int b = blockIdx.x - nb1;
  const int64_t n4 = (int64_t)2 * C * C / 4;
  const int64_t e4 = (int64_t)b * 256 + threadIdx.x;
  if (e4 < n4) {
    f4 v;
    if (s2 <= 8) {
      f4 pv[8];
#pragma unroll
      for (int sp = 0; sp < 8; ++sp) pv[sp] = p2[(int64_t)(sp < s2 ? sp : s2 - 1) * n4 + e4];
      v = pv[0];
#pragma unroll
      for (int sp = 1; sp < 8; ++sp) v = sp < s2 ? v + pv[sp] : v;
    } else {
      v = p2[e4];
      for (int sp = 1; sp < s2; ++sp) v += p2[(int64_t)sp * n4 + e4];
    }
    dw2[e4] = v;
  }
  const int64_t m = (int64_t)b * 256 + threadIdx.x;
  if (m < 2 * C) {
    float v = p2b[m];
    for (int sp = 1; sp < s2b; ++sp) v += p2b[(int64_t)sp * 2 * C + m];
    db2[m] = v;
  }
}

}  // namespace mrp_cs

extern "C" int64_t mrp_edge_encoder_bwd_fused_workspace(int32_t num_edges, int32_t C) {
  if (num_edges <= 0 || C <= 0 || num_edges % BK != 0 || C % 32 != 0) return 0;
  return mrp_cs::enc_plan(num_edges, C).bytes;
}

extern "C" int mrp_edge_encoder_bwd_fused(const float* dz, const float* w2T, const void* w2T_packed, const float* hT,
                                          const float* pose, int32_t num_edges, int32_t C, float* dw1, float* db1,
                                          float* dw2, float* db2, void* workspace, int64_t workspace_bytes,
                                          void* stream) {
  using namespace mrp_cs;
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (C == 0) return hipSuccess;
  if (!dw1 || !db1 || !dw2 || !db2) return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int64_t E = num_edges, C2 = 2 * (int64_t)C;
  if (E == 0) {  // empty sums
    if (hipMemsetAsync(dw1, 0, (size_t)C * kNin * 4, st) != hipSuccess ||
        hipMemsetAsync(db1, 0, (size_t)C * 4, st) != hipSuccess ||
        hipMemsetAsync(dw2, 0, (size_t)C2 * C * 4, st) != hipSuccess || hipMemsetAsync(db2, 0, (size_t)C2 * 4, st) != hipSuccess)
      return hipErrorUnknown;
    return hipSuccess;
  }
  if (E % BK != 0 || C % 32 != 0) return hipErrorNotSupported;
  if (!dz || !w2T || !hT || !pose || !aligned16(dz) || !aligned16(w2T) || !aligned16(hT) || !aligned16(dw2))
    return hipErrorInvalidValue;
  const EncPlan pl = enc_plan(E, C);
  if (workspace == nullptr || !aligned16(workspace) || workspace_bytes < pl.bytes) return hipErrorInvalidValue;
  float* ws = static_cast<float*>(workspace);
  float* dzT = ws + pl.off_dzT;
  // W2^T's packed image (mrp_compress_split_pack(w2, C, 1, C, 2C)): the dh^T product reads its A by
  // LDS-DMA instead of splitting W2^T in every workgroup; and (enc_bwd_psa 2, the default) dz^T is
  // written as a packed image too (dzT_pack, with db2's partials), so the dW2 product reads both its
  // operands' A side pre-split.  enc_bwd_psa 0: both split in the kernel, 1: only W2^T pre-split.
  const int mode = mrp_host::tuning().enc_bwd_psa;
  const bool psa1 = w2T_packed != nullptr && aligned16(w2T_packed) && mode >= 1 && (int64_t)C * C2 * 6 < kOffMax;
  const bool psa2 = psa1 && mode >= 2 && C2 * E * 6 < kOffMax;
  hipError_t e;
  if (psa2) {
    hipLaunchKernelGGL(dzT_pack, dim3((unsigned)((C2 + 63) / 64), (unsigned)((E + 63) / 64)), dim3(256), 0, st, dz,
                       num_edges, (int)C2, reinterpret_cast<u4*>(dzT), ws + pl.off_p2b);
    e = hipGetLastError();
  } else {
    e = (hipError_t)mrp_edge_encoder_bwd_prep(dz, num_edges, C, dzT, E, stream);
  }
  if (e != hipSuccess) return e;
  NTArgs a1 = {};  // dh^T (C x E) = W2^T (C x 2C) . dz^T: rows u, k = j
  a1.g = w2T;
  a1.gs = C * C2;
  a1.s0 = dz;
  a1.s0s = E * C2;
  a1.s1 = dz;
  a1.s1s = E * C2;
  a1.n0 = (int32_t)E;
  a1.P = (int32_t)C2;
  a1.out = ws + pl.off_p1;
  a1.outb = nullptr;
  a1.ktot = C2;
  a1.kchunk = pl.kc1;
  a1.M = C;
  a1.N = (int32_t)E;
  a1.mtiles = (int32_t)((C + NTGeo<4>::TM - 1) / NTGeo<4>::TM);
  a1.ntiles = (int32_t)((E + TN - 1) / TN);
  a1.ap = psa1 ? static_cast<const u4*>(w2T_packed) : nullptr;
  NTArgs a2 = {};  // dW2 (2C x C) = dz^T (2C x E) . h: rows j, k = e; row sums = db2
  a2.g = dzT;
  a2.gs = C2 * E;
  a2.s0 = hT;
  a2.s0s = (int64_t)C * E;
  a2.s1 = hT;
  a2.s1s = (int64_t)C * E;
  a2.n0 = C;
  a2.P = (int32_t)E;
  a2.out = ws + pl.off_p2;
  a2.outb = psa2 ? nullptr : ws + pl.off_p2b;  // psa2: db2's partials came from dzT_pack
  a2.ap = psa2 ? reinterpret_cast<const u4*>(dzT) : nullptr;
  a2.ktot = E;
  a2.kchunk = pl.kc2;
  a2.M = (int32_t)C2;
  a2.N = C;
  a2.mtiles = (int32_t)((C2 + NTGeo<4>::TM - 1) / NTGeo<4>::TM);
  a2.ntiles = (int32_t)((C + TN - 1) / TN);
  const int grid1 = pl.t1 * pl.s1, grid2 = pl.t2 * pl.s2;
  using GN = NTGeo<4>;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_dual_mf16),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, GN::LDS_BYTES);
  if (attr != hipSuccess) return attr;
  static const hipError_t attr_p = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_dual_psa1),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, GN::LDS_BYTES);
  if (attr_p != hipSuccess) return attr_p;
  static const hipError_t attr_p2 = hipFuncSetAttribute(reinterpret_cast<const void*>(&gemm_nt_dual_psa2),
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, GN::LDS_BYTES);
  if (attr_p2 != hipSuccess) return attr_p2;
  a1.group = a2.group = mrp_host::tuning().nt_group;
  if (psa2)
    hipLaunchKernelGGL(gemm_nt_dual_psa2, dim3((unsigned)(grid1 + grid2)), dim3(GN::THREADS), GN::LDS_BYTES, st, a1,
                       a2, grid1);
  else if (psa1)
    hipLaunchKernelGGL(gemm_nt_dual_psa1, dim3((unsigned)(grid1 + grid2)), dim3(GN::THREADS), GN::LDS_BYTES, st, a1,
                       a2, grid1);
  else
    hipLaunchKernelGGL(gemm_nt_dual_mf16, dim3((unsigned)(grid1 + grid2)), dim3(GN::THREADS), GN::LDS_BYTES, st, a1,
                       a2, grid1);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int nb1 = C;
  const int64_t nb2 = (C2 * C / 4 + 255) / 256;  // >= 2C / 256 blocks: db2 rides along
  hipLaunchKernelGGL(encoder_bwd_reduce, dim3((unsigned)(nb1 + nb2)), dim3(256), 0, st, ws + pl.off_p1, pl.s1, hT, pose,
                     num_edges, C, dw1, db1, nb1, reinterpret_cast<const f4*>(ws + pl.off_p2), ws + pl.off_p2b,
                     pl.s2, psa2 ? (int)((E + 63) / 64) : pl.s2, reinterpret_cast<f4*>(dw2), db2);
  return hipGetLastError();
}
