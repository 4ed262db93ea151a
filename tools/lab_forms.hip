// lab_forms.hip — kernel lab (not product code): round 4's compress GEMM forms that the product
// library no longer builds (round 5 moved them here).  Each lost to the product's
// default at every BASELINE config shape:
//   * gemm_nn_split_w4      256-row NN on 32x32x16 MFMAs, 32-k stages      (7-12 % slower than gemm_nn_split_w4_mf16)
//   * gemm_nn_split3_w4/_w2 the pipelined 16-k-stage NN forms, both operands by LDS-DMA (same)
//   * gemm_nt_split_w4      the 32-k-stage weight gradient on 32x32x16 MFMAs (4-5 % slower than _mf16)
//   * gemm_nt_split3_w4     the pipelined 16-k-stage weight gradient        (same)
// The product's helpers, argument structs and defaults come from compress_split.hip, included here;
// tools/gemm_ablate.hip builds its ablations on gemm_nn_split3_body.
// build (a lab binary, e.g.): hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/lab_forms.hip
#include "../multi-robot-perception-gnn-1_amd/csrc/compress_split.hip"

namespace mrp_cs {

// ------------------------------------------------------------------------------------------------
// Pipelined NN form (256 x 128 tiles, 8 waves of 64 x 64): stages of ONE 16-k step in a ring of
// NBUF = L + 2 LDS buffers; stage t's operands are requested L stages before they are needed.
// Per stage s a wave
//   - waits for its own requests of stage s + 2 (issued at stage s - L: counted vmcnt, the younger
//     requests stay in flight), splits its B piece of stage s + 2 into buffer (s + 2) % NBUF, then
//     requests stage s + 2 + L: its A pieces by LDS-DMA into buffer (s + 2 + L) % NBUF and its B
//     piece into the registers the split just freed (L register sets);
//   - runs stage s's 24 MFMAs (fragments already in registers) and, as each fragment's last MFMA
//     issues, reads the same fragment of stage s + 1 into its registers (no second fragment set);
//   - waits for its LDS writes, barrier: stage s + 2 is complete for every wave.
// Buffer (s + 2 + L) % NBUF = s % NBUF held stage s, whose fragments were read during stage s - 1
// (before the barrier that ended it); buffer (s + 2) % NBUF held stage s + 2 - NBUF = s - L, read
// during stage s - L - 1.  One barrier per 24 MFMAs; after it the MFMAs start at once.
// The B pieces travel by LDS-DMA too (global_load_lds, one 16-byte piece per lane into a raw fp32
// slot; each thread reads back exactly the piece its own lane requested, so its own counted vmcnt
// orders the read): hipcc waits vmcnt(0) before the first use of an ordinary load's result whenever
// an LDS-DMA is in flight (cdna_hip_programming.md, "Pipelining across barriers"), which would drain
// the pipeline every stage.  Every wait is explicit and counted (per stage, in issue order: the 3 A
// pieces, then the B piece).
// ------------------------------------------------------------------------------------------------
template <int WMW, int L>
struct Geo3 {
  static constexpr int TM = 64 * WMW, NW = 2 * WMW, THREADS = 64 * NW;
  static constexpr int BKS = 16;                     // k per stage
  static constexpr int A_PIECES = (TM / 32) * 3;     // 1 KiB pieces per stage
  static constexpr int A_BYTES = A_PIECES * 1024;
  static constexpr int B_PART = BKS * TN * 2;        // one bf16 part of the B stage: 4 KiB
  static constexpr int BUF_BYTES = A_BYTES + 3 * B_PART;
  static constexpr int NBUF = L + 2;
  static constexpr int B_RAW = BKS * TN * 4;         // the fp32 B stage as loaded: 8 KiB
  static constexpr int RAW_OFF = NBUF * BUF_BYTES;   // L raw B slots after the ring
  static constexpr int LDS_BYTES = RAW_OFF + L * B_RAW;  // 160 KiB at WMW 4, L 2
  static constexpr int PPW = A_PIECES / NW;          // DMA pieces per wave per stage
  static constexpr int BJ = BKS * TN / 4 / THREADS;  // 16-byte B pieces per thread per stage
  static constexpr int KR = THREADS / 32;            // B rows per pass
  static constexpr int OPS = PPW + BJ;               // vector-memory requests per wave per stage
  static_assert(BJ * THREADS * 4 == BKS * TN, "whole B pieces per thread");
  static_assert(A_PIECES % NW == 0, "whole DMA pieces per wave");
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int WMW, int L, int ABL = 0>  // ABL: lab ablation bits (tools/gemm_ablate.hip; 0 in the library)
__device__ __forceinline__ void gemm_nn_split3_body(const Args& a) {
  using G = Geo3<WMW, L>;
  constexpr int TM = G::TM, NW = G::NW, A_BYTES = G::A_BYTES, BUF_BYTES = G::BUF_BYTES, B_PART = G::B_PART;
  constexpr int NBUF = G::NBUF, OPS = G::OPS;
  static_assert(L == 1 || L == 2, "one or two stages of request lead");
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int mt = id % a.mtiles, nt = id / a.mtiles;
  const int64_t nbase = (int64_t)nt * TN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int nst = a.K / 16, ks0 = a.k0 / 16, MB = a.M / 32;

  // ---- A: LDS-DMA pieces pc = mbl 3 + p (local m block, part), pc = w + NW i
  const __amdgpu_buffer_rsrc_t ra = rsrc(a.ap);
  uint32_t va[G::PPW];
#pragma unroll
  for (int i = 0; i < G::PPW; ++i) {
    const int pc = w + NW * i;
    const int mbl = pc / 3, p = pc % 3;
    const int mb = min(mt * (TM / 32) + mbl, MB - 1);  // blocks past M: any valid data, never stored
    va[i] = (uint32_t)((((int64_t)mb * nst * 3 + p) * 64 + lane) * 16);
  }
  auto issue_a = [&](int s, int buf) {
#pragma unroll
    for (int i = 0; i < G::PPW; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, lds + (buf * BUF_BYTES + (w + NW * i) * 1024) / 16, 16, va[i],
                                               (uint32_t)s * 3 * 1024, 0, 0);
  };

  // ---- B: thread t loads the 16-byte pieces (rows (t >> 5) + KR j, columns 4 (t & 31) ..) of a stage
  constexpr int BJ = G::BJ, KR = G::KR;
  const int fc = threadIdx.x & 31, kr = threadIdx.x >> 5;
  int64_t col = nbase + 4 * fc;
  if (col > a.ncols - 4) col = a.ncols - 4;  // columns past the end: any valid data, never stored
  const int64_t node = col / a.P, pix = col - node * a.P;
  // buffer resources based at the tile's first node and the stage's first channel (scalar, rebuilt
  // per stage), so a lane's offset spans at most the tile's few nodes (global_load_lds would be a
  // FLAT-encoded load, after which hipcc waits lgkmcnt(0) before the next MFMA)
  const int64_t node0 = nbase / a.P;
  uint32_t vb0[BJ], vb1[BJ];
#pragma unroll
  for (int j = 0; j < BJ; ++j) {
    vb0[j] = (uint32_t)(((node - node0) * a.b0s + pix + (int64_t)(kr + KR * j) * a.P) * 4);
    vb1[j] = (uint32_t)(((node - node0) * a.b1s + pix + (int64_t)(kr + KR * j) * a.P) * 4);
  }
  const float* const bb0 = a.b0 + node0 * a.b0s;
  const float* const bb1 = a.b1 + node0 * a.b1s;
  char* const raw = ldsb + G::RAW_OFF;
  // piece j of thread t lands at raw + slot B_RAW + 16 (j THREADS + t)
  auto load_b = [&](int s, int slot) {
    const bool lo = s < ks0;
    const __amdgpu_buffer_rsrc_t rb = rsrc(lo ? bb0 + (int64_t)s * 16 * a.P : bb1 + (int64_t)(s - ks0) * 16 * a.P);
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, lds + (G::RAW_OFF + slot * G::B_RAW + j * G::THREADS * 16 + w * 1024) / 16, 16, lo ? vb0[j] : vb1[j], 0,
          0, 0);
  };
  // the raw read by inline asm too (a compiler-visible read there makes hipcc wait for it before the
  // first MFMA of the stage); its result is guarded by an asm lgkmcnt wait naming the registers,
  // which must precede every use
  const uint32_t raw_addr = (uint32_t)reinterpret_cast<uintptr_t>(raw + 16 * threadIdx.x);
  struct Raw {
    f4 v[BJ];
  };
  auto raw_b = [&](int slot) {
    Raw r;
#pragma unroll
    for (int j = 0; j < BJ; ++j)
      asm volatile("ds_read_b128 %0, %1 offset:%2"
                   : "=v"(r.v[j])
                   : "v"(raw_addr + (uint32_t)(slot * G::B_RAW)), "i"(j * G::THREADS * 16)
                   : "memory");
    return r;
  };
  auto raw_wait = [&](Raw& r) {
#pragma unroll
    for (int j = 0; j < BJ; ++j) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r.v[j])::"memory");
  };
  auto store_b = [&](const Raw& r, int buf) {
#pragma unroll
    for (int j = 0; j < BJ; ++j) {
      char* bimg = ldsb + buf * BUF_BYTES + A_BYTES + boff(kr + KR * j, fc >> 1) + 8 * (fc & 1);
      u2 p0, p1, p2;
      f2 lo, hi;
      lo.x = r.v[j].x, lo.y = r.v[j].y, hi.x = r.v[j].z, hi.y = r.v[j].w;
      uint32_t l0, l1, l2, h0, h1, h2;
      split2(lo, l0, l1, l2);
      split2(hi, h0, h1, h2);
      p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
      *reinterpret_cast<u2*>(bimg) = p0;
      *reinterpret_cast<u2*>(bimg + B_PART) = p1;
      *reinterpret_cast<u2*>(bimg + 2 * B_PART) = p2;
    }
  };

  // ---- fragment reads: A by row pieces (ds_read_b128), B by ds_read_b64_tr_b16
  const int g16 = lane >> 4, i16 = lane & 15, hh = lane >> 5;
  const int trq = i16 >> 2, trp = i16 & 3;
  bf8 af[2][3], bfr[2][3];
  auto read_a = [&](int buf, int mi) {
    const char* base = ldsb + buf * BUF_BYTES + lane * 16;
#pragma unroll
    for (int p = 0; p < 3; ++p)
      af[mi][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + ((2 * wm + mi) * 3 + p) * 1024));
  };
  // B fragments by inline-asm ds_read_b64_tr_b16: the builtin carries no memory operand, so hipcc
  // would wait for every LDS-DMA in flight (vmcnt(0)) before it, though the DMA fills another buffer;
  // the waits these reads need are placed by hand below (LDS operations retire in order)
  uint32_t tra[2][2];  // byte address of read (ni, t) in buffer 0, part 0
#pragma unroll
  for (int ni = 0; ni < 2; ++ni)
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int row = 8 * hh + 4 * t + trq;
      const int ch = (64 * wn + 32 * ni + 16 * (g16 & 1)) / 8 + (trp >> 1);
      tra[ni][t] = (uint32_t)reinterpret_cast<uintptr_t>(ldsb + A_BYTES + boff(row, ch) + 8 * (trp & 1));
    }
  auto read_b = [&](int buf, int ni) {
    const uint32_t o = (uint32_t)(buf * BUF_BYTES);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      s4 v[2];
#pragma unroll
      for (int t = 0; t < 2; ++t)
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v[t]) : "v"(tra[ni][t] + o), "i"(p * B_PART));
      u4 u;
      u.x = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[0], v[0], 0, 1));
      u.y = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[0], v[0], 2, 3));
      u.z = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[1], v[1], 0, 1));
      u.w = __builtin_bit_cast(uint32_t, __builtin_shufflevector(v[1], v[1], 2, 3));
      bfr[ni][p] = __builtin_bit_cast(bf8, u);
    }
  };

  Acc2 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;

  // ---- prologue: stages 0 and 1 complete in buffers 0 and 1; stages 2 .. 1 + L requested (stage
  // t's raw B piece in slot t % L)
  issue_a(0, 0);
  load_b(0, 0);
  vm_wait<0>();
  Raw v0 = raw_b(0);
  raw_wait(v0);
  store_b(v0, 0);
  issue_a(1, 1);  // nst >= 2 (K % 32 == 0)
  load_b(1, L - 1);
  vm_wait<0>();
  Raw v1 = raw_b(L - 1);
  raw_wait(v1);
  store_b(v1, 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the raw reads retired before the slots refill
#pragma unroll
  for (int t = 2; t < 2 + L; ++t)
    if (t < nst) {
      issue_a(t, t);
      load_b(t, t % L);
    }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  read_a(0, 0);
  read_a(0, 1);
  read_b(0, 0);
  read_b(0, 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);

  // Fragment reads of stage s + 1 (LDS operations in issue order): group 2 = A block 0 (3 reads),
  // group 3 = B block 0 (6), group 4 = A block 1 + B block 1 (9).  The barrier that ends stage s waits
  // for all but group 4; the MFMAs of block (0, 1) of stage s + 1 wait for group 4 too.
  auto stage = [&](int s, int slot) {  // slot = (s + 2) % L: stage s + 2's raw B piece, then s + 2 + L's
    const int cur = s % NBUF;
    const int nxt = cur + 1 == NBUF ? 0 : cur + 1;   // stage s + 1 (past the last stage: never used)
    const int fil = nxt + 1 == NBUF ? 0 : nxt + 1;   // stage s + 2
    // stage s + 2's requests (issued L stages ago) landed; each later stage issued OPS requests.
    // Past the last stage the raw read and the split are harmless: the split goes to a buffer no
    // wave reads again (stage s + 2 - NBUF's, read during stage s + 1 - NBUF)
    if (L == 2 && s + 3 < nst)
      vm_wait<OPS>();
    else
      vm_wait<0>();
    Raw v = raw_b(slot);  // its latency runs under the first six MFMAs
    __builtin_amdgcn_sched_barrier(0);
    mma6(af[0], bfr[0], acc[0][0]);
    __builtin_amdgcn_sched_barrier(0);
    raw_wait(v);  // the raw read (and all older LDS reads)
    if (!(ABL & 8)) store_b(v, fil);
    if (s + 2 + L < nst) {
      if (!(ABL & 1)) issue_a(s + 2 + L, cur);  // buffer s % NBUF: stage s's fragments are in registers
      if (!(ABL & 2)) load_b(s + 2 + L, slot);  // after the split consumed the slot's piece
    }
    __builtin_amdgcn_sched_barrier(0);
    // group 4 of the previous stage retired (stage s's B block 1; the raw read above retired with
    // it); the LDS writes may not have (2 or 3 instructions per piece: hipcc may pair two of them)
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(2 * BJ) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    mma6(af[0], bfr[1], acc[0][1]);
    __builtin_amdgcn_sched_barrier(0);
    read_a(nxt, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma6(af[1], bfr[0], acc[1][0]);
    __builtin_amdgcn_sched_barrier(0);
    read_b(nxt, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma6(af[1], bfr[1], acc[1][1]);
    __builtin_amdgcn_sched_barrier(0);
    read_a(nxt, 1);
    read_b(nxt, 1);
    __builtin_amdgcn_sched_barrier(0);
    // every LDS operation but group 4 retired: stage s + 2 is complete for all waves after the
    // barrier, and no wave writes a buffer another may still read
    asm volatile("s_waitcnt lgkmcnt(9)" ::: "memory");
    if (!(ABL & 4)) __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll 1
  for (int s = 0; s < nst; ++s) stage(s, L == 2 ? s & 1 : 0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the (unused) reads past the last stage

  // ---- epilogue (as gemm_nn_split_body)
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

__global__ void __launch_bounds__(512, 1) gemm_nn_split3_w4(Args a) { gemm_nn_split3_body<4, 2>(a); }
// 128-row workgroups of 4 waves, two per CU (80 KiB of LDS each): the two workgroups' barriers and
// request bursts are independent, so one's run under the other's MFMAs
__global__ void __launch_bounds__(256, 2) gemm_nn_split3_w2(Args a) { gemm_nn_split3_body<2, 1>(a); }


__global__ void __launch_bounds__(512, 1) gemm_nn_split_w4(Args a) { gemm_nn_split_body<4>(a); }

template <int WMW, bool MF16 = false>
__device__ __forceinline__ void gemm_nt_split_body_r4(const NTArgs& a, int orig, int nwg) {
  using G = NTGeo<WMW>;
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tiles = a.mtiles * a.ntiles;
  const int split = id / tiles, tid = id - split * tiles;
  const int mt = tid % a.mtiles, nt = tid / a.mtiles;
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
  // fragments of one 16-k step: lane (r, hh) reads k = 16 ksl + 8 hh .. + 7 of row r: chunk 2 ksl + hh
  const int hh = lane >> 5, rl = lane & 31;
  auto read_step = [&](int buf, int ksl, bf8 (&af)[2][3], bf8 (&bf)[2][3]) {
    const char* base = ldsb + buf * G::BUF_BYTES;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const int row = 64 * wm + 32 * mi + rl;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        af[mi][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + p * G::A_PART + rowoff(row, 2 * ksl + hh)));
    }
    const char* bb = base + 3 * G::A_PART;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      const int row = 64 * wn + 32 * ni + rl;
#pragma unroll
      for (int p = 0; p < 3; ++p)
        bf[ni][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(bb + p * G::B_PART + rowoff(row, 2 * ksl + hh)));
    }
  };

  if constexpr (MF16) {
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
  } else {
  Acc2 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;

  if (nst > 0) load();
#pragma unroll 1
  for (int s = 0; s < nst; ++s) {
    const int buf = s & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    store(buf);  // its buffer was last read in stage s - 2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nst) load();
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

  float* out = a.out + (int64_t)split * a.M * a.N;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int n = nbase + 64 * wn + 32 * ni + rl;
    if (n >= a.N) continue;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mbase + 64 * wm + 32 * mi + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < a.M) out[(int64_t)m * a.N + n] = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
      }
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


__global__ void __launch_bounds__(512, 1) gemm_nt_split_w4(NTArgs a) {
  gemm_nt_split_body_r4<4>(a, blockIdx.x, gridDim.x);
}

// Pipelined weight-gradient form (round 4; the default where its layout conditions hold).  The NN
// kernel's schedule (gemm_nn_split3_body) for two activation operands: 256 x 128 tiles of 8 waves of
// 64 x 64, stages of ONE 16-k step.  Every thread's three 16-byte pieces of a stage (two A rows, one B
// row, four k each) travel by LDS-DMA into a raw slot (two slots: stage t in slot t % 2, requested two
// stages ahead), are read back by the same lane (its own counted vmcnt orders the read), split and
// stored as three bf16 row images ([row][16 k], 32-byte rows, the two 16-byte chunks swapped every 8
// rows so a fragment read meets every bank once) into a ring of three buffers (stage t in t % 3).
// Per stage a wave waits for its own requests of stage s + 2, splits them into buffer (s + 2) % 3 —
// which held stage s - 1, whose fragments every wave read before the barrier that ended stage s - 1 —
// requests stage s + 4 into the slot it just read, and runs stage s's 24 MFMAs with the next stage's
// fragments read as each fragment's last MFMA issues; one raw barrier per stage, no vmcnt(0) in the
// loop.  LDS: 3 x 36 KiB + 2 x 24 KiB = 156 KiB.  The products and their order per output are
// gemm_nt_split_body's: at the same split the dW outputs are bit-identical (the row sums, summed per
// thread over other k groupings, are not).  Requires N % 16 == 0 and n0 % 16 == 0 (a wave's 16 B rows
// lie in one source tensor).
struct NT3 {
  static constexpr int TM = 256, THREADS = 512, BKS = 16;
  static constexpr int ROWB = BKS * 2;                       // bytes per [row][16 k] bf16 row
  static constexpr int A_PART = TM * ROWB, B_PART = TN * ROWB;  // 8 KiB, 4 KiB
  static constexpr int BUF_BYTES = 3 * (A_PART + B_PART);    // 36 KiB
  static constexpr int NBUF = 3;
  static constexpr int RAW_A = TM * BKS * 4;                 // 16 KiB of fp32 A pieces per stage
  static constexpr int RAW_BYTES = RAW_A + TN * BKS * 4;     // + 8 KiB of B
  static constexpr int RAW_OFF = NBUF * BUF_BYTES;
  static constexpr int LDS_BYTES = RAW_OFF + 2 * RAW_BYTES;  // 156 KiB
  static constexpr int OPS = 3;                              // LDS-DMA requests per thread per stage
  static_assert(LDS_BYTES <= 160 * 1024, "LDS");
};

__device__ __forceinline__ uint32_t nt3_off(int row, int chunk) {
  return (uint32_t)(32 * row + 16 * (chunk ^ ((row >> 3) & 1)));
}

template <int ABL = 0>  // ABL: lab ablation bits (0 in the library)
__device__ __forceinline__ void gemm_nt_split3_body(const NTArgs& a, int orig, int nwg) {
  using G = NT3;
  extern __shared__ u4 lds[];
  char* ldsb = reinterpret_cast<char*>(lds);
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int tiles = a.mtiles * a.ntiles;
  const int split = id / tiles, tid = id - split * tiles;
  const int mt = tid % a.mtiles, nt = tid / a.mtiles;
  const int mbase = mt * G::TM, nbase = nt * TN;
  const int64_t kbeg = (int64_t)split * a.kchunk;
  const int64_t kend = kbeg + a.kchunk < a.ktot ? kbeg + a.kchunk : a.ktot;
  const int nst = kend > kbeg ? (int)((kend - kbeg) / G::BKS) : 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int t = threadIdx.x, qd = t & 3, r0 = t >> 2;  // k quad, row

  // ---- requests: A rows r0 and r0 + 128 (rows past M clamped: any valid data, never stored), B row r0
  uint32_t va[2];
#pragma unroll
  for (int j = 0; j < 2; ++j)
    va[j] = (uint32_t)(((int64_t)min(mbase + r0 + 128 * j, a.M - 1) * a.P + 4 * qd) * 4);
  const int nrow = min(nbase + r0, a.N - 1);
  const bool bhi = __builtin_amdgcn_readfirstlane(nrow >= a.n0 ? 1 : 0) != 0;  // the wave's 16 rows: one side
  const uint32_t vb = (uint32_t)(((int64_t)(bhi ? nrow - a.n0 : nrow) * a.P + 4 * qd) * 4);
  // stages are requested in order, one at a time: the (node, pixel) of the next request is advanced
  // incrementally (no 64-bit division per stage)
  int64_t ind = kbeg / a.P;
  int ipx = (int)(kbeg - ind * a.P);
  auto issue = [&](int slot) {
    const __amdgpu_buffer_rsrc_t ra = rsrc(a.g + ind * a.gs + ipx);
    const __amdgpu_buffer_rsrc_t rb = rsrc(bhi ? a.s1 + ind * a.s1s + ipx : a.s0 + ind * a.s0s + ipx);
    const int base = G::RAW_OFF + slot * G::RAW_BYTES + w * 1024;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, lds + (base + j * 8192) / 16, 16, va[j], 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, lds + (base + G::RAW_A) / 16, 16, vb, 0, 0, 0);
    ipx += G::BKS;
    if (ipx == a.P) {
      ipx = 0;
      ++ind;
    }
  };
  // the raw read by inline asm (a compiler-visible read of a DMA'd location makes hipcc wait vmcnt(0)),
  // its result guarded by an asm lgkmcnt wait naming the registers
  const uint32_t raw_addr = (uint32_t)reinterpret_cast<uintptr_t>(ldsb + G::RAW_OFF + 16 * t);
  struct Raw {
    f4 v[3];
  };
  auto raw_read = [&](int slot) {
    Raw r;
    const uint32_t ad = raw_addr + (uint32_t)(slot * G::RAW_BYTES);
    asm volatile("ds_read_b128 %0, %1 offset:0" : "=v"(r.v[0]) : "v"(ad) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:8192" : "=v"(r.v[1]) : "v"(ad) : "memory");
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r.v[2]) : "v"(ad), "i"(G::RAW_A) : "memory");
    return r;
  };
  auto raw_wait = [&](Raw& r) {
#pragma unroll
    for (int j = 0; j < 3; ++j) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r.v[j])::"memory");
  };
  float rsum[2] = {0.f, 0.f};
  auto put = [&](char* img, int part_bytes, int row, const f4& v) {
    u2 p0, p1, p2;
    f2 lo, hi;
    lo.x = v.x, lo.y = v.y, hi.x = v.z, hi.y = v.w;
    uint32_t l0, l1, l2, h0, h1, h2;
    split2(lo, l0, l1, l2);
    split2(hi, h0, h1, h2);
    p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
    const uint32_t o = nt3_off(row, qd >> 1) + 8 * (qd & 1);
    *reinterpret_cast<u2*>(img + o) = p0;
    *reinterpret_cast<u2*>(img + part_bytes + o) = p1;
    *reinterpret_cast<u2*>(img + 2 * part_bytes + o) = p2;
  };
  auto store = [&](const Raw& r, int buf) {
    char* base = ldsb + buf * G::BUF_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      rsum[j] += (r.v[j].x + r.v[j].y) + (r.v[j].z + r.v[j].w);
      put(base, G::A_PART, r0 + 128 * j, r.v[j]);
    }
    put(base + 3 * G::A_PART, G::B_PART, r0, r.v[2]);
  };
  // ---- fragments: lane (rl, hh) reads k 8 hh .. 8 hh + 7 of its row: chunk hh
  const int hh = lane >> 5, rl = lane & 31;
  bf8 af[2][3], bfr[2][3];
  auto read_a = [&](int buf, int mi) {
    const char* base = ldsb + buf * G::BUF_BYTES + nt3_off(64 * wm + 32 * mi + rl, hh);
#pragma unroll
    for (int p = 0; p < 3; ++p) af[mi][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + p * G::A_PART));
  };
  auto read_b = [&](int buf, int ni) {
    const char* base = ldsb + buf * G::BUF_BYTES + 3 * G::A_PART + nt3_off(64 * wn + 32 * ni + rl, hh);
#pragma unroll
    for (int p = 0; p < 3; ++p) bfr[ni][p] = __builtin_bit_cast(bf8, *reinterpret_cast<const u4*>(base + p * G::B_PART));
  };

  Acc2 acc[2][2];
#pragma unroll
  for (int mi = 0; mi < 2; ++mi)
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[mi][ni].hi[r] = acc[mi][ni].lo[r] = 0.f;

  if (nst > 0) {
    // ---- prologue: stages 0 and 1 split into buffers 0 and 1, stages 2 and 3 requested
    issue(0);
    if (nst > 1) issue(1);
    vm_wait<0>();
    Raw v0 = raw_read(0);
    raw_wait(v0);
    store(v0, 0);
    if (nst > 1) {
      Raw v1 = raw_read(1);
      raw_wait(v1);
      store(v1, 1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (nst > 2) issue(0);
    if (nst > 3) issue(1);
    __builtin_amdgcn_s_barrier();
    // the loop's read order (A block 0, B block 0, A block 1, B block 1): hipcc's wait before the first
    // MFMAs of a stage merges the states of both paths into the loop
    __builtin_amdgcn_sched_barrier(0);
    read_a(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_b(0, 0);
    __builtin_amdgcn_sched_barrier(0);
    read_a(0, 1);
    read_b(0, 1);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll 1
    for (int s = 0; s < nst; ++s) {
      const int cur = s % 3;
      const int nxt = cur == 2 ? 0 : cur + 1;
      const int fil = nxt == 2 ? 0 : nxt + 1;
      const int slot = s & 1;
      const bool have2 = s + 2 < nst;
      // stage s + 2's requests (issued two stages ago) landed; stage s + 3's (OPS younger) may not have
      if (s + 3 < nst)
        vm_wait<G::OPS>();
      else
        vm_wait<0>();
      // the raw read after the first MFMAs: hipcc does not count the asm reads, and its wait for this
      // stage's first fragments would otherwise cover them too; issued here, their latency runs under
      // those MFMAs
      __builtin_amdgcn_sched_barrier(0);
      mma6(af[0], bfr[0], acc[0][0]);
      __builtin_amdgcn_sched_barrier(0);
      if (have2) {
        Raw v = raw_read(slot);
        raw_wait(v);  // also retires the previous stage's last fragment reads
        if (!(ABL & 8)) store(v, fil);
      }
      if (s + 4 < nst && !(ABL & 1)) issue(slot);  // stage s + 4, into the slot this lane's read just emptied
      __builtin_amdgcn_sched_barrier(0);
      mma6(af[0], bfr[1], acc[0][1]);
      __builtin_amdgcn_sched_barrier(0);
      read_a(nxt, 0);  // past the last stage: stale data, never used
      __builtin_amdgcn_sched_barrier(0);
      mma6(af[1], bfr[0], acc[1][0]);
      __builtin_amdgcn_sched_barrier(0);
      read_b(nxt, 0);
      __builtin_amdgcn_sched_barrier(0);
      mma6(af[1], bfr[1], acc[1][1]);
      __builtin_amdgcn_sched_barrier(0);
      read_a(nxt, 1);
      read_b(nxt, 1);
      __builtin_amdgcn_sched_barrier(0);
      // every LDS operation but the 12 fragment reads just issued retired (this stage's split stores):
      // after the barrier stage s + 2 is complete for every wave
      asm volatile("s_waitcnt lgkmcnt(12)" ::: "memory");
      if (!(ABL & 4)) __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }

  float* out = a.out + (int64_t)split * a.M * a.N;
#pragma unroll
  for (int ni = 0; ni < 2; ++ni) {
    const int n = nbase + 64 * wn + 32 * ni + rl;
    if (n >= a.N) continue;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = mbase + 64 * wm + 32 * mi + (r & 3) + 8 * (r >> 2) + 4 * hh;
        if (m < a.M) out[(int64_t)m * a.N + n] = __fadd_rn(acc[mi][ni].hi[r], acc[mi][ni].lo[r]);
      }
  }
  if (a.outb != nullptr && nt == 0) {  // the column-tile-0 workgroups write the split's row sums
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      float v = rsum[j];  // the 4 threads of a row are 4 consecutive lanes (t & 3)
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      const int m = mbase + r0 + 128 * j;
      if (qd == 0 && m < a.M) a.outb[(int64_t)split * a.M + m] = v;
    }
  }
}

__global__ void __launch_bounds__(512, 1) gemm_nt_split3_w4(NTArgs a) {
  gemm_nt_split3_body<0>(a, blockIdx.x, gridDim.x);
}

template <int WMW, int L>
hipError_t launch3(Args a, hipStream_t st, void (*kern)(Args)) {
  using G = Geo3<WMW, L>;
  // the B operands' buffer offsets span a column tile's nodes (+ one for a ragged tile): 32-bit
  const int64_t span = ((int64_t)TN / a.P + 2) * (a.b0s > a.b1s ? a.b0s : a.b1s) * 4;
  if (span >= kOffMax) return hipErrorNotSupported;
  a.mtiles = (a.M + G::TM - 1) / G::TM;
  const int64_t grid = (int64_t)a.mtiles * ((a.ncols + TN - 1) / TN);
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS_BYTES);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(G::THREADS), G::LDS_BYTES, st, a);
  return hipGetLastError();
}


}  // namespace mrp_cs
