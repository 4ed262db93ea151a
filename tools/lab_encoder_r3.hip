// lab_encoder_r3.hip — kernel lab (not product code): round 3's split-bf16 edge encoder with the hidden
// layer computed per wave (encoder_body<CB, KS>: one wave per 32 edges x 64 CB columns, W2 by LDS-DMA in
// a four-stage ring, optional hidden split over two wave sets), moved out of the product library in
// round 5: the shared-hidden form (encoder2_body) replaced it (headline 16.7 vs
// 18.7 us; tools/enc_lab.cpp).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/lab_encoder_r3.hip
#include "../multi-robot-perception-gnn-1_amd/csrc/encoder_split.hip"

namespace mrp_x6 {

// LDS stage of one hidden block, shared by the workgroup's four waves (one per 32-edge block, one
// column slab of CB column blocks): NP = 6 CB + 3 pieces of 1 KiB (64 lanes x 16 B, a lane's fragment
// at 16 lane): pieces 0 .. 6 CB - 1 the W2 parts (c, s, p) = 6 c + 3 s + p, then the 3 W1 parts.
// Piece pc is DMA'd by wave pc % 4.
template <int CB>
struct Stage {
  static constexpr int NP = 6 * CB + 3;
  static constexpr int U4 = NP * 64;   // 16-B units per stage
  static constexpr int PW = (NP + 3) / 4;  // most pieces a wave issues per stage
};
constexpr int kStages = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}

// s_waitcnt vmcnt(n) for a wave-uniform n <= 4 (the immediate must be a constant)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
  }
}

template <int CB, int KS>
__device__ __forceinline__ void encoder_body(const FwdArgs& a) {
  using S = Stage<CB>;
  constexpr int NF = S::NP;  // fragments per stage
  constexpr int W1F = 6 * CB;  // first W1 fragment
  extern __shared__ u4 lds_all[];
  // workgroup -> (edge group of 128, column slab of 32 CB); consecutive ids share a slab (its W2
  // image) and, after the remap, an XCD and its L2
  const int nwg = gridDim.x;
  const int orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int eg = id % a.egroups, cs = id / a.egroups;
  const int lane = threadIdx.x & 63;
  const int wall = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wv = wall & 3;   // edge block of the workgroup (and DMA slot within the wave set)
  const int kh = wall >> 2;  // hidden half (KS = 2)
  const int e0 = (eg * 4 + wv) * 32;
  const int HB = a.C / 32 / KS;   // hidden blocks this wave walks
  const int hb0 = kh * HB;        // its first
  u4* lds = lds_all + kh * kStages * S::U4;  // its wave set's stage ring
  const int r = lane & 31, hh = lane >> 5;

  // ---- LDS-DMA: wave wv issues pieces wv, wv + 4, ... of every stage (npw of them)
  const int npw = (S::NP - wv + 3) / 4;
  const int64_t cstride = (int64_t)(a.C / 32) * 2 * 3 * 64;  // 16-B units per W2 column block (all hidden blocks)
  const __amdgpu_buffer_rsrc_t rw = rsrc(a.packed);
  uint32_t voff[S::PW], sstep[S::PW];
#pragma unroll
  for (int i = 0; i < S::PW; ++i) {
    const int pc = wv + 4 * i;
    int64_t unit;  // the piece's first unit at hidden block 0, and its advance per hidden block
    if (pc < W1F) {
      const int c = pc / 6, sp = pc % 6;  // sp = 3 s + p
      unit = w1_units(a.C) + (int64_t)(CB * cs + c) * cstride + sp * 64;
      sstep[i] = 6 * 64 * 16;
    } else {
      unit = (int64_t)(pc < NF ? pc - W1F : 0) * 64;
      sstep[i] = 3 * 64 * 16;
    }
    voff[i] = (uint32_t)((unit + lane) * 16);
  }
  auto issue = [&](int hb) {
    u4* st = lds + (hb % kStages) * S::U4;
#pragma unroll
    for (int i = 0; i < S::PW; ++i)
      if (i < npw)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rw, st + (wv + 4 * i) * 64, 16, voff[i], (uint32_t)(hb0 + hb) * sstep[i], 0, 0);
  };
  // pose fragment (B operand of X = W1' pose'^T): lane's edge, k = 8 hh + j; k = 9 is the 1.0 of b1
  bf8 pp[3];
  {
    const int e = min(e0 + r, a.E - 1);
    const float* pr = a.pose + (int64_t)e * kNin;
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

  issue(0);
  if (HB > 1) issue(1);

  f16v Z[CB], ZL[CB];  // z: a0 b0 products, the five small ones
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) Z[c][i] = ZL[c][i] = 0.f;
  bf8 hp[2][3];  // the previous block's ReLU'd hidden values, split (A operand per 16-unit step)

  // Stage hb landed (own pieces; the younger stage hb + 1 may still be in flight), then the barrier
  // publishes every wave's pieces and certifies that all reads of the previous iteration are done.
  auto stage_ready = [&](int hb) {
    wait_vmcnt(hb + 1 < HB ? npw : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // a stage's fragments into registers: W1 parts first (X needs them first), then the W2 parts
  auto read_frags = [&](int hb, u4 (&w)[NF]) {
    const u4* st = lds + (hb % kStages) * S::U4 + lane;
#pragma unroll
    for (int k = 0; k < 3; ++k) w[W1F + k] = st[(W1F + k) * 64];
#pragma unroll
    for (int k = 0; k < W1F; ++k) w[k] = st[k * 64];
  };
  auto x_block = [&](const u4 (&w)[NF]) {  // X = W1' pose'^T
    bf8 wa[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) wa[p] = as_bf8(w[W1F + p]);
    f16v X;
#pragma unroll
    for (int i = 0; i < 16; ++i) X[i] = 0.f;
    return mma6(wa, pp, X);
  };
  auto split_x = [&](const f16v& X) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      float hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = relu(X[8 * s + j]);
      split8(hv, hp[s]);
    }
  };
  auto z_block = [&](const u4 (&w)[NF]) {  // z += relu(X)^T W2^T (hp holds relu(X) split)
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        bf8 wb[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) wb[p] = as_bf8(w[6 * c + 3 * s + p]);
        mma6_2(hp[s], wb, Z[c], ZL[c]);
      }
  };

  // Iteration hb: the barrier of stage hb, DMA of stage hb + 2 into the buffer stage hb - 2 used, then
  // stage hb's fragments into registers (in flight) while the matrix cores run X of block hb (its W1
  // fragments are read first) and z of block hb - 1 (fragments already in registers), then X's ReLU
  // and split on the VALU.
  u4 F[NF], G[NF];
  auto step = [&](int hb, u4 (&cur)[NF], u4 (&nxt)[NF]) {  // cur: stage hb - 1's fragments
    stage_ready(hb);
    if (hb + 2 < HB) issue(hb + 2);
    read_frags(hb, nxt);
    const f16v X = x_block(nxt);
    z_block(cur);
    split_x(X);
  };
  stage_ready(0);
  if (HB > 2) issue(2);
  read_frags(0, F);
  split_x(x_block(F));
  int hb = 1;
#pragma unroll 1
  for (; hb + 1 < HB; hb += 2) {  // two blocks per trip, so the fragment sets swap roles without copies
    step(hb, F, G);
    step(hb + 1, G, F);
  }
  if (hb < HB) {
    step(hb, F, G);
#pragma unroll
    for (int k = 0; k < NF; ++k) F[k] = G[k];
  }
  z_block(F);
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) Z[c][i] = __fadd_rn(Z[c][i], ZL[c][i]);

  if constexpr (KS == 2) {
    // the second wave set's partials through LDS (the stage rings are idle: every DMA was waited
    // for and every fragment read retired before this barrier), added in a fixed order
    float* zx = reinterpret_cast<float*>(lds_all);
    __syncthreads();
    if (kh == 1) {
#pragma unroll
      for (int c = 0; c < CB; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) zx[((wv * CB + c) * 16 + i) * 64 + lane] = Z[c][i];
    }
    __syncthreads();
    if (kh == 1) return;
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int i = 0; i < 16; ++i) Z[c][i] += zx[((wv * CB + c) * 16 + i) * 64 + lane];
  }
  // epilogue: accumulator register i of lane (r, hh) is edge e0 + (i & 3) + 8 (i >> 2) + 4 hh, column r
  if (e0 >= a.E) return;  // a wave past the last edge (only the stores are skipped: it took part in the barriers)
  const int N = 2 * a.C;
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    const int col = (CB * cs + c) * 32 + r;
    const float bias = a.b2 != nullptr ? a.b2[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = e0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (e < a.E) a.z[(int64_t)e * N + col] = __fadd_rn(Z[c][i], bias);
    }
  }
}

// one kernel per (column-block count, hidden split) (plain kernels around the template body)
__global__ void __launch_bounds__(256) encoder_fwd_cb1(FwdArgs a) { encoder_body<1, 1>(a); }
__global__ void __launch_bounds__(256) encoder_fwd_cb2(FwdArgs a) { encoder_body<2, 1>(a); }
__global__ void __launch_bounds__(512) encoder_fwd_cb1_k2(FwdArgs a) { encoder_body<1, 2>(a); }
__global__ void __launch_bounds__(512) encoder_fwd_cb2_k2(FwdArgs a) { encoder_body<2, 2>(a); }

template <int CB, int KS>
hipError_t launch_cfg(void (*kern)(FwdArgs), const FwdArgs& a, int64_t grid, hipStream_t st) {
  const size_t lds = (size_t)KS * kStages * Stage<CB>::U4 * 16;  // >= the KS = 2 exchange (4 CB KiB x 4)
  static_assert(KS == 1 || (size_t)KS * kStages * Stage<CB>::U4 * 16 >= (size_t)4 * CB * 16 * 64 * 4, "exchange fits");
  static const hipError_t attr =
      hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256 * KS), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_fwd(int cb, int ks, const FwdArgs& a, int64_t grid, hipStream_t st) {
  if (ks == 2)
    return cb == 2 ? launch_cfg<2, 2>(encoder_fwd_cb2_k2, a, grid, st) : launch_cfg<1, 2>(encoder_fwd_cb1_k2, a, grid, st);
  return cb == 2 ? launch_cfg<2, 1>(encoder_fwd_cb2, a, grid, st) : launch_cfg<1, 1>(encoder_fwd_cb1, a, grid, st);
}


}  // namespace mrp_x6
