// encoder_split.hip — the edge encoder before its Sigmoid in one launch on the bf16 matrix cores,
// at fp32 accuracy, gfx950 (MI355X / CDNA4).
//
// Reference (xjh19971/multi-robot-perception-gnn-1, dgl/model/models.py:146-149):
//     z = Linear(C, 2C)(ReLU(Linear(9, C)(pose)))          pose (E, 9) -> z (E, 2C)
// (the Sigmoid of models.py:150 runs inside the aggregation kernels, MRP_AGG_GB_LOGITS).
//
// Arithmetic.  Every fp32 operand value x is split exactly into three bf16 parts,
//     x = x0 + x1 + x2 (+ a residual below 2^-24 |x|),  x0 = bf16(x), x1 = bf16(x - x0), x2 = bf16(x - x0 - x1)
// (each subtraction is exact in fp32; round-to-nearest conversions, v_cvt_pk_bf16_f32), and a product
// a b is the sum of the six partial products a_i b_j with i + j <= 2 — each exact in the MFMA (8 x 8
// significant bits), summed into an fp32 accumulator, smallest terms first.  The omitted terms are
// below 2^-25 |a b|, so the result is as accurate as an fp32 GEMM (tests/test_gpu_encoder.py checks
// it against float64 with the same yardstick as the fp32 kernels); it runs on
// v_mfma_f32_32x32x16_bf16, six of which cost 192 cycles per 16 k against 512 for the fp32 MFMA.
//
// Structure: the shared-hidden form below (encoder2_body).  A workgroup of 4 or 8 waves owns one
// block of 32 edges and one 32-column block of z per wave; the hidden layer X (32 units x 32 edges per
// hidden block) is computed on the MFMAs by the waves in turn, ReLU'd, split and shared through LDS
// slots, and every wave runs z for its own columns with its W2 fragments loaded from the packed image
// straight into registers, four sets in rotation.  Round 3's per-wave form and the two-column-block
// and hidden-split forms are lab code (tools/lab_encoder_r3.hip); round 6's split-K over workgroups
// (hidden-block slices, the last arriver of a tile summing the partials) measured slower at the
// headline — 23.4 / 26.0 us for 2 / 4 slices against 21.8 in-step — and is kept as
// tools/lab_patches/r06_encoder_splitk.patch.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrp_gnn.h"
#include "tuning.hpp"

#include "encoder_split.hpp"

namespace mrp_x6 {

__global__ void __launch_bounds__(256) pack(const float* __restrict__ w1, const float* __restrict__ b1,
                                            const float* __restrict__ w2, int C, u4* __restrict__ out) {
  const int HB = C / 32;
  const int64_t n1 = (int64_t)HB * 64, n2 = (int64_t)(2 * C / 32) * HB * 2 * 64;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n1 + n2) return;
  float v[8];
  bf8 p[3];
  int64_t dst;
  const int l = (int)(t & 63);
  const int h = l >> 5;
  if (t < n1) {
    const int hb = (int)(t >> 6);
    const int u = 32 * hb + (l & 31);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * h + j;
      v[j] = k < kNin ? w1[(int64_t)u * kNin + k] : (k == kNin ? b1[u] : 0.f);
    }
    dst = (int64_t)hb * 3 * 64 + l;
  } else {
    const int64_t g = (t - n1) >> 6;  // ((cb * HB + hb) * 2 + s)
    const int s = (int)(g & 1);
    const int64_t cbhb = g >> 1;
    const int hb = (int)(cbhb % HB);
    const int cb = (int)(cbhb / HB);
    const int col = 32 * cb + (l & 31);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = w2[(int64_t)col * C + 32 * hb + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3)];
    dst = w1_units(C) + g * 3 * 64 + l;
  }
  split8(v, p);
#pragma unroll
  for (int q = 0; q < 3; ++q) out[dst + q * 64] = as_u4(p[q]);
}

struct FwdArgs {
  const float* pose;
  const u4* packed;
  const float* b2;
  float* z;
  float* hT;     // shared-hidden forms, training: relu(pose W1^T + b1) transposed, (C, E) rows of hts floats
  int64_t hts;
  int32_t E, C, egroups;
};

// ------------------------------------------------------------------------------------------------
// Shared-hidden form (mrp_edge_encoder_fwd_split's default).  A workgroup's NWV waves share one block
// of 32 edges and own NWV x CB adjacent 32-column blocks of z.  Per round of NWV hidden blocks, wave w
// computes X (32 units x 32 edges) of hidden block round NWV + w on the matrix cores, applies the ReLU,
// splits it and stores its A-operand fragments (6 x 16 B per lane, lane-linear) in an LDS slot; after
// one barrier every wave reads all NWV blocks' fragments with ds_read_b128 (the same registers the
// computing wave held) and runs z for its own columns, its W2 fragments loaded straight from the
// packed image into registers one hidden block ahead (no wave of the workgroup shares them).
// The hidden layer is computed 2C / (32 NWV CB) times per edge instead of 2C / (32 CB) times, its
// ReLU/split VALU work is spread over the waves, and the grid has E/32 x 2C/(32 NWV CB) workgroups.
// The next round's X runs after the current round's z (its W1 loads issued before), so with two
// waves per SIMD one wave's VALU split runs beside the other's MFMAs.
// ------------------------------------------------------------------------------------------------
template <int CB, int NWV, int ABL = 0, bool ALLX = false>  // ABL: lab ablation bits (tools/enc_ablate.hip; 0 here)
__device__ __forceinline__ void encoder2_body(const FwdArgs& a) {
  extern __shared__ u4 lds_all[];
  const int HB = a.C / 32;
  const int ncb = 2 * a.C / 32;                 // 32-column blocks of z
  constexpr int CPG = NWV * CB;                  // column blocks per workgroup
  const int eblocks = (a.E + 31) / 32;
  // workgroup -> (column group, edge block); consecutive ids share a column group (its W2 slab) and,
  // after the remap, an XCD and its L2
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  const int id = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
  const int eb = id % eblocks, cg = id / eblocks;
  const int ngroups = (ncb + CPG - 1) / CPG;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, hh = lane >> 5;
  const int e0 = eb * 32;
  const u4* img = a.packed;

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
  // this wave's column blocks (past the last: clamped for loads, never stored)
  int cbw[CB];
  const u4* w2p[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    cbw[c] = cg * CPG + w * CB + c;
    w2p[c] = img + w1_units(a.C) + (int64_t)min(cbw[c], ncb - 1) * HB * 6 * 64 + lane;
  }
  typedef u4 W2F[CB][6];
  auto load_w2 = [&](int hb, W2F& f) {
#pragma unroll
    for (int c = 0; c < CB; ++c)
#pragma unroll
      for (int k = 0; k < 6; ++k) {
        if (ABL & 1)
          f[c][k] = u4{(uint32_t)hb, (uint32_t)k, (uint32_t)lane, 0u};
        else
          f[c][k] = w2p[c][(int64_t)(hb * 6 + k) * 64];
      }
  };
  // X of hidden block hb, ReLU'd and split, into LDS slot (buf, w)
  u4 w1f[3], w1g[3];
  auto load_w1_into = [&](int hb, u4 (&dst)[3]) {
#pragma unroll
    for (int p = 0; p < 3; ++p) dst[p] = img[(int64_t)(min(hb, HB - 1) * 3 + p) * 64 + lane];
  };
  auto load_w1 = [&](int hb) { load_w1_into(hb, w1f); };
  // all-X form, training: relu(X) of the wave's two hidden blocks kept here and h^T stored after the z
  // loop, so the stores and their addressing do not sit between the W2 requests and the first z block
  // (round 5, tools/ab_encoder_libs.py --train: 18.0 vs 18.5 us at the headline shape, bit-identical)
  f16v Xk[2];
  auto x_store_from = [&](int buf, int hbx, const u4 (&wsrc)[3]) {
    bf8 wa[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) wa[p] = as_bf8(wsrc[p]);
    f16v X;
#pragma unroll
    for (int i = 0; i < 16; ++i) X[i] = 0.f;
    if (!(ABL & 2)) X = mma6(wa, pp, X);
    // training: h^T written by one workgroup per (edge block, hidden block) — every column group computes
    // every X of its edge block, so the column groups take the hidden blocks round robin and share the
    // stores (register i of lane (r, hh) is unit (i & 3) + 8 (i >> 2) + 4 hh of the block, edge e0 + r:
    // each register's 32 lanes store 128 contiguous bytes of a row)
    if constexpr (ALLX) {
      Xk[buf] = X;
    } else if (a.hT != nullptr && hbx % ngroups == cg && hbx < HB && e0 + r < a.E) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        a.hT[(int64_t)(hbx * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * a.hts + e0 + r] = relu(X[i]);
    }
    u4* slot = lds_all + (buf * NWV + w) * 6 * 64 + lane;
    if (ABL & 64) return;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float hv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) hv[j] = relu(X[8 * s2 + j]);
      bf8 hp[3];
      split8(hv, hp);
#pragma unroll
      for (int p = 0; p < 3; ++p) slot[(s2 * 3 + p) * 64] = as_u4(hp[p]);
    }
  };
  auto x_store = [&](int buf, int hbx) { x_store_from(buf, hbx, w1f); };
  f16v Z[CB], ZL[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c)
#pragma unroll
    for (int i = 0; i < 16; ++i) Z[c][i] = ZL[c][i] = 0.f;
  auto z_block = [&](int buf, int j, const W2F& f) {
    const u4* slot = lds_all + (buf * NWV + j) * 6 * 64 + lane;
    bf8 hp[2][3];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int p = 0; p < 3; ++p)
        hp[s2][p] = (ABL & 16) ? as_bf8(u4{(uint32_t)j, (uint32_t)p, (uint32_t)lane, (uint32_t)s2})
                               : as_bf8(slot[(s2 * 3 + p) * 64]);
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        bf8 wb[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) wb[p] = as_bf8(f[c][3 * s2 + p]);
        if (ABL & 8) {
#pragma unroll
          for (int p = 0; p < 3; ++p) Z[c][p] += __builtin_bit_cast(float, as_u4(hp[s2][p]).x ^ as_u4(wb[p]).x);
        } else {
          mma6_2(hp[s2], wb, Z[c], ZL[c]);
        }
      }
  };

  const int rounds = (HB + NWV - 1) / NWV;
  // W2 fragments of hidden blocks hb in set hb % 4, requested three blocks ahead (one block's z is 12 CB
  // MFMAs per wave: too short to cover an L2 round trip under load); NWV % 4 == 0, so a round's
  // blocks take the sets in a fixed order
  static_assert(NWV % 4 == 0, "four W2 sets per round");
  W2F f0, f1, f2, f3;
  // every hidden block fits the two slot sets (HB <= 2 NWV: C <= 512 with 8 waves): all of X first — each
  // wave computes blocks w and w + NWV — one barrier, then z straight through all HB blocks with no
  // further barrier or X in between (the rounds below put a barrier and a VALU split phase between
  // every NWV blocks, with both waves of a SIMD in the split at the same time)
  constexpr bool allx = ALLX;  // the launcher's choice: HB <= 2 NWV
  load_w1(w);
  if (allx && w + NWV < HB) load_w1_into(w + NWV, w1g);
  load_w2(0, f0);
  if (1 < HB) load_w2(1, f1);
  if (2 < HB) load_w2(2, f2);
  x_store(0, w);
  if constexpr (allx) {
    if (w + NWV < HB) x_store_from(1, w + NWV, w1g);
    __syncthreads();
#pragma unroll 1
    for (int hb = 0; hb < HB; hb += 4) {
      if (hb + 3 < HB) load_w2(hb + 3, f3);
      z_block(hb / NWV, hb % NWV, f0);
      if (hb + 4 < HB) load_w2(hb + 4, f0);
      if (hb + 1 < HB) z_block((hb + 1) / NWV, (hb + 1) % NWV, f1);
      if (hb + 5 < HB) load_w2(hb + 5, f1);
      if (hb + 2 < HB) z_block((hb + 2) / NWV, (hb + 2) % NWV, f2);
      if (hb + 6 < HB) load_w2(hb + 6, f2);
      if (hb + 3 < HB) z_block((hb + 3) / NWV, (hb + 3) % NWV, f3);
    }
    if (a.hT != nullptr && e0 + r < a.E) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int hbx = w + q * NWV;
        if (hbx < HB && hbx % ngroups == cg) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            a.hT[(int64_t)(hbx * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * a.hts + e0 + r] = relu(Xk[q][i]);
        }
      }
    }
  } else {
  __syncthreads();
#pragma unroll 1
  for (int rd = 0; rd < rounds; ++rd) {
    const int buf = rd & 1;
    const bool more = rd + 1 < rounds;
    if (more) load_w1((rd + 1) * NWV + w);  // the next round's X, under this round's MFMAs
#pragma unroll
    for (int j = 0; j < NWV; j += 4) {
      const int hb = rd * NWV + j;
      if (hb + 3 < HB) load_w2(hb + 3, f3);
      if (hb < HB) z_block(buf, j, f0);
      if (hb + 4 < HB) load_w2(hb + 4, f0);
      if (hb + 1 < HB) z_block(buf, j + 1, f1);
      if (hb + 5 < HB) load_w2(hb + 5, f1);
      if (hb + 2 < HB) z_block(buf, j + 2, f2);
      if (hb + 6 < HB) load_w2(hb + 6, f2);
      if (hb + 3 < HB) z_block(buf, j + 3, f3);
    }
    if (more) x_store(buf ^ 1, (rd + 1) * NWV + w);  // slot buf ^ 1: last read in round rd - 1, before the last barrier
    if (!(ABL & 4)) __syncthreads();
  }
  }
  // epilogue: accumulator register i of lane (r, hh) is edge e0 + (i & 3) + 8 (i >> 2) + 4 hh, column r
  const int N = 2 * a.C;
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    if (cbw[c] >= ncb) continue;
    const int col = cbw[c] * 32 + r;
    const float bias = a.b2 != nullptr ? a.b2[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = e0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      const float v = __fadd_rn(__fadd_rn(Z[c][i], ZL[c][i]), bias);
      if ((ABL & 32) ? (v == 1.2345f && e < a.E) : e < a.E) a.z[(int64_t)e * N + col] = v;
    }
  }
}

__global__ void __launch_bounds__(256) encoder2_cb1_w4(FwdArgs a) { encoder2_body<1, 4>(a); }
__global__ void __launch_bounds__(512) encoder2_cb1_w8(FwdArgs a) { encoder2_body<1, 8>(a); }
__global__ void __launch_bounds__(256) encoder2_cb1_w4_allx(FwdArgs a) { encoder2_body<1, 4, 0, true>(a); }
__global__ void __launch_bounds__(512) encoder2_cb1_w8_allx(FwdArgs a) { encoder2_body<1, 8, 0, true>(a); }

template <int CB, int NWV>
hipError_t launch2_cfg(void (*kern)(FwdArgs), const FwdArgs& a, hipStream_t st) {
  const int64_t eblocks = (a.E + 31) / 32;
  const int64_t groups = (2 * (int64_t)a.C / 32 + NWV * CB - 1) / (NWV * CB);
  const int64_t grid = eblocks * groups;
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  const size_t lds = (size_t)2 * NWV * 6 * 64 * 16;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64 * NWV), lds, st, a);
  return hipGetLastError();
}

hipError_t launch_fwd2(int nwv, const FwdArgs& a, hipStream_t st) {
  const bool allx = a.C / 32 <= 2 * nwv && mrp_host::tuning().edge_allx;  // every X before z (encoder2_body)
  if (nwv == 8)
    return allx ? launch2_cfg<1, 8>(encoder2_cb1_w8_allx, a, st) : launch2_cfg<1, 8>(encoder2_cb1_w8, a, st);
  return allx ? launch2_cfg<1, 4>(encoder2_cb1_w4_allx, a, st) : launch2_cfg<1, 4>(encoder2_cb1_w4, a, st);
}

// the form per shape (mrp_tuning_set "edge_split_v": 3 = 8 waves, 1 = 4 waves per workgroup): 8 waves
// when that gives one round of 192..256 workgroups, else 4 (round 5; round 4: at least 192).  Per shape (tools/enc_lab.cpp, us, round 3's per-wave
// hidden layer / (1, 4) / (1, 8)): E=1792 C=512 18.7 / 18.5 / 16.7, E=896 C=512 13.3 / 12.6 / 15.3,
// E=1792 C=1280 99.7 / 91.3 / 94.7, E=448 C=2048 55.4 / 60.5 / 52.6, E=512 C=1024 21.0 / 21.2 / 26.4;
// two column blocks per wave slower everywhere.  Round 3's per-wave form (edge_split_v 0) and the
// two-column-block forms are no longer built (their source: tools/lab_encoder_r3.hip).
// Round 5 (tools/ab_encoder_waves.py, HIP-graph timed, us for 4 / 8 waves): E=1792 C=512 19.1 / 17.7,
// E=896 C=512 13.1 / 16.0, E=1792 C=1280 88.5 / 92.4, E=448 C=2048 57.3 / 51.6, E=512 C=1024 20.4 / 25.1:
// 8 waves only where their grid is one round of 192..256 workgroups (one per CU)
int fwd2_waves(int32_t num_edges, int32_t C) {
  int v = mrp_host::tuning().edge_split_v;
  if (v < 0) {
    const int64_t grid8 = ((int64_t)(num_edges + 31) / 32) * (2 * (int64_t)C / 256);
    v = grid8 >= 192 && grid8 <= 256 ? 3 : 1;
  }
  return v == 3 ? 8 : 4;
}

}  // namespace mrp_x6

using namespace mrp_x6;

namespace {
// the kernels address the packed image with 32-bit byte offsets (buffer resource, num_records
// 0x7fffffff): the image (96 C + 12 C^2 bytes) must stay below 2^31 bytes, i.e. C <= 13344
bool image_fits(int32_t C) { return (w1_units(C) + w2_units(C)) * 16 < ((int64_t)1 << 31); }
}  // namespace

extern "C" int64_t mrp_edge_encoder_pack_bytes(int32_t C) {
  if (C <= 0 || C % 32 != 0) return 0;
  return (w1_units(C) + w2_units(C)) * 16;
}

extern "C" int mrp_edge_encoder_pack(const float* w1, const float* b1, const float* w2, int32_t C, void* packed,
                                     void* stream) {
  if (C <= 0) return hipErrorInvalidValue;
  if (C % 32 != 0 || !image_fits(C)) return hipErrorNotSupported;
  if (!w1 || !b1 || !w2 || !packed || (reinterpret_cast<uintptr_t>(packed) & 15)) return hipErrorInvalidValue;
  const int64_t threads = (w1_units(C) + w2_units(C)) / 3;
  if ((threads + 255) / 256 > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, static_cast<hipStream_t>(stream), w1,
                     b1, w2, C, static_cast<u4*>(packed));
  return hipGetLastError();
}

extern "C" int mrp_edge_encoder_fwd_split(const float* pose, const void* packed, const float* b2, int32_t num_edges,
                                          int32_t C, float* z, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (C % 32 != 0 || !image_fits(C)) return hipErrorNotSupported;
  if (!pose || !packed || !z || (reinterpret_cast<uintptr_t>(packed) & 15)) return hipErrorInvalidValue;
  FwdArgs a;
  a.pose = pose;
  a.packed = static_cast<const u4*>(packed);
  a.b2 = b2;
  a.z = z;
  a.hT = nullptr;
  a.hts = 0;
  a.E = num_edges;
  a.C = C;
  a.egroups = (num_edges + 127) / 128;
  return launch_fwd2(fwd2_waves(num_edges, C), a, static_cast<hipStream_t>(stream));
}

extern "C" int mrp_edge_encoder_fwd_split_train(const float* pose, const void* packed, const float* b2,
                                                int32_t num_edges, int32_t C, float* z, float* hT, int64_t hT_stride,
                                                void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (C % 32 != 0 || !image_fits(C)) return hipErrorNotSupported;
  if (!pose || !packed || !z || !hT || hT_stride < num_edges || (reinterpret_cast<uintptr_t>(packed) & 15))
    return hipErrorInvalidValue;
  FwdArgs a;
  a.pose = pose;
  a.packed = static_cast<const u4*>(packed);
  a.b2 = b2;
  a.z = z;
  a.hT = hT;
  a.hts = hT_stride;
  a.E = num_edges;
  a.C = C;
  a.egroups = (num_edges + 127) / 128;
  // the shared-hidden form, its column groups sharing the h^T stores (per-shape choice as the inference entry)
  return launch_fwd2(fwd2_waves(num_edges, C), a, static_cast<hipStream_t>(stream));
}
