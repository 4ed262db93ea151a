// edge_encoder.hip — first layer of the FiLM parameter generator for gfx950 (MI355X / CDNA4).
//
// The reference edge encoder (dgl/model/models.py:146-154) is
//     z = W2 relu(W1 pose + b1) + b2 ;  gamma/beta = sigmoid(z).view(E, C, 2)
// On this path it is split three ways:
//   * h = relu(W1 pose + b1)  — this kernel: K = 9, so it is a streaming write of E x C floats
//     (one launch instead of torch's GEMM + ReLU pair);
//   * z = h W2^T + b2         — a plain fp32 library GEMM (hipBLASLt/rocBLAS via torch.addmm, bias in
//     its epilogue): M = E, N = 2C, K = C, the only dense contraction of the encoder;
//   * sigmoid                 — fused into the aggregation kernels, which read the (E, C, 2) logits
//     (MRP_AGG_GB_LOGITS) and apply it while building their weight tiles.
// (A fully fused single-kernel encoder on the fp32 MFMA was built and measured at 41-49 us against
// 24 us for the library GEMM at E=1792, C=512: this GEMM is too small per CU — 1.75 waves per SIMD —
// for a barrier-synchronised LDS pipeline.  See DESIGN.md.)

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "mrp_gnn.h"

namespace mrp_enc {

constexpr int NIN = 9;  // relative pose width (dgl/utils.py:77)

constexpr int EPB = 4;  // edges per workgroup

// Workgroup = EPB edges x all C hidden units; thread -> hidden units k = tid, tid + 256, ... whose W1
// rows and b1 it keeps in registers across the EPB edges.  Edge pose values are wave-uniform
// (scalar loads); each store instruction writes 256 contiguous bytes of h.
template <int KPT>
__global__ void __launch_bounds__(256) edge_hidden_fwd(const float* __restrict__ pose, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, float* __restrict__ h, int E,
                                                       int C) {
  float w[KPT][NIN + 1];
#pragma unroll
  for (int j = 0; j < KPT; ++j) {
    const int k = threadIdx.x + 256 * j;
#pragma unroll
    for (int i = 0; i < NIN; ++i) w[j][i] = k < C ? w1[(int64_t)k * NIN + i] : 0.f;
    w[j][NIN] = k < C ? b1[k] : 0.f;
  }
  const int e_end = min(E, (int)(blockIdx.x + 1) * EPB);
  for (int e = blockIdx.x * EPB; e < e_end; ++e) {
    float p[NIN];
#pragma unroll
    for (int i = 0; i < NIN; ++i) p[i] = pose[(int64_t)e * NIN + i];
#pragma unroll
    for (int j = 0; j < KPT; ++j) {
      const int k = threadIdx.x + 256 * j;
      if (k >= C) break;
      float acc = w[j][NIN];
#pragma unroll
      for (int i = 0; i < NIN; ++i) acc = fmaf(p[i], w[j][i], acc);
      h[(int64_t)e * C + k] = acc > 0.f ? acc : 0.f;
    }
  }
}

}  // namespace mrp_enc

extern "C" int mrp_edge_hidden_fwd(const float* pose, const float* w1, const float* b1, int32_t num_edges,
                                   int32_t C, float* h, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (!pose || !w1 || !b1 || !h) return hipErrorInvalidValue;
  const int64_t blocks = ((int64_t)num_edges + mrp_enc::EPB - 1) / mrp_enc::EPB;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  const int kpt = (C + 255) / 256;  // hidden units per thread
  hipStream_t st = static_cast<hipStream_t>(stream);
#define MRP_HIDDEN(KPT) \
  hipLaunchKernelGGL(mrp_enc::edge_hidden_fwd<KPT>, dim3((unsigned)blocks), dim3(256), 0, st, pose, w1, b1, h, num_edges, C)
  if (kpt <= 1) MRP_HIDDEN(1);
  else if (kpt <= 2) MRP_HIDDEN(2);
  else if (kpt <= 4) MRP_HIDDEN(4);
  else if (kpt <= 8) MRP_HIDDEN(8);
  else if (kpt <= 16) MRP_HIDDEN(16);
  else return hipErrorInvalidValue;  // C > 4096
#undef MRP_HIDDEN
  return hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// Backward of the encoder's small reductions (dgl/model/models.py:147-149), after the two library
// GEMMs dh = dz W2 and dW2 = dz^T h:
//   db2[j]    = sum_e dz[e, j]                         (2C columns)
//   dw1[k, i] = sum_e dh[e, k] [h[e, k] > 0] pose[e, i] (ReLU backward folded in)
//   db1[k]    = sum_e dh[e, k] [h[e, k] > 0]
// Torch runs these as compare + mul + a K = E GEMM + two column reductions (five launches).  Here:
// pass 1 = one thread per output column per chunk of kRows edges (coalesced row reads, the 9 pose
// values wave-uniform), partial sums to a workspace; pass 2 = the sum over chunks in chunk order.
// Deterministic: no atomics, a fixed summation order.
// ---------------------------------------------------------------------------------------------
namespace mrp_enc {

constexpr int kRows = 16;  // edges per chunk: 672 workgroups at E = 1792, C = 512 (64 rows: 168 workgroups, 24 us; 16 rows: 7.4 us)

// workspace row per chunk: [0, 2C) db2 partials, then per hidden unit k: 9 dw1 + 1 db1 partials
__global__ void __launch_bounds__(256) encoder_bwd_partial(const float* __restrict__ dz, const float* __restrict__ dh,
                                                           const float* __restrict__ h, const float* __restrict__ pose,
                                                           int E, int C, float* __restrict__ ws) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;  // [0, 2C): dz column, [2C, 3C): hidden unit
  const int chunk = blockIdx.y;
  const int e0 = chunk * kRows;
  const int e1 = min(E, e0 + kRows);
  float* out = ws + (int64_t)chunk * 12 * C;
  if (col < 2 * C) {
    float acc = 0.f;
#pragma unroll 4
    for (int e = e0; e < e1; ++e) acc += dz[(int64_t)e * 2 * C + col];
    out[col] = acc;
  } else if (col < 3 * C) {
    const int k = col - 2 * C;
    float acc[NIN + 1];
#pragma unroll
    for (int i = 0; i <= NIN; ++i) acc[i] = 0.f;
#pragma unroll 4
    for (int e = e0; e < e1; ++e) {
      const float g = dh[(int64_t)e * C + k];
      const float d = h[(int64_t)e * C + k] > 0.f ? g : 0.f;
#pragma unroll
      for (int i = 0; i < NIN; ++i) acc[i] = fmaf(d, pose[(int64_t)e * NIN + i], acc[i]);
      acc[NIN] += d;
    }
#pragma unroll
    for (int i = 0; i <= NIN; ++i) out[2 * C + k * (NIN + 1) + i] = acc[i];
  }
}

// 16 outputs x 16 chunk segments per workgroup (12C/16 workgroups: 384 at C = 512); each segment's
// partial goes through LDS and segment 0 adds them in segment order (deterministic)
__global__ void __launch_bounds__(256) encoder_bwd_final(const float* __restrict__ ws, int nchunks, int C,
                                                         float* __restrict__ db2, float* __restrict__ dw1,
                                                         float* __restrict__ db1) {
  __shared__ float part[16][16];
  const int o = threadIdx.x & 15, sg = threadIdx.x >> 4;
  const int t = blockIdx.x * 16 + o;
  const int per = (nchunks + 15) / 16;
  const int c0 = sg * per, c1 = min(nchunks, c0 + per);
  float acc = 0.f;
  if (t < 12 * C) {
#pragma unroll 4
    for (int c = c0; c < c1; ++c) acc += ws[(int64_t)c * 12 * C + t];
  }
  part[sg][o] = acc;
  __syncthreads();
  if (sg != 0 || t >= 12 * C) return;
  acc = part[0][o];
#pragma unroll
  for (int k = 1; k < 16; ++k) acc += part[k][o];
  if (t < 2 * C) {
    if (db2) db2[t] = acc;
  } else {
    const int k = (t - 2 * C) / (NIN + 1), i = (t - 2 * C) - k * (NIN + 1);
    if (i < NIN) {
      if (dw1) dw1[(int64_t)k * NIN + i] = acc;
    } else if (db1) {
      db1[k] = acc;
    }
  }
}

}  // namespace mrp_enc

extern "C" int64_t mrp_edge_encoder_bwd_workspace(int32_t num_edges, int32_t C) {
  if (num_edges <= 0 || C <= 0) return 0;
  const int64_t nchunks = ((int64_t)num_edges + mrp_enc::kRows - 1) / mrp_enc::kRows;
  return nchunks * 12 * (int64_t)C * (int64_t)sizeof(float);
}

extern "C" int mrp_edge_encoder_bwd(const float* dz, const float* dh, const float* h, const float* pose,
                                    int32_t num_edges, int32_t C, float* db2, float* dw1, float* db1,
                                    float* workspace, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (C == 0) return hipSuccess;
  if (num_edges == 0) {  // empty sums
    hipError_t e = hipSuccess;
    if (db2) e = hipMemsetAsync(db2, 0, sizeof(float) * 2 * (size_t)C, st);
    if (e == hipSuccess && dw1) e = hipMemsetAsync(dw1, 0, sizeof(float) * mrp_enc::NIN * (size_t)C, st);
    if (e == hipSuccess && db1) e = hipMemsetAsync(db1, 0, sizeof(float) * (size_t)C, st);
    return e;
  }
  if (!dz || !dh || !h || !pose || !workspace) return hipErrorInvalidValue;
  if ((int64_t)C * 12 > 0x7fffffff / 2) return hipErrorInvalidValue;
  const int nchunks = (num_edges + mrp_enc::kRows - 1) / mrp_enc::kRows;
  if (nchunks > 65535) return hipErrorInvalidValue;  // grid.y limit: E up to ~4.2M edges
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_partial, dim3((3 * C + 255) / 256, nchunks), dim3(256), 0, st, dz, dh, h,
                     pose, num_edges, C, workspace);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_final, dim3((12 * C + 15) / 16), dim3(256), 0, st, workspace, nchunks, C,
                     db2, dw1, db1);
  return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Backward in the transposed layout of the split-bf16 training path (encoder.py, EdgeEncoderSplitFunction):
// the forward wrote h^T (C, E); the two GEMMs dh^T = W2^T dz^T and dW2 = dz^T h run on the split-bf16
// weight-gradient kernel (compress_split.hip, mrp_edge_encoder_bwd_split, which also takes db2 as the
// row sums of dz^T), whose operands are rows with k contiguous — so dz is first transposed:
//   mrp_edge_encoder_bwd_prep:  dzT[j][e] = dz[e][j]
//   mrp_edge_encoder_bwd_t:     dpre = dh^T (.) [h^T > 0];  dw1[k][i] = sum_e dpre[k][e] pose[e][i],
//                               db1[k] = sum_e dpre[k][e]
// The e sums run per 256-edge block (fixed lane order, fixed butterfly) into partials summed over the
// blocks in order by a second pass: deterministic.
// ------------------------------------------------------------------------------------------------
namespace mrp_enc {

typedef float f4t __attribute__((ext_vector_type(4)));

// 64 (e) x 64 (j) tile through LDS (+1 padding), 16-byte accesses both ways: thread t moves the 4-float
// pieces (t & 15) of rows (t >> 4) + 16 i; E % 4 == 0 and N2 % 4 == 0 (checked by the entry point)
__global__ void __launch_bounds__(256) dz_transpose(const float* __restrict__ dz, int E, int N2,
                                                    float* __restrict__ dzT, int64_t dzT_stride) {
  __shared__ float tile[64][65];
  const int j0 = blockIdx.x * 64, e0 = blockIdx.y * 64;
  const int c4 = threadIdx.x & 15, r0 = threadIdx.x >> 4;
  f4t v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = e0 + r0 + 16 * i, j = j0 + 4 * c4;
    v[i] = (e < E && j < N2) ? *reinterpret_cast<const f4t*>(dz + (int64_t)e * N2 + j) : f4t{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) tile[r0 + 16 * i][4 * c4 + q] = v[i][q];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int jr = r0 + 16 * i, j = j0 + jr, e = e0 + 4 * c4;
    f4t o;
#pragma unroll
    for (int q = 0; q < 4; ++q) o[q] = tile[4 * c4 + q][jr];
    if (j < N2 && e < E) *reinterpret_cast<f4t*>(dzT + (int64_t)j * dzT_stride + e) = o;
  }
}

constexpr int BT_E = 256;  // edges per block of encoder_bwd_t

// block (k group of 4, e block): wave w sums unit k = 4 blockIdx.x + w over the block's 256 edges; the
// block's pose rows are staged in LDS once; partial [e block][k][10] (9 dw1 terms, db1)
__global__ void __launch_bounds__(256) encoder_bwd_t(const float* __restrict__ dhT, int64_t dhs,
                                                     const float* __restrict__ hT, int64_t hs,
                                                     const float* __restrict__ pose, int E, int C,
                                                     float* __restrict__ part) {
  __shared__ float ps[BT_E * NIN];
  const int eb = blockIdx.y, ebase = eb * BT_E;
  const int nrow = E - ebase < BT_E ? E - ebase : BT_E;
  for (int i = threadIdx.x; i < nrow * NIN; i += 256) ps[i] = pose[(int64_t)ebase * NIN + i];
  __syncthreads();
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (k >= C) return;
  float hv[BT_E / 64], dv[BT_E / 64];
#pragma unroll
  for (int it = 0; it < BT_E / 64; ++it) {
    const int el = lane + 64 * it;
    hv[it] = el < nrow ? hT[(int64_t)k * hs + ebase + el] : 0.f;
    dv[it] = el < nrow ? dhT[(int64_t)k * dhs + ebase + el] : 0.f;
  }
  float acc[NIN + 1];
#pragma unroll
  for (int i = 0; i <= NIN; ++i) acc[i] = 0.f;
#pragma unroll
  for (int it = 0; it < BT_E / 64; ++it) {
    const int el = lane + 64 * it;
    const float d = hv[it] > 0.f ? dv[it] : 0.f;
    if (el < nrow) {
#pragma unroll
      for (int i = 0; i < NIN; ++i) acc[i] = fmaf(d, ps[el * NIN + i], acc[i]);
    }
    acc[NIN] += d;
  }
#pragma unroll
  for (int i = 0; i <= NIN; ++i)
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) acc[i] += __shfl_xor(acc[i], o, 64);
  if (lane <= NIN) {
    float v = acc[0];
#pragma unroll
    for (int i = 1; i <= NIN; ++i) v = lane == i ? acc[i] : v;
    part[((int64_t)eb * C + k) * (NIN + 1) + lane] = v;
  }
}

// (k, i) per thread: the e-block partials summed in block order
__global__ void __launch_bounds__(256) encoder_bwd_t_final(const float* __restrict__ part, int neb, int C,
                                                           float* __restrict__ dw1, float* __restrict__ db1) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= C * (NIN + 1)) return;
  float s = 0.f;
  for (int b = 0; b < neb; ++b) s += part[(int64_t)b * C * (NIN + 1) + t];
  const int k = t / (NIN + 1), i = t - k * (NIN + 1);
  if (i < NIN) {
    if (dw1 != nullptr) dw1[(int64_t)k * NIN + i] = s;
  } else if (db1 != nullptr) {
    db1[k] = s;
  }
}

// dpose[e][i] = sum_k dpre[k][e] w1[k][i] (the pose gradient, models.py:146's input; K = C, 9 outputs per
// edge).  Block (64-edge block, k slice s): wave w walks k = k0 + w, k0 + w + 4, ... of the slice, one
// edge per lane (dh^T / h^T rows read 64 floats at a time, coalesced; w1's row uniform across the wave);
// the 4 waves' sums meet in LDS in wave order, then either straight into dpose (one slice) or into
// part[s][e][9], summed over the slices in order by encoder_bwd_pose_final: deterministic.
__global__ void __launch_bounds__(256) encoder_bwd_pose(const float* __restrict__ dhT, int64_t dhs,
                                                        const float* __restrict__ hT, int64_t hs,
                                                        const float* __restrict__ w1, int E, int C, int kslice,
                                                        float* __restrict__ out) {
  __shared__ float red[4][64][NIN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + lane;
  const int k0 = blockIdx.y * kslice, k1 = min(C, k0 + kslice);
  float acc[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) acc[i] = 0.f;
  if (e < E) {
#pragma unroll 4
    for (int k = k0 + w; k < k1; k += 4) {
      const float h = hT[(int64_t)k * hs + e], g = dhT[(int64_t)k * dhs + e];
      const float d = h > 0.f ? g : 0.f;
#pragma unroll
      for (int i = 0; i < NIN; ++i) acc[i] = fmaf(d, w1[k * NIN + i], acc[i]);
    }
  }
#pragma unroll
  for (int i = 0; i < NIN; ++i) red[w][lane][i] = acc[i];
  __syncthreads();
  for (int t = threadIdx.x; t < 64 * NIN; t += 256) {
    const int el = t / NIN, i = t - el * NIN, ee = blockIdx.x * 64 + el;
    if (ee < E)
      out[((int64_t)blockIdx.y * E + ee) * NIN + i] = ((red[0][el][i] + red[1][el][i]) + red[2][el][i]) + red[3][el][i];
  }
}

__global__ void __launch_bounds__(256) encoder_bwd_pose_final(const float* __restrict__ part, int ns, int64_t n,
                                                              float* __restrict__ dpose) {
  const int64_t t = blockIdx.x * (int64_t)256 + threadIdx.x;
  if (t >= n) return;
  float s = part[t];
  for (int b = 1; b < ns; ++b) s += part[(int64_t)b * n + t];
  dpose[t] = s;
}

// k slices of encoder_bwd_pose: enough blocks to cover the chip (>= 1024 with 64-edge blocks), each
// wave keeping >= 16 k terms; a multiple of 4 so every wave's k walk starts on its own residue
inline int pose_slices(int E, int C, int* kslice) {
  const int neb = (E + 63) / 64;
  int s = (1024 + neb - 1) / neb;
  s = std::max(1, std::min(s, C / 64));
  int ks = (C + s - 1) / s;
  ks = (ks + 3) / 4 * 4;
  s = (C + ks - 1) / ks;
  *kslice = ks;
  return s;
}

}  // namespace mrp_enc

extern "C" int64_t mrp_edge_encoder_bwd_pose_workspace(int32_t num_edges, int32_t C) {
  if (num_edges <= 0 || C <= 0) return 0;
  int ks;
  const int s = mrp_enc::pose_slices(num_edges, C, &ks);
  return s > 1 ? (int64_t)s * num_edges * mrp_enc::NIN * 4 : 0;
}

extern "C" int mrp_edge_encoder_bwd_pose(const float* dhT, int64_t dhT_stride, const float* hT, int64_t hT_stride,
                                         const float* w1, int32_t num_edges, int32_t C, float* dpose,
                                         void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0) return hipSuccess;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!dpose) return hipErrorInvalidValue;
  if (C == 0) return hipMemsetAsync(dpose, 0, (size_t)num_edges * mrp_enc::NIN * 4, st);
  if (!dhT || !hT || !w1 || dhT_stride < num_edges || hT_stride < num_edges ||
      (int64_t)C * mrp_enc::NIN >= ((int64_t)1 << 31))
    return hipErrorInvalidValue;
  int ks;
  const int s = mrp_enc::pose_slices(num_edges, C, &ks);
  if (s > 1 && (!workspace || workspace_bytes < mrp_edge_encoder_bwd_pose_workspace(num_edges, C)))
    return hipErrorInvalidValue;
  float* out = s > 1 ? static_cast<float*>(workspace) : dpose;
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_pose, dim3((num_edges + 63) / 64, s), dim3(256), 0, st, dhT, dhT_stride,
                     hT, hT_stride, w1, num_edges, C, ks, out);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || s == 1) return e;
  const int64_t n = (int64_t)num_edges * mrp_enc::NIN;
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_pose_final, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, out, s, n,
                     dpose);
  return hipGetLastError();
}

extern "C" int mrp_edge_encoder_bwd_prep(const float* dz, int32_t num_edges, int32_t C, float* dzT,
                                         int64_t dzT_stride, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  const int N2 = 2 * C;
  if (!dz || !dzT || dzT_stride < num_edges) return hipErrorInvalidValue;
  if (num_edges % 4 != 0 || N2 % 4 != 0 || dzT_stride % 4 != 0 || (reinterpret_cast<uintptr_t>(dz) & 15) ||
      (reinterpret_cast<uintptr_t>(dzT) & 15))
    return hipErrorNotSupported;
  hipLaunchKernelGGL(mrp_enc::dz_transpose, dim3((N2 + 63) / 64, (num_edges + 63) / 64), dim3(256), 0,
                     static_cast<hipStream_t>(stream), dz, num_edges, N2, dzT, dzT_stride);
  return hipGetLastError();
}

extern "C" int64_t mrp_edge_encoder_bwd_t_workspace(int32_t num_edges, int32_t C) {
  if (num_edges <= 0 || C <= 0) return 0;
  return (int64_t)((num_edges + mrp_enc::BT_E - 1) / mrp_enc::BT_E) * C * (mrp_enc::NIN + 1) * 4;
}

extern "C" int mrp_edge_encoder_bwd_t(const float* dhT, int64_t dhT_stride, const float* hT, int64_t hT_stride,
                                      const float* pose, int32_t num_edges, int32_t C, float* dw1, float* db1,
                                      void* workspace, int64_t workspace_bytes, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (C == 0 || (dw1 == nullptr && db1 == nullptr)) return hipSuccess;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (num_edges == 0) {  // empty sums
    if (dw1 && hipMemsetAsync(dw1, 0, (size_t)C * mrp_enc::NIN * 4, st) != hipSuccess) return hipErrorUnknown;
    if (db1 && hipMemsetAsync(db1, 0, (size_t)C * 4, st) != hipSuccess) return hipErrorUnknown;
    return hipSuccess;
  }
  if (!dhT || !hT || !pose || dhT_stride < num_edges || hT_stride < num_edges || !workspace ||
      workspace_bytes < mrp_edge_encoder_bwd_t_workspace(num_edges, C))
    return hipErrorInvalidValue;
  const int neb = (num_edges + mrp_enc::BT_E - 1) / mrp_enc::BT_E;
  float* part = static_cast<float*>(workspace);
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_t, dim3((C + 3) / 4, neb), dim3(256), 0, st, dhT, dhT_stride, hT,
                     hT_stride, pose, num_edges, C, part);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(mrp_enc::encoder_bwd_t_final, dim3((C * (mrp_enc::NIN + 1) + 255) / 256), dim3(256), 0, st, part, neb, C,
                     dw1, db1);
  return hipGetLastError();
}
