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
