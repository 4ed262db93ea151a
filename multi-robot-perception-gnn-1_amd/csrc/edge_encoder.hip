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

// One thread per (edge, 4 consecutive hidden units): the edge's 9 pose values are a broadcast
// load shared by the C/4 threads of the edge; W1 rows are L1/L2-resident.
__global__ void __launch_bounds__(256) edge_hidden_fwd(const float* __restrict__ pose, const float* __restrict__ w1,
                                                       const float* __restrict__ b1, float* __restrict__ h, int E,
                                                       int C) {
  const int64_t cq = ((int64_t)C + 3) / 4;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)E * cq) return;
  const int64_t e = idx / cq;
  const int k0 = (int)(idx - e * cq) * 4;
  float p[NIN];
#pragma unroll
  for (int i = 0; i < NIN; ++i) p[i] = pose[e * NIN + i];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int k = k0 + q;
    if (k >= C) break;
    float acc = b1[k];
#pragma unroll
    for (int i = 0; i < NIN; ++i) acc = fmaf(p[i], w1[(int64_t)k * NIN + i], acc);
    h[e * C + k] = acc > 0.f ? acc : 0.f;
  }
}

}  // namespace mrp_enc

extern "C" int mrp_edge_hidden_fwd(const float* pose, const float* w1, const float* b1, int32_t num_edges,
                                   int32_t C, float* h, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (!pose || !w1 || !b1 || !h) return hipErrorInvalidValue;
  const int64_t threads = (int64_t)num_edges * ((C + 3) / 4);
  const int64_t blocks = (threads + 255) / 256;
  if (blocks > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mrp_enc::edge_hidden_fwd, dim3((unsigned)blocks), dim3(256), 0,
                     static_cast<hipStream_t>(stream), pose, w1, b1, h, num_edges, C);
  return hipGetLastError();
}
