// edge_encoder.hip — fused FiLM parameter generator for gfx950 (MI355X / CDNA4).
//
// Replaces edge_encoder.forward, dgl/model/models.py:146-154:
//     Linear(9, C) -> ReLU -> Linear(C, 2C) -> Sigmoid      (then .view(E, C, 2))
// as ONE kernel: out[e, n] = sigmoid(b2[n] + sum_k W2[n, k] * relu(b1[k] + sum_i pose[e, i] W1[k, i]))
// The (E, 2C) result is exactly the interleaved (E, C, 2) gamma/beta tensor the aggregation reads.
//
// The second Linear is the only dense contraction (M = E edges, N = 2C, K = C): it runs on the fp32
// MFMA (v_mfma_f32_16x16x4_f32: exact fp32, an fma chain in k order).  The hidden activations are
// never written to HBM: each K-chunk of h (BM edges x BK) is computed into LDS from the staged pose
// rows and W1/b1 chunk, then consumed by the MFMAs.
//
// Tiling: workgroup = BM = 32 edges x BN = 64 outputs, 4 waves as 2 (rows) x 2 (cols); a wave owns
// 16 x 32 = two 16x16 accumulators.  K advances in chunks of BK = 32 (8 MFMA k-steps of 4).
// LDS rows are padded by one float (stride 33) so the MFMA operand reads (16 rows x 4 k per
// instruction) are bank-conflict free.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrp_gnn.h"

namespace mrp_enc {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int BM = 32;
constexpr int BN = 64;
constexpr int BK = 32;
constexpr int LDK = BK + 1;  // padded LDS row (floats)
constexpr int NIN = 9;       // relative pose width (dgl/utils.py:77)

__global__ void __launch_bounds__(256) edge_encoder_fwd(const float* __restrict__ pose, const float* __restrict__ w1,
                                                        const float* __restrict__ b1, const float* __restrict__ w2,
                                                        const float* __restrict__ b2, float* __restrict__ out, int E,
                                                        int C) {
  __shared__ float ps[BM][NIN + 1];   // pose rows of this tile
  __shared__ float w1s[BK][NIN + 1];  // W1 rows of the K-chunk + b1 in column NIN
  __shared__ float hs[BM][LDK];       // h chunk: rows = edges, cols = k
  __shared__ float ws[BN][LDK];       // W2 chunk: rows = outputs n, cols = k

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1;  // 16-row half of the 32-edge tile
  const int wc = wave & 1;   // 32-column half of the 64-output tile
  const int N2 = 2 * C;
  const int e0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;

  for (int t = tid; t < BM * NIN; t += 256) {
    const int m = t / NIN, i = t - m * NIN;
    ps[m][i] = (e0 + m < E) ? pose[(int64_t)(e0 + m) * NIN + i] : 0.f;
  }

  f4 acc[2];
  acc[0] = f4{0.f, 0.f, 0.f, 0.f};
  acc[1] = f4{0.f, 0.f, 0.f, 0.f};

  for (int k0 = 0; k0 < C; k0 += BK) {
    __syncthreads();  // previous chunk's hs/ws fully consumed (and ps staged, first time)
    // W1/b1 rows of this chunk
    for (int t = tid; t < BK * (NIN + 1); t += 256) {
      const int r = t / (NIN + 1), i = t - r * (NIN + 1);
      const int k = k0 + r;
      float v = 0.f;
      if (k < C) v = (i < NIN) ? w1[(int64_t)k * NIN + i] : b1[k];
      w1s[r][i] = v;
    }
    // W2 chunk: thread -> (row n = tid / 4, 8 consecutive k); two 16-byte loads when aligned
    {
      const int r = tid >> 2;
      const int kk = (tid & 3) * 8;
      const int n = n0 + r;
      float v[8];
      if (n < N2 && k0 + kk + 8 <= C && (C & 3) == 0) {
        const f4* src = reinterpret_cast<const f4*>(w2 + (int64_t)n * C + k0 + kk);
        const f4 a = src[0], b = src[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = k0 + kk + i;
          v[i] = (n < N2 && k < C) ? w2[(int64_t)n * C + k] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ws[r][kk + i] = v[i];
    }
    __syncthreads();  // w1s, ps visible
    // h chunk: thread -> (edge m = tid / 8, 4 consecutive k)
    {
      const int m = tid >> 3;
      const int kk = (tid & 7) * 4;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = kk + i;
        float h = w1s[r][NIN];  // b1 first, then the 9 products in order (torch addmm adds bias to the
#pragma unroll                  // product; any order is within fp32 rounding of the reference)
        for (int q = 0; q < NIN; ++q) h = fmaf(ps[m][q], w1s[r][q], h);
        hs[m][r] = h > 0.f ? h : 0.f;  // ReLU
      }
    }
    __syncthreads();  // hs, ws visible
    // 8 MFMA k-steps of 4: A[i][k] = hs[16*wr + (lane&15)][k], B[k][j] = ws[32*wc + 16*t + (lane&15)][k]
#pragma unroll
    for (int ks = 0; ks < BK; ks += 4) {
      const int k = ks + (lane >> 4);
      const float a = hs[wr * 16 + (lane & 15)][k];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const float b = ws[wc * 32 + t * 16 + (lane & 15)][k];
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
      }
    }
  }

  // Epilogue: D[row = 4*(lane>>4) + r][col = lane&15] of each 16x16 tile; bias + sigmoid.
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int n = n0 + wc * 32 + t * 16 + (lane & 15);
    if (n >= N2) continue;
    const float bias = b2[n];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = e0 + wr * 16 + (lane >> 4) * 4 + r;
      if (e >= E) continue;
      const float z = acc[t][r] + bias;
      out[(int64_t)e * N2 + n] = 1.f / (1.f + expf(-z));
    }
  }
}

}  // namespace mrp_enc

extern "C" int mrp_edge_encoder_fwd(const float* pose, const float* w1, const float* b1, const float* w2,
                                    const float* b2, int32_t num_edges, int32_t C, float* out, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (!pose || !w1 || !b1 || !w2 || !b2 || !out) return hipErrorInvalidValue;
  const int64_t gx = (2 * (int64_t)C + mrp_enc::BN - 1) / mrp_enc::BN;
  const int64_t gy = ((int64_t)num_edges + mrp_enc::BM - 1) / mrp_enc::BM;
  if (gx > 0x7fffffff || gy > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(mrp_enc::edge_encoder_fwd, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0,
                     static_cast<hipStream_t>(stream), pose, w1, b1, w2, b2, out, num_edges, C);
  return hipGetLastError();
}
