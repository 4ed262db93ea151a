// lab_fp32_encoder.hip — kernel lab (not product code): round 3's one-launch fp32 edge encoder
// (mrp_edge_encoder_fwd, fp32 MFMA, W2 by LDS-DMA, the hidden layer computed into the A image), moved
// out of the product library in round 5: the split-bf16 one-launch encoder
// (encoder_split.hip, mrp_edge_encoder_fwd_split) replaced it at every shape (headline 16-17 us vs
// 21-23 us), and shapes it declines take mrp_edge_hidden_fwd + mrp_edge_logits_fwd.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/lab_fp32_encoder.hip
#include "../multi-robot-perception-gnn-1_amd/csrc/compress_gemm.hip"

// ------------------------------------------------------------------------------------------------
// The whole edge encoder before its Sigmoid in one kernel (dgl/model/models.py:146-149):
//     z = relu(pose W1^T + b1) W2^T + b2
// The hidden layer has K = 9, so its tile is computed, not loaded: per stage (32 hidden units) each
// wave evaluates 4-unit chunks of relu(pose W1^T + b1) for the tile's 64 edges (lane = edge row;
// W1 and b1 in LDS for the whole kernel, read as broadcasts) and writes them into the stage's A
// image in the swizzled layout LDS-DMA would produce, so the MFMA pipeline of the GEMMs above runs
// unchanged on it while W2 streams in by LDS-DMA.  h never reaches HBM: no second launch, no
// 4 E C bytes written and read back.  Same arithmetic as mrp_edge_hidden_fwd (acc = b1, fmaf over
// the 9 pose values in order, relu), so h is bit-identical to the two-kernel path.
// ------------------------------------------------------------------------------------------------
namespace mrp_cg {

template <int WN_, int NBUF_>
struct EncCfg : Cfg<32, 32, NBUF_, 2, WN_, 32> {
  using Base = Cfg<32, 32, NBUF_, 2, WN_, 32>;
  static constexpr int PA = 0;  // no LDS-DMA pieces for A: stage_barrier counts only B's
  static constexpr int CHW = Base::CPR / Base::NW;  // A-image chunks per wave per stage
  static_assert(Base::CPR % Base::NW == 0, "chunks must divide over the waves");
};

struct EncArgs {
  const float* pose;
  const float* w1;
  const float* b1;
  const float* w2;
  const float* b2;
  float* z;
  int32_t E, C, mtiles;
};

template <class G>
__global__ void __launch_bounds__(G::THREADS, 2) edge_encoder_fwd(EncArgs a) {
  using AC = Acc<G::MF>;
  constexpr int NIN = 9;
  extern __shared__ f4 smem4[];
  float* smemf = reinterpret_cast<float*>(smem4);
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = id % a.mtiles, nt = id / a.mtiles;
  const int mbase = mt * G::TM, nbase = nt * G::TN;
  const int N = 2 * a.C;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const int nst = a.C / G::BK;
  const __amdgpu_buffer_rsrc_t rb = rsrc(a.w2);
  uint32_t vb[G::PB];
#pragma unroll
  for (int jj = 0; jj < G::PB; ++jj) {
    const int row = G::RPP * (w + jj * G::NW) + lane / G::CPR;
    const int c = (lane % G::CPR) ^ swz_a<G::BK>(row);
    vb[jj] = (uint32_t)(((int64_t)min(nbase + row, N - 1) * a.C + 4 * c) * 4);
  }
  auto issue_b = [&](int stage, int buf) {
    const uint32_t sk = (uint32_t)stage * G::BK * 4;
#pragma unroll
    for (int jj = 0; jj < G::PB; ++jj)
      dma16(rb, &smem4[(buf * G::BUF + G::A_FLOATS + (w + jj * G::NW) * 256) / 4], vb[jj], sk);
  };
  // W2 for the first stages is requested before anything else: its latency overlaps the staging of
  // W1 and the pose rows
#pragma unroll
  for (int s = 0; s < G::NBUF; ++s)
    if (s < nst) issue_b(s, s);

  // W1 (C x 9, as stored) and b1 after the stage buffers, for the whole K loop
  float* w1s = smemf + G::NBUF * G::BUF;
  float* b1s = w1s + a.C * NIN;
  for (int i = threadIdx.x; i < a.C * NIN / 4; i += G::THREADS)
    reinterpret_cast<f4*>(w1s)[i] = reinterpret_cast<const f4*>(a.w1)[i];
  for (int i = threadIdx.x; i < a.C / 4; i += G::THREADS)
    reinterpret_cast<f4*>(b1s)[i] = reinterpret_cast<const f4*>(a.b1)[i];
  // the lane's edge (row of the A tile) for every chunk it computes
  float p[NIN];
  {
    const int e = min(mbase + lane, a.E - 1);
#pragma unroll
    for (int i = 0; i < NIN; ++i) p[i] = a.pose[(int64_t)e * NIN + i];
  }
  __syncthreads();

  auto issue_a = [&](int stage, int buf) {
    float* As = smemf + buf * G::BUF;
#pragma unroll
    for (int jj = 0; jj < G::CHW; ++jj) {
      const int c = w + jj * G::NW;
      const int u0 = stage * G::BK + 4 * c;
      float wr[4 * NIN];
#pragma unroll
      for (int q = 0; q < NIN; ++q) {
        const f4 v = *reinterpret_cast<const f4*>(w1s + u0 * NIN + 4 * q);
        wr[4 * q] = v.x, wr[4 * q + 1] = v.y, wr[4 * q + 2] = v.z, wr[4 * q + 3] = v.w;
      }
      const f4 bv = *reinterpret_cast<const f4*>(b1s + u0);
      f4 hv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float acc = bv[j];
#pragma unroll
        for (int i = 0; i < NIN; ++i) acc = fmaf(p[i], wr[NIN * j + i], acc);
        hv[j] = acc > 0.f ? acc : 0.f;
      }
      *reinterpret_cast<f4*>(As + lane * G::BK + 4 * (c ^ swz_a<G::BK>(lane))) = hv;
    }
  };
#pragma unroll
  for (int s = 0; s < G::NBUF; ++s)
    if (s < nst) issue_a(s, s);
  auto issue = [&](int stage, int buf) {
    issue_b(stage, buf);
    issue_a(stage, buf);
  };

  const int wm = w / G::WN, wn = w % G::WN;
  int aoff[G::BK / 16][G::CH], boff[G::BK / 16][G::CH];
  a_offsets<G>(wm * G::WT, lane, aoff);
  a_offsets<G>(wn * G::WT, lane, boff);
  typename AC::T acc[G::FB][G::FB];
#pragma unroll
  for (int mb = 0; mb < G::FB; ++mb)
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb)
#pragma unroll
      for (int r = 0; r < AC::R; ++r) acc[mb][nb][r] = 0.f;
  const float* smem = smemf;
  auto read = [&](int buf, int g, float (&fr)[2][G::FB][G::T]) {
    const float* As = smem + buf * G::BUF;
    const float* Bs = As + G::A_FLOATS;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb) read_a<G>(As, aoff, g, mb, fr[0][mb]);
#pragma unroll
    for (int nb = 0; nb < G::FB; ++nb) read_a<G>(Bs, boff, g, nb, fr[1][nb]);
  };
  auto mma = [&](const float (&fr)[2][G::FB][G::T]) { mma_group<G>(acc, fr[0], fr[1]); };
  kloop<G, true>(nst, issue, read, mma);

#pragma unroll
  for (int nb = 0; nb < G::FB; ++nb) {
    const int col = nbase + wn * G::WT + nb * G::MF + AC::col(lane);
    if (col >= N) continue;
    const float bias = a.b2 ? a.b2[col] : 0.f;
#pragma unroll
    for (int mb = 0; mb < G::FB; ++mb)
#pragma unroll
      for (int r = 0; r < AC::R; ++r) {
        const int row = mbase + wm * G::WT + mb * G::MF + AC::row(lane, r);
        if (row < a.E) a.z[(int64_t)row * N + col] = __fadd_rn(acc[mb][nb][r], bias);
      }
  }
}

template <class G>
hipError_t launch_enc(EncArgs a, hipStream_t st) {
  const size_t lds = (size_t)G::NBUF * G::BUF * 4 + (size_t)a.C * 10 * 4;
  if (lds > 160 * 1024) return hipErrorNotSupported;
  a.mtiles = (a.E + G::TM - 1) / G::TM;
  const int64_t grid = (int64_t)a.mtiles * ((2 * (int64_t)a.C + G::TN - 1) / G::TN);
  if (grid > 0x7fffffff) return hipErrorInvalidValue;
  static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(&edge_encoder_fwd<G>),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr != hipSuccess) return attr;
  hipLaunchKernelGGL(edge_encoder_fwd<G>, dim3((unsigned)grid), dim3(G::THREADS), lds, st, a);
  return hipGetLastError();
}

// variants (mrp_tuning_set "edge_fused"): 64 x (32 WN) tiles, NBUF stage buffers
#define MRP_ENC_VARIANTS(X) \
  X(0, (EncCfg<2, 2>)) X(1, (EncCfg<2, 3>)) X(2, (EncCfg<4, 2>)) X(3, (EncCfg<4, 3>)) X(4, (EncCfg<4, 4>))

}  // namespace mrp_cg

int lab_edge_fused = 2;  // the variant (was mrp_tuning_set "edge_fused"; 2 was the product default)

extern "C" int mrp_edge_encoder_fwd(const float* pose, const float* w1, const float* b1, const float* w2,
                                    const float* b2, int32_t num_edges, int32_t C, float* z, void* stream) {
  if (num_edges < 0 || C < 0) return hipErrorInvalidValue;
  if (num_edges == 0 || C == 0) return hipSuccess;
  if (!pose || !w1 || !b1 || !w2 || !z) return hipErrorInvalidValue;
  if (C % 32 != 0 || !aligned16(w1) || !aligned16(b1) || !aligned16(w2)) return hipErrorNotSupported;
  if ((int64_t)2 * C * C * 4 >= kOffMax) return hipErrorNotSupported;
  EncArgs a = {pose, w1, b1, w2, b2, z, num_edges, C, 0};
  hipStream_t st = static_cast<hipStream_t>(stream);
  switch (lab_edge_fused) {
#define MRP_ENC_CASE(i, C) \
  case i:                  \
    return launch_enc<MRP_UNPAREN C>(a, st);
#define MRP_UNPAREN(...) __VA_ARGS__
    MRP_ENC_VARIANTS(MRP_ENC_CASE)
#undef MRP_ENC_CASE
#undef MRP_UNPAREN
    default:
      return hipErrorInvalidValue;
  }
}
