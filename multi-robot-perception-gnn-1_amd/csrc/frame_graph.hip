// frame_graph.hip — per-frame robot graphs built on the GPU (gfx950 / MI355X).
//
// Replaces the host-side graph construction of the reference's dataset path:
//   edge list   dgl/dataloader.py:88-95   every ordered pair i != j, i-major
//   edge feature dgl/dataloader.py:116-122 cal_relative_pose(pose_i, pose_j) per edge
//   relative pose dgl/utils.py:54-77     [t_j - t_i, first two columns of R(conj(q_i) q_j)]
// plus the k-NN(k) topology of the BASELINE configs (the reference builds complete graphs only):
// each destination v takes the k robots u != v nearest to it, |t_u - t_v| in float64 with ties to
// the lower index, listed in ascending u (the host builder `graph.knn_edges` in device form).
//
// One thread per (graph, destination robot): it selects v's in-edges, writes their relative poses,
// its CSR row (indptr, src, eid) and, for v == 0, its graph's node offset.  Work per batch is a few
// hundred threads: the point is to keep the per-batch host work (numpy loops, a host-to-device copy
// of the edge features) off the training step, not bandwidth.
//
// Arithmetic follows the reference's float32 numpy expression order exactly (compiled with
// -ffp-contract=off, no FMA contraction), so edge poses are bit-identical to the host path
// (`pose.relative_pose_batch` on float32 rows, itself pinned to the reference's own outputs).

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mrp_gnn.h"

namespace mrp_graph {

constexpr int kThreads = 128;

// cal_relative_pose(p1 = source, p2 = destination), dgl/utils.py:69-77, float32.
__device__ __forceinline__ void relative_pose(const float* p1, const float* p2, float* out) {
  const float x1 = -p1[3], y1 = -p1[4], z1 = -p1[5], w1 = p1[6];  // conjugate of q1
  const float x2 = p2[3], y2 = p2[4], z2 = p2[5], w2 = p2[6];
  // q2 * q1^-1 in the reference's expansion, evaluated left to right
  const float x = __fsub_rn(__fadd_rn(__fadd_rn(__fmul_rn(w1, x2), __fmul_rn(x1, w2)), __fmul_rn(y1, z2)),
                            __fmul_rn(z1, y2));
  const float y = __fadd_rn(__fadd_rn(__fsub_rn(__fmul_rn(w1, y2), __fmul_rn(x1, z2)), __fmul_rn(y1, w2)),
                            __fmul_rn(z1, x2));
  const float z = __fadd_rn(__fsub_rn(__fadd_rn(__fmul_rn(w1, z2), __fmul_rn(x1, y2)), __fmul_rn(y1, x2)),
                            __fmul_rn(z1, w2));
  const float w = __fsub_rn(__fsub_rn(__fsub_rn(__fmul_rn(w1, w2), __fmul_rn(x1, x2)), __fmul_rn(y1, y2)),
                            __fmul_rn(z1, z2));
  out[0] = __fsub_rn(p2[0], p1[0]);
  out[1] = __fsub_rn(p2[1], p1[1]);
  out[2] = __fsub_rn(p2[2], p1[2]);
  // quat_to_so3 (dgl/utils.py:54-66), first six entries: a00 a10 a20 a01 a11 a21
  const float yy = __fmul_rn(y, y), zz = __fmul_rn(z, z), xx = __fmul_rn(x, x);
  out[3] = __fsub_rn(__fsub_rn(1.f, __fmul_rn(2.f, yy)), __fmul_rn(2.f, zz));
  out[4] = __fadd_rn(__fmul_rn(__fmul_rn(2.f, x), y), __fmul_rn(__fmul_rn(2.f, z), w));
  out[5] = __fsub_rn(__fmul_rn(__fmul_rn(2.f, x), z), __fmul_rn(__fmul_rn(2.f, y), w));
  out[6] = __fsub_rn(__fmul_rn(__fmul_rn(2.f, x), y), __fmul_rn(__fmul_rn(2.f, z), w));
  out[7] = __fsub_rn(__fsub_rn(1.f, __fmul_rn(2.f, xx)), __fmul_rn(2.f, zz));
  out[8] = __fadd_rn(__fmul_rn(__fmul_rn(2.f, y), z), __fmul_rn(__fmul_rn(2.f, x), w));
}

__device__ __forceinline__ void write_pose(float* edge_pose, int64_t e, const float* p) {
  if (edge_pose == nullptr) return;
#pragma unroll
  for (int i = 0; i < 9; ++i) edge_pose[e * 9 + i] = p[i];
}

__global__ void __launch_bounds__(kThreads) frame_graph_build(const float* __restrict__ poses, int B, int n, int k,
                                                             float* __restrict__ edge_pose, int32_t* __restrict__ indptr,
                                                             int32_t* __restrict__ src, int32_t* __restrict__ eid,
                                                             int32_t* __restrict__ goff) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nt = (int64_t)B * n;
  if (t >= nt) return;
  const int b = (int)(t / n);
  const int v = (int)(t - (int64_t)b * n);
  const int64_t node0 = (int64_t)b * n;
  const float* pv = poses + t * 7;
  if (goff != nullptr && v == 0) {
    goff[b] = (int32_t)node0;
    if (b == B - 1) goff[B] = (int32_t)nt;
  }
  float rel[9];
  if (k == 0) {
    // complete graph: in-edges of v are u = 0..n-1, u != v, at edge id b*n(n-1) + u(n-1) + (v<u ? v : v-1)
    const int64_t ebase = (int64_t)b * n * (n - 1);
    const int64_t row = ebase + (int64_t)v * (n - 1);  // CSR row start = v's rank among destinations
    if (indptr != nullptr) {
      indptr[t] = (int32_t)row;
      if (t == nt - 1) indptr[nt] = (int32_t)(nt * (n - 1));
    }
    int j = 0;
    for (int u = 0; u < n; ++u) {
      if (u == v) continue;
      const int64_t e = ebase + (int64_t)u * (n - 1) + (v < u ? v : v - 1);
      relative_pose(poses + (node0 + u) * 7, pv, rel);
      write_pose(edge_pose, e, rel);
      if (src != nullptr) src[row + j] = (int32_t)(node0 + u);
      if (eid != nullptr) eid[row + j] = (int32_t)e;
      ++j;
    }
    return;
  }
  // k-NN: k nearest sources by float64 Euclidean distance of the translations (numpy's
  // norm: sqrt((dx^2 + dy^2) + dz^2)), ties to the lower index
  double d[MRP_MAX_NODES];
  const double tvx = pv[0], tvy = pv[1], tvz = pv[2];
  for (int u = 0; u < n; ++u) {
    const float* pu = poses + (node0 + u) * 7;
    const double dx = __dsub_rn((double)pu[0], tvx);
    const double dy = __dsub_rn((double)pu[1], tvy);
    const double dz = __dsub_rn((double)pu[2], tvz);
    d[u] = __dsqrt_rn(__dadd_rn(__dadd_rn(__dmul_rn(dx, dx), __dmul_rn(dy, dy)), __dmul_rn(dz, dz)));
  }
  unsigned chosen = 0u;
  for (int j = 0; j < k; ++j) {
    int best = -1;
    for (int u = 0; u < n; ++u) {
      if (u == v || ((chosen >> u) & 1u)) continue;
      if (best < 0 || d[u] < d[best]) best = u;  // strict: equal distance keeps the lower index
    }
    chosen |= 1u << best;
  }
  const int64_t row = t * k;
  if (indptr != nullptr) {
    indptr[t] = (int32_t)row;
    if (t == nt - 1) indptr[nt] = (int32_t)(nt * k);
  }
  int j = 0;
  for (int u = 0; u < n; ++u) {
    if (!((chosen >> u) & 1u)) continue;
    const int64_t e = row + j;  // edges are numbered destination-major, sources ascending
    relative_pose(poses + (node0 + u) * 7, pv, rel);
    write_pose(edge_pose, e, rel);
    if (src != nullptr) src[e] = (int32_t)(node0 + u);
    if (eid != nullptr) eid[e] = (int32_t)e;
    ++j;
  }
}

}  // namespace mrp_graph

extern "C" int mrp_frame_graph_build(const float* poses, int32_t num_graphs, int32_t n, int32_t knn_k,
                                     float* edge_pose, int32_t* indptr, int32_t* src, int32_t* eid,
                                     int32_t* graph_off, void* stream) {
  if (num_graphs < 0 || n < 0 || n > MRP_MAX_NODES || knn_k < 0) return hipErrorInvalidValue;
  if (knn_k > 0 && knn_k >= n) return hipErrorInvalidValue;  // k-NN needs k < n (knn_edges raises too)
  const int64_t nt = (int64_t)num_graphs * n;
  const int64_t ne = knn_k > 0 ? nt * knn_k : nt * (n > 0 ? n - 1 : 0);
  if (nt >= 0x7fffffff || ne >= 0x7fffffff) return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (nt == 0) {
    // no nodes: only the offsets (all zero) and the CSR terminator exist
    if (graph_off != nullptr && num_graphs >= 0) {
      hipError_t e = hipMemsetAsync(graph_off, 0, sizeof(int32_t) * ((size_t)num_graphs + 1), st);
      if (e != hipSuccess) return e;
    }
    if (indptr != nullptr) return hipMemsetAsync(indptr, 0, sizeof(int32_t), st);
    return hipSuccess;
  }
  if (poses == nullptr) return hipErrorInvalidValue;
  const unsigned blocks = (unsigned)((nt + mrp_graph::kThreads - 1) / mrp_graph::kThreads);
  hipLaunchKernelGGL(mrp_graph::frame_graph_build, dim3(blocks), dim3(mrp_graph::kThreads), 0, st, poses,
                     (int)num_graphs, (int)n, (int)knn_k, edge_pose, indptr, src, eid, graph_off);
  return hipGetLastError();
}
