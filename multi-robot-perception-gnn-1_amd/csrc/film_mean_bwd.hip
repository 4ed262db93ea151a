// film_mean_bwd.hip — backward C ABI (mrp_film_mean_bwd).  The kernel launches are instantiated
// in film_mean_bwd_{1_8,9_12,13_16}.hip (split by graph size so they compile in parallel);
// kernels and design notes: film_mean_kernels.hpp.
#include "film_mean_kernels.hpp"

using namespace mrp_host;

namespace {

// Geometry of film_bwd_regular (N > 8, uniform in-degree k <= 8) for slice width vec.
Geometry regular_geometry(int C, int P, int vec) {
  const Tuning& tu = tuning();
  return vec == 2 ? make_geometry(C, P, 2, tu.bwd_regular_lanes, tu.bwd_regular_lanes, mrp::kMaxChanPerBlock)
                  : make_geometry(C, P, 1, 2 * tu.bwd_regular_lanes, 2 * tu.bwd_regular_lanes, mrp::kMaxChanPerBlock);
}

hipError_t dispatch_bwd(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st) {
  if (nt >= 1 && nt <= 8) return dispatch_bwd_1_8(nt, complete, a, g, st);
  if (nt >= 9 && nt <= 12) return dispatch_bwd_9_12(nt, complete, a, g, st);
  if (nt >= 13 && nt <= 16) return dispatch_bwd_13_16(nt, complete, a, g, st);
  return hipErrorInvalidValue;
}

}  // namespace

extern "C" {

int mrp_film_mean_bwd(const float* grad_out, int64_t g_node_stride, const float* x, int64_t x_node_stride,
                      const float* gb, const int32_t* indptr, const int32_t* src, const int32_t* eid,
                      const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes, int32_t graph_kind,
                      int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P, int32_t mode_flags, float* grad_x,
                      int64_t gx_node_stride, const float* grad_x_base, int64_t base_node_stride, float* grad_gb,
                      void* stream) {
  return mrp_film_mean_bwd_ex(grad_out, g_node_stride, x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs,
                              max_nodes, graph_kind, num_nodes, num_edges, C, P, mode_flags, grad_x, gx_node_stride,
                              grad_x_base, base_node_stride, grad_gb, nullptr, nullptr, 0, stream);
}

// No backward kernel of this library version needs scratch (the plane-split k-NN backward that used
// it measured slower and is gone, round 3); kept so callers written against the workspace
// contract keep working.
int64_t mrp_film_mean_bwd_workspace(int32_t, int32_t, int32_t, int32_t, int32_t) { return 0; }

int mrp_film_mean_bwd_ex(const float* grad_out, int64_t g_node_stride, const float* x, int64_t x_node_stride,
                         const float* gb, const int32_t* indptr, const int32_t* src, const int32_t* eid,
                         const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes, int32_t graph_kind,
                         int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P, int32_t mode_flags,
                         float* grad_x, int64_t gx_node_stride, const float* grad_x_base, int64_t base_node_stride,
                         float* grad_gb, const mrp_agg_epilogue* ep, void* workspace, int64_t workspace_bytes,
                         void* stream) {
  const float agg_scale = ep != nullptr ? ep->agg_scale : 1.f;
  const float self_scale = ep != nullptr ? ep->self_scale : 0.f;
  const int32_t logits = (mode_flags & MRP_AGG_GB_LOGITS) ? 1 : 0;
  const int32_t mode = mode_flags & ~MRP_AGG_GB_LOGITS;
  if (!common_args_ok(indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind, num_nodes, num_edges, C, P,
                      mode))
    return hipErrorInvalidValue;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool copy = mode == MRP_AGG_COPY_MEAN;
  if (grad_gb != nullptr && num_edges > 0 && C > 0 && (copy || num_nodes == 0 || P == 0 || agg_scale == 0.f)) {
    // gamma/beta do not influence the output: their gradient is zero.
    hipError_t e = hipMemsetAsync(grad_gb, 0, (size_t)num_edges * C * 2 * sizeof(float), st);
    if (e != hipSuccess) return e;
  }
  const bool want_dgb = grad_gb != nullptr && !copy && num_edges > 0 && agg_scale != 0.f;
  const bool want_dx = grad_x != nullptr;
  if (!want_dgb && !want_dx) return hipSuccess;
  if (num_graphs == 0 || num_nodes == 0 || max_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (grad_out == nullptr || g_node_stride < plane) return hipErrorInvalidValue;
  if (want_dx && gx_node_stride < plane) return hipErrorInvalidValue;
  if (want_dx && grad_x_base != nullptr && base_node_stride < plane) return hipErrorInvalidValue;
  if (want_dgb && (x == nullptr || x_node_stride < plane)) return hipErrorInvalidValue;
  if (!copy && num_edges > 0 && gb == nullptr) return hipErrorInvalidValue;
  bool vec4 = (P % 4 == 0) && (g_node_stride % 4 == 0) && aligned16(grad_out);
  if (want_dx) vec4 = vec4 && (gx_node_stride % 4 == 0) && aligned16(grad_x);
  if (want_dx && grad_x_base) vec4 = vec4 && (base_node_stride % 4 == 0) && aligned16(grad_x_base);
  if (want_dgb) vec4 = vec4 && (x_node_stride % 4 == 0) && aligned16(x);
  // 16-byte slices: with the DPP lane reduction they beat 8-byte slices (310 vs 322 us at B=32,
  // N=8, C=512, 32x32) despite 2 waves/SIMD instead of 3.  VEC=2 stays compiled for experiments.
  int vec = vec4 ? 4 : 1;
  Geometry g;
  const int kdeg = MRP_GRAPH_IS_REGULAR(graph_kind) ? MRP_GRAPH_REGULAR_K(graph_kind) : 0;
  if (max_nodes > 8 && kdeg >= 1 && kdeg <= 8) {
    // film_bwd_regular: 8-byte slices on 16 lanes per plane (367 us against 569 us on 64 lanes at
    // k-NN(4) N=16 C=1024 16x16): its prologue and lane reduction are amortised over more slices
    const Tuning& tu = tuning();
    vec = (vec4 && kdeg <= 4 && tu.bwd_regular_vec == 2) ? 2 : 1;
    g = regular_geometry(C, P, vec);
  } else if (max_nodes <= 8) {
    // film_bwd_fused: up to 128 lanes (two waves) per plane, two slices per lane: 283 vs 306 us at
    // 64 lanes at the bench size (tools/fwd_lab.hip backward sweep; 256 lanes: 297 us)
    const Tuning& tu = tuning();
    g = make_geometry(C, P, vec, tu.bwd_fused_lo, tu.bwd_fused_hi, tu.bwd_fused_cap);
  } else {
    g = make_geometry(C, P, vec, 64, 64, mrp::kMaxChanPerBlock);  // film_bwd_dx + Gram pass
  }
  (void)workspace;
  (void)workspace_bytes;
  // film_bwd_mfma: regular graphs of 9..16 nodes and complete graphs, whole pixel groups of 64
  const bool complete = graph_kind == MRP_GRAPH_COMPLETE;
  const bool mfma_kind = (max_nodes > 8 && kdeg >= 1 && kdeg <= 8 && tuning().bwd_regular_mfma) ||
                         (complete && max_nodes > 8 && tuning().bwd_complete_mfma);
  if (mfma_kind && vec4 && P % 64 == 0) {
    // per-lane row offsets are 32-bit: 15 node strides + two planes (a block's channel pair)
    const int64_t lim = (int64_t)1 << 32;
    const int64_t span = (int64_t)plane * 4 + (int64_t)P * 4;
    bool fits = (int64_t)15 * g_node_stride * 4 + span < lim;
    if (want_dx) fits = fits && (int64_t)15 * gx_node_stride * 4 + span < lim;
    if (want_dx && grad_x_base) fits = fits && (int64_t)15 * base_node_stride * 4 + span < lim;
    if (want_dgb) fits = fits && (int64_t)15 * x_node_stride * 4 + span < lim;
    if (fits) {
      const int cpw = tuning().bwd_mfma_cpw >= 2 ? 2 : 1;  // instantiated: 1, 2
      g.mfma_npb = 16;
      g.vec = 4;
      g.lpc = 64;
      g.cpb = 4 * cpw * (16 / g.mfma_npb);  // 4 waves x blocks per wave x channels per block
      g.threads = 256;
      g.ncb = (C + g.cpb - 1) / g.cpb;
    }
  }
  g.grid = (int64_t)num_graphs * g.ncb;
  if (g.grid > 0x7fffffff) return hipErrorInvalidValue;
  AggArgs a = {};
  a.x = x;
  a.xs = x_node_stride;
  a.g = grad_out;
  a.gs = g_node_stride;
  a.gb = gb;
  a.indptr = indptr;
  a.src = src;
  a.eid = eid;
  a.goff = graph_off;
  a.out = grad_x;
  a.os = gx_node_stride;
  a.dgb = grad_gb;
  a.C = C;
  a.P = P;
  a.PV = P / g.vec;
  a.mode = mode;
  a.lpc = g.lpc;
  a.cpb = g.cpb;
  a.ncb = g.ncb;
  a.want_dx = want_dx ? 1 : 0;
  a.want_dgb = want_dgb ? 1 : 0;
  a.logits = logits;
  a.dxb = want_dx ? grad_x_base : nullptr;
  a.dxbs = base_node_stride;
  a.kdeg = kdeg;
  a.agg_scale = agg_scale;
  a.self_scale = self_scale;
  a.epi = (agg_scale != 1.f || self_scale != 0.f) ? 1 : 0;
  a.psplit = 1;
  a.nmax = max_nodes;
  return dispatch_bwd(max_nodes, graph_kind == MRP_GRAPH_COMPLETE, a, g, st);
}

}  // extern "C"

