// film_mean_fwd.hip — forward launchers and C ABI (mrp_film_mean_fwd, mrp_film_mean_cat_fwd).
// Kernels and design notes: film_mean_kernels.hpp.
#include "film_mean_kernels.hpp"

using namespace mrp_host;

namespace {

template <int NT, bool COMPLETE>
hipError_t launch_fwd_nt(const AggArgs& a, const Geometry& g, hipStream_t st) {
  const size_t lds = lds_fwd<NT>(g.cpb);
  if (g.vec == 4)
    MRP_LAUNCH((mrp::film_fwd<NT, 4, COMPLETE>), lds);
  else if (g.vec == 2)
    MRP_LAUNCH((mrp::film_fwd<NT, 2, COMPLETE>), lds);
  else if (g.vec == 1)
    MRP_LAUNCH((mrp::film_fwd<NT, 1, COMPLETE>), lds);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t dispatch_fwd(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st) {
  MRP_DISPATCH_NT(nt, complete, launch_fwd_nt, a, g, st)
}
}  // namespace

extern "C" {

int mrp_abi_version(void) { return 9; }

const char* mrp_error_string(int code) { return hipGetErrorString(static_cast<hipError_t>(code)); }

}  // extern "C"

namespace {

int film_fwd_impl(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr, const int32_t* src,
                  const int32_t* eid, const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                  int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P, int32_t mode_flags,
                  float* out, int64_t out_node_stride, float* xcopy, int64_t xcopy_node_stride, void* stream) {
  const int32_t logits = (mode_flags & MRP_AGG_GB_LOGITS) ? 1 : 0;
  const int32_t mode = mode_flags & ~MRP_AGG_GB_LOGITS;
  if (!common_args_ok(indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind, num_nodes, num_edges, C, P,
                      mode))
    return hipErrorInvalidValue;
  if (num_graphs == 0 || num_nodes == 0 || max_nodes == 0 || C == 0 || P == 0) return hipSuccess;
  const int64_t plane = (int64_t)C * P;
  if (x == nullptr || out == nullptr || x_node_stride < plane || out_node_stride < plane)
    return hipErrorInvalidValue;
  if (mode != MRP_AGG_COPY_MEAN && num_edges > 0 && gb == nullptr) return hipErrorInvalidValue;
  if (xcopy != nullptr && xcopy_node_stride < plane) return hipErrorInvalidValue;
  bool vec4 =
      (P % 4 == 0) && (x_node_stride % 4 == 0) && (out_node_stride % 4 == 0) && aligned16(x) && aligned16(out);
  if (xcopy != nullptr) vec4 = vec4 && (xcopy_node_stride % 4 == 0) && aligned16(xcopy);
  // 16-byte slices beat 8-byte ones at every measured size (tools/kernel_lab.hip product sweep)
  Geometry g = make_geometry(C, P, vec4 ? 4 : 1, 16, 64, mrp::kMaxChanPerBlock);
  // COMPLETE graphs: one slice per lane, the plane split over ceil(PV / lpc) workgroups (their
  // prologue is one round of independent gamma/beta loads, hidden under the first slice).  CSR
  // graphs keep whole planes: their prologue walks the CSR (dependent loads) and a split repeats it
  // per segment (k-NN(4) N=16 C=1024 16x16: 304 us split vs 225 us whole)
  const int32_t pv = P / g.vec;
  const int32_t psplit = graph_kind == MRP_GRAPH_COMPLETE ? (pv + g.lpc - 1) / g.lpc : 1;
  g.grid = (int64_t)num_graphs * g.ncb * psplit;
  if (g.grid > 0x7fffffff) return hipErrorInvalidValue;
  AggArgs a = {};
  a.x = x;
  a.xs = x_node_stride;
  a.gb = gb;
  a.indptr = indptr;
  a.src = src;
  a.eid = eid;
  a.goff = graph_off;
  a.out = out;
  a.os = out_node_stride;
  a.C = C;
  a.P = P;
  a.PV = P / g.vec;
  a.mode = mode;
  a.lpc = g.lpc;
  a.cpb = g.cpb;
  a.ncb = g.ncb;
  a.logits = logits;
  a.xc = xcopy;
  a.xcs = xcopy_node_stride;
  a.psplit = psplit;
  a.kdeg = MRP_GRAPH_IS_REGULAR(graph_kind) ? MRP_GRAPH_REGULAR_K(graph_kind) : 0;
  return dispatch_fwd(max_nodes, graph_kind == MRP_GRAPH_COMPLETE, a, g, static_cast<hipStream_t>(stream));
}

}  // namespace

extern "C" {

int mrp_film_mean_fwd(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                      const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                      int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C,
                      int32_t P, int32_t mode_flags, float* out, int64_t out_node_stride, void* stream) {
  return film_fwd_impl(x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind,
                       num_nodes, num_edges, C, P, mode_flags, out, out_node_stride, nullptr, 0, stream);
}

int mrp_film_mean_cat_fwd(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                          const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                          int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C,
                          int32_t P, int32_t mode_flags, float* cat, int64_t cat_node_stride, void* stream) {
  if (cat == nullptr || cat_node_stride < 2 * (int64_t)C * P) return hipErrorInvalidValue;
  return film_fwd_impl(x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind,
                       num_nodes, num_edges, C, P, mode_flags, cat + (int64_t)C * P, cat_node_stride, cat,
                       cat_node_stride, stream);
}

}  // extern "C"
