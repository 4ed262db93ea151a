// film_mean_fwd.hip — forward launchers and C ABI (mrp_film_mean_fwd, mrp_film_mean_cat_fwd).
// Kernels and design notes: film_mean_kernels.hpp.
#include <cstring>
#include <unordered_map>

#include "film_mean_kernels.hpp"

using namespace mrp_host;

namespace {

template <int NT, int KMAX>
hipError_t launch_fwd_regular(const AggArgs& a, const Geometry& g, hipStream_t st) {
  const size_t lds = lds_fwd_regular<NT, KMAX>(g.cpb);
  // k-NN(4) in a mean mode (BASELINE configs[4]): compile-time degree, exact division by 4
  if constexpr (KMAX == 4) {
    if (g.vec == 4 && a.kdeg == 4 && a.mode != MRP_AGG_FILM_SUM) {
      MRP_LAUNCH((mrp::film_fwd_regular<NT, KMAX, 4, 4>), lds);
      return hipGetLastError();
    }
  }
  if (g.vec == 4)
    MRP_LAUNCH((mrp::film_fwd_regular<NT, KMAX, 4>), lds);
  else if (g.vec == 1)
    MRP_LAUNCH((mrp::film_fwd_regular<NT, KMAX, 1>), lds);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template <int NT, bool COMPLETE>
hipError_t launch_fwd_nt(const AggArgs& a, const Geometry& g, hipStream_t st) {
  if constexpr (!COMPLETE) {
    // per-edge-slot weights for uniform in-degree (k-NN frames)
    if (a.kdeg >= 1 && a.kdeg <= 4) return launch_fwd_regular<NT, 4>(a, g, st);
    if (a.kdeg >= 5 && a.kdeg <= 8) return launch_fwd_regular<NT, 8>(a, g, st);
  }
  const size_t lds = lds_fwd<NT>(g.cpb);
  if constexpr (COMPLETE && NT >= 2 && NT <= 8) {
    // the reference's own configuration: mode and mean divisor compile-time (film_fwd MODE)
    if (g.vec == 4 && a.mode == MRP_AGG_FILM_MEAN) {
      MRP_LAUNCH((mrp::film_fwd<NT, 4, true, MRP_AGG_FILM_MEAN>), lds);
      return hipGetLastError();
    }
    if (g.vec == 2 && a.mode == MRP_AGG_FILM_MEAN) {
      MRP_LAUNCH((mrp::film_fwd<NT, 2, true, MRP_AGG_FILM_MEAN>), lds);
      return hipGetLastError();
    }
  }
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

// The streaming yardstick beside the aggregation rooflines (mrp_stream_copy): one nontemporal 16-byte
// load and store per thread per trip, grid-stride, 256 threads, one trip per thread where the grid
// allows (tools/copy_ceiling.hip's copy1, the best of round 1's copy sweep).
__global__ void __launch_bounds__(256) stream_copy(const mrp::f4* __restrict__ in, mrp::f4* __restrict__ out,
                                                   size_t n) {
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(in + i), out + i);
}

namespace mrp_host {
Tuning& tuning() {
  static Tuning t;
  return t;
}
}  // namespace mrp_host

extern "C" {

int mrp_abi_version(void) { return 21; }

int mrp_tuning_set(const char* name, int32_t value) {
  if (name == nullptr) return hipErrorInvalidValue;
  Tuning& t = tuning();
  if (std::strcmp(name, "reset") == 0) {
    t = Tuning();
    return hipSuccess;
  }
  struct Knob {
    const char* name;
    int* field;
    int lo, hi;
  } knobs[] = {
      {"fwd_lo", &t.fwd_lo, 1, 256},
      {"fwd_hi", &t.fwd_hi, 1, 256},
      {"fwd_cap", &t.fwd_cap, 1, 16},
      {"fwd_vec2_below", &t.fwd_vec2_below, 0, 1 << 20},
      {"fwd_regular_split", &t.fwd_regular_split, 0, 1},
      {"fwd_regular_lo", &t.fwd_regular_lo, 1, 256},
      {"fwd_regular_hi", &t.fwd_regular_hi, 1, 256},
      {"fwd_regular_cap", &t.fwd_regular_cap, 1, 16},
      {"bwd_fused_lo", &t.bwd_fused_lo, 1, 256},
      {"bwd_fused_hi", &t.bwd_fused_hi, 1, 256},
      {"bwd_fused_cap", &t.bwd_fused_cap, 1, 64},
      {"bwd_pre2", &t.bwd_pre2, 0, 2},
      {"bwd_regular_vec", &t.bwd_regular_vec, 1, 2},
      {"bwd_regular_lanes", &t.bwd_regular_lanes, 1, 64},
      {"bwd_regular_mfma", &t.bwd_regular_mfma, 0, 1},
      {"bwd_complete_mfma", &t.bwd_complete_mfma, 0, 1},
      {"bwd_mfma_cpw", &t.bwd_mfma_cpw, 1, 2},
      {"edge_split_v", &t.edge_split_v, -1, 3},
      {"edge_allx", &t.edge_allx, 0, 1},
      {"gemm_split", &t.gemm_split, -1, 7},
      {"split_nt", &t.split_nt, -1, 4},
      {"gemm_group", &t.gemm_group, 0, 64},
      {"nt_group", &t.nt_group, 0, 64},
      {"enc_bwd_psa", &t.enc_bwd_psa, 0, 2},
      {"enc_s1", &t.enc_s1, 0, 64},
      {"enc_s2", &t.enc_s2, 0, 64},
  };
  for (const Knob& k : knobs) {
    if (std::strcmp(name, k.name) == 0) {
      if (value < k.lo || value > k.hi) return hipErrorInvalidValue;
      // knobs that name kernels accept only the product's: gemm_split -1 (per shape), 2 or 7;
      // split_nt -1 (per shape), 3 or 4 (compress_split.hip; round 4's other forms: tools/lab_forms.hip)
      if (k.field == &t.gemm_split && value != -1 && value != 2 && value != 7) return hipErrorInvalidValue;
      if (k.field == &t.split_nt && value != -1 && value != 3 && value != 4) return hipErrorInvalidValue;
      if (k.field == &t.edge_split_v && value != -1 && value != 1 && value != 3) return hipErrorInvalidValue;
      *k.field = value;
      return hipSuccess;
    }
  }
  return hipErrorInvalidValue;
}

const char* mrp_error_string(int code) { return hipGetErrorString(static_cast<hipError_t>(code)); }

int mrp_stream_join(void* waiter, void* signaller) {
  if (waiter == signaller) return hipSuccess;
  // one event per signalling stream and host thread, re-recorded each call: a wait enqueued earlier
  // keeps the record it was enqueued behind
  thread_local std::unordered_map<void*, hipEvent_t> events;
  hipEvent_t& ev = events[signaller];
  if (ev == nullptr) {
    const hipError_t c = hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventReleaseToDevice);
    if (c != hipSuccess) {
      ev = nullptr;
      return c;
    }
  }
  hipError_t e = hipEventRecord(ev, static_cast<hipStream_t>(signaller));
  if (e == hipSuccess) e = hipStreamWaitEvent(static_cast<hipStream_t>(waiter), ev, 0);
  return e;
}

int mrp_stream_copy(const void* src, void* dst, int64_t bytes, void* stream) {
  if (bytes < 0 || (bytes % 16) != 0) return hipErrorInvalidValue;
  if (bytes == 0) return hipSuccess;
  if (!src || !dst || !aligned16(src) || !aligned16(dst)) return hipErrorInvalidValue;
  const size_t n = (size_t)bytes / 16;
  const size_t blocks = std::min<size_t>((n + 255) / 256, (size_t)1 << 30);
  hipLaunchKernelGGL(stream_copy, dim3((unsigned)blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     static_cast<const mrp::f4*>(src), static_cast<mrp::f4*>(dst), n);
  return hipGetLastError();
}

}  // extern "C"

namespace {

int film_fwd_impl(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr, const int32_t* src,
                  const int32_t* eid, const int32_t* graph_off, int32_t num_graphs, int32_t max_nodes,
                  int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C, int32_t P, int32_t mode_flags,
                  float* out, int64_t out_node_stride, const mrp_agg_epilogue* ep, void* stream) {
  float* xcopy = ep != nullptr ? ep->xcopy : nullptr;
  const int64_t xcopy_node_stride = ep != nullptr ? ep->xcopy_node_stride : 0;
  const float* x0 = ep != nullptr ? ep->x0 : nullptr;
  const int64_t x0_node_stride = ep != nullptr ? ep->x0_node_stride : 0;
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
  if (x0 != nullptr && x0_node_stride < plane) return hipErrorInvalidValue;
  bool vec4 =
      (P % 4 == 0) && (x_node_stride % 4 == 0) && (out_node_stride % 4 == 0) && aligned16(x) && aligned16(out);
  if (xcopy != nullptr) vec4 = vec4 && (xcopy_node_stride % 4 == 0) && aligned16(xcopy);
  if (x0 != nullptr) vec4 = vec4 && (x0_node_stride % 4 == 0) && aligned16(x0);
  const int32_t kdeg = MRP_GRAPH_IS_REGULAR(graph_kind) ? MRP_GRAPH_REGULAR_K(graph_kind) : 0;
  const bool regular = kdeg >= 1 && kdeg <= 8;
  // 16-byte slices beat 8-byte ones at every measured size (tools/kernel_lab.hip product sweep)
  const Tuning& tu = tuning();
  const int fvec = vec4 ? (P < tu.fwd_vec2_below ? 2 : 4) : 1;
  Geometry g = regular ? make_geometry(C, P, vec4 ? 4 : 1, tu.fwd_regular_lo, tu.fwd_regular_hi, tu.fwd_regular_cap)
                       : make_geometry(C, P, fvec, tu.fwd_lo, tu.fwd_hi, tu.fwd_cap);
  // COMPLETE graphs: one slice per lane, the plane split over ceil(PV / lpc) workgroups (their
  // prologue is one round of independent gamma/beta loads, hidden under the first slice).  CSR
  // graphs keep whole planes: their prologue walks the CSR (dependent loads) and a split repeats it
  // per segment (k-NN(4) N=16 C=1024 16x16: 304 us split vs 225 us whole)
  const int32_t pv = P / g.vec;
  const int32_t psplit = (graph_kind == MRP_GRAPH_COMPLETE || (regular && tu.fwd_regular_split))
                             ? (pv + g.lpc - 1) / g.lpc
                             : 1;
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
  a.kdeg = kdeg;
  a.agg_scale = 1.f;
  if (ep != nullptr) {
    a.agg_scale = ep->agg_scale;
    a.self_scale = ep->self_scale;
    a.x0 = x0;
    a.x0s = x0_node_stride;
    a.x0_scale = ep->x0_scale;
    a.epi = (ep->agg_scale != 1.f || ep->self_scale != 0.f || x0 != nullptr) ? 1 : 0;
  }
  return dispatch_fwd(max_nodes, graph_kind == MRP_GRAPH_COMPLETE, a, g, static_cast<hipStream_t>(stream));
}

}  // namespace

extern "C" {

int mrp_film_mean_fwd(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                      const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                      int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C,
                      int32_t P, int32_t mode_flags, float* out, int64_t out_node_stride, void* stream) {
  return film_fwd_impl(x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind,
                       num_nodes, num_edges, C, P, mode_flags, out, out_node_stride, nullptr, stream);
}

int mrp_film_mean_fwd_ex(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                         const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                         int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C,
                         int32_t P, int32_t mode_flags, float* out, int64_t out_node_stride,
                         const mrp_agg_epilogue* epilogue, void* stream) {
  return film_fwd_impl(x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind,
                       num_nodes, num_edges, C, P, mode_flags, out, out_node_stride, epilogue, stream);
}

int mrp_film_mean_cat_fwd(const float* x, int64_t x_node_stride, const float* gb, const int32_t* indptr,
                          const int32_t* src, const int32_t* eid, const int32_t* graph_off, int32_t num_graphs,
                          int32_t max_nodes, int32_t graph_kind, int32_t num_nodes, int32_t num_edges, int32_t C,
                          int32_t P, int32_t mode_flags, float* cat, int64_t cat_node_stride, void* stream) {
  if (cat == nullptr || cat_node_stride < 2 * (int64_t)C * P) return hipErrorInvalidValue;
  mrp_agg_epilogue ep = {1.f, 0.f, nullptr, 0, 0.f, cat, cat_node_stride};
  return film_fwd_impl(x, x_node_stride, gb, indptr, src, eid, graph_off, num_graphs, max_nodes, graph_kind,
                       num_nodes, num_edges, C, P, mode_flags, cat + (int64_t)C * P, cat_node_stride, &ep, stream);
}

}  // extern "C"
