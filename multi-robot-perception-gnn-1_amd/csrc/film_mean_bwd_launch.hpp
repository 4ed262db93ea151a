// film_mean_bwd_launch.hpp — backward launch templates, included by the film_mean_bwd_*.hip parts.
#pragma once
#include "film_mean_kernels.hpp"

namespace mrp_host {

template <int NT, bool COMPLETE, bool DXB>
hipError_t launch_bwd_ntb(const AggArgs& a_in, const Geometry& g, hipStream_t st) {
  if constexpr (NT <= 8) {
    const AggArgs& a = a_in;
    const size_t lds = lds_bwd<NT>(g.cpb, COMPLETE && a.logits, g.lpc);
    // exactly two slices per lane: both prefetched (film_bwd_fused PRE2; bwd_pre2 = 2: not with a
    // grad_x base, whose instantiation then prefetches the base rows instead)
    const int pre2 = tuning().bwd_pre2;
    if (g.vec == 4 && a.PV == 2 * g.lpc && (pre2 == 1 || (pre2 == 2 && !DXB))) {
      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 4, COMPLETE, DXB, 1, true>), lds);
      return hipGetLastError();
    }
    if (g.vec == 4)
      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 4, COMPLETE, DXB>), lds);
    else if (g.vec == 2)
      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 2, COMPLETE, DXB>), lds);
    else
      MRP_LAUNCH((mrp::film_bwd_fused<NT, NT, 1, COMPLETE, DXB>), lds);
    return hipGetLastError();
  } else {
    if (a_in.want_dx) {
      const AggArgs& a = a_in;
      const size_t lds = lds_dx<NT>(g.cpb);
      if (g.vec == 4)
        MRP_LAUNCH((mrp::film_bwd_dx<NT, 4, COMPLETE, DXB>), lds);
      else if (g.vec == 2)
        MRP_LAUNCH((mrp::film_bwd_dx<NT, 2, COMPLETE, DXB>), lds);
      else
        MRP_LAUNCH((mrp::film_bwd_dx<NT, 1, COMPLETE, DXB>), lds);
      hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    if (a_in.want_dgb) {
      AggArgs a = a_in;
      a.want_dx = 0;
      const size_t lds = lds_bwd<NT>(g.cpb, COMPLETE && a.logits);
      if (g.vec == 4)
        MRP_LAUNCH((mrp::film_bwd_fused<NT, 4, 4, COMPLETE>), lds);
      else if (g.vec == 2)
        MRP_LAUNCH((mrp::film_bwd_fused<NT, 4, 2, COMPLETE>), lds);
      else
        MRP_LAUNCH((mrp::film_bwd_fused<NT, 4, 1, COMPLETE>), lds);
      return hipGetLastError();
    }
    return hipSuccess;
  }
}

template <int NT, int KMAX, bool DXB>
hipError_t launch_bwd_regular(const AggArgs& a, const Geometry& g, hipStream_t st) {
  // VEC 4 would need 4*NT registers more per operand and spills; KMAX 8 only fits at VEC 1
  const size_t lds = lds_regular<NT, KMAX>(g.cpb);
  bool done = false;
  if constexpr (KMAX <= 4) {
    if (g.vec == 2) {
      MRP_LAUNCH((mrp::film_bwd_regular<NT, KMAX, 2, DXB>), lds);
      done = true;
    }
  }
  if (!done) MRP_LAUNCH((mrp::film_bwd_regular<NT, KMAX, 1, DXB>), lds);
  return hipGetLastError();
}

// film_bwd_mfma (mrp_film_mean_bwd_ex chose it and set g.mfma_npb, g.cpb = 4 x blocks per wave x
// channels per block)
template <bool COMPLETE, int NPB, int KMAX>
hipError_t launch_bwd_mfma_k(const AggArgs& a, const Geometry& g, hipStream_t st) {
  const size_t lds = lds_mfma(g.cpb, NPB, KMAX);
  const int cpw = g.cpb / (4 * (16 / NPB));
  if (a.dxb) {
    if (cpw == 1)
      MRP_LAUNCH((mrp::film_bwd_mfma<COMPLETE, NPB, KMAX, true, 1>), lds);
    else
      MRP_LAUNCH((mrp::film_bwd_mfma<COMPLETE, NPB, KMAX, true, 2>), lds);
  } else {
    if (cpw == 1)
      MRP_LAUNCH((mrp::film_bwd_mfma<COMPLETE, NPB, KMAX, false, 1>), lds);
    else
      MRP_LAUNCH((mrp::film_bwd_mfma<COMPLETE, NPB, KMAX, false, 2>), lds);
  }
  return hipGetLastError();
}


template <int NT, bool COMPLETE>
hipError_t launch_bwd_mfma(const AggArgs& a, const Geometry& g, hipStream_t st) {
  if constexpr (COMPLETE) {
    if constexpr (NT > 8) return launch_bwd_mfma_k<true, 16, 1>(a, g, st);
    return hipErrorInvalidValue;  // complete graphs of <= 8 nodes run film_bwd_fused
  } else {
    if constexpr (NT > 8) {
      if (a.kdeg >= 1 && a.kdeg <= 4) return launch_bwd_mfma_k<false, 16, 4>(a, g, st);
      if (a.kdeg >= 5 && a.kdeg <= 8) return launch_bwd_mfma_k<false, 16, 8>(a, g, st);
    }
    return hipErrorInvalidValue;
  }
}

template <int NT, bool COMPLETE>
hipError_t launch_bwd_nt(const AggArgs& a, const Geometry& g, hipStream_t st) {
  if (g.mfma_npb) return launch_bwd_mfma<NT, COMPLETE>(a, g, st);
  if constexpr (NT > 8 && !COMPLETE) {
    // regular in-degree (k-NN): per-edge-slot Gram, one sweep
    if (a.kdeg >= 1 && a.kdeg <= 4)
      return a.dxb ? launch_bwd_regular<NT, 4, true>(a, g, st) : launch_bwd_regular<NT, 4, false>(a, g, st);
    if (a.kdeg >= 5 && a.kdeg <= 8)
      return a.dxb ? launch_bwd_regular<NT, 8, true>(a, g, st) : launch_bwd_regular<NT, 8, false>(a, g, st);
  }
  return a.dxb ? launch_bwd_ntb<NT, COMPLETE, true>(a, g, st) : launch_bwd_ntb<NT, COMPLETE, false>(a, g, st);
}

}  // namespace mrp_host
