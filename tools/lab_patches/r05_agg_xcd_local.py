# the aggregation kernels with a LOCAL XCD-aware order: within each span of 8 G consecutive workgroups,
# the G that share gamma/beta lines (one graph, adjacent channel blocks / plane segments) are dealt to
# one XCD (physical 8 i + x -> logical G x + i), so each z line is fetched into one L2 instead of up to
# eight, while the grid as a whole still advances through memory in the same order (r05_agg_xcd.py's
# whole-grid chunks per XCD measured 7-11 % slower).  Outputs unchanged.
import os

G = int(os.environ.get("XCD_G", "16"))
HELPER = """__device__ __forceinline__ float sigmoidf(float z) { return mrp_math::sigmoid(z); }  // fast_math.hpp"""
HELPER_NEW = """__device__ __forceinline__ int xcd_block() {
  constexpr int G = %d, span = 8 * G;
  const int nwg = (int)gridDim.x, p = (int)blockIdx.x;
  const int base = p / span * span;
  if (base + span > nwg) return p;
  const int r = p - base;
  return base + (r %% 8) * G + r / 8;
}
""" % G + HELPER
A = """  const int item = blockIdx.x / ps;
  const int seg = blockIdx.x - item * ps;"""
A_NEW = """  const int bidx = xcd_block();
  const int item = bidx / ps;
  const int seg = bidx - item * ps;"""
B = """  const int b = blockIdx.x / a.ncb;
  const int cb = blockIdx.x - b * a.ncb;"""
B_NEW = """  const int bidx = xcd_block();
  const int b = bidx / a.ncb;
  const int cb = bidx - b * a.ncb;"""
PATCH = [("film_mean_kernels.hpp", HELPER, HELPER_NEW), ("film_mean_kernels.hpp", B, B_NEW)]
if os.environ.get("XCD_FWD", "1") == "1":  # the forward kernels too (XCD_FWD=0: the backward kernels only)
    PATCH.append(("film_mean_kernels.hpp", A, A_NEW))
