# the aggregation kernels with an XCD-aware workgroup order: the hardware deals workgroups to the 8 XCDs
# round robin (blockIdx % 8), so the workgroups that share a gamma/beta line of z (one graph, adjacent
# channel blocks and plane segments: consecutive ids) each fetched it into a different XCD's L2 — the
# PMC passes show ~7 x |z| of extra fetch in film_fwd and film_bwd_fused.  Logical ids dealt in
# contiguous chunks per XCD instead; the outputs are unchanged (bit-identical).
HELPER = """__device__ __forceinline__ float sigmoidf(float z) { return mrp_math::sigmoid(z); }  // fast_math.hpp"""
HELPER_NEW = """__device__ __forceinline__ int xcd_block() {
  const int nwg = (int)gridDim.x, orig = (int)blockIdx.x;
  const int q = nwg / 8, rr = nwg % 8, xcd = orig % 8;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + orig / 8;
}
""" + HELPER
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
PATCH = [("film_mean_kernels.hpp", HELPER, HELPER_NEW), ("film_mean_kernels.hpp", A, A_NEW),
         ("film_mean_kernels.hpp", B, B_NEW)]
