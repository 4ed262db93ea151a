// fast_div.hpp — x / D for a small compile-time integer D, correctly rounded (the IEEE quotient the
// reference's mean and the oracle compute), in three instructions instead of the ~10 of the IEEE
// division sequence:  q0 = x * RN(1/D),  r = fma(-q0, D, x) (exact),  q = fma(r, RN(1/D), q0).
// Checked exhaustively over all 2^32 fp32 x for D = 2..15 (tools/check_div_const.c): equal to x / D
// except for |x| < 2^-124, +-0 and +-inf.  Callers test a whole set of quotients once
// (div_fast_ok on the min / max of |x|) and take the IEEE division for the set otherwise, so the fast
// path has no per-quotient branch.
#pragma once

namespace mrp_math {

template <int D>
__device__ __forceinline__ float div_fast(float x) {
  if constexpr (D == 1) {
    return x;
  } else {
    constexpr float y = 1.0f / (float)D;
    const float q0 = __fmul_rn(x, y);
    const float r = __builtin_fmaf(-q0, (float)D, x);
    return __builtin_fmaf(r, y, q0);
  }
}

// min |x| >= 2^-124 and max |x| < inf over the set (NaN inputs give NaN either way)
__device__ __forceinline__ bool div_fast_ok(float mn, float mx) { return mn >= 0x1p-124f && mx < __builtin_inff(); }

}  // namespace mrp_math
