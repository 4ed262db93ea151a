// fast_math.hpp — x / D for a small compile-time integer D, correctly rounded (the IEEE quotient the
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

// sigmoid(z) = 1 / (1 + e^-z) as v_exp_f32 + v_rcp_f32 (4 instructions instead of ~22 for expf and
// an IEEE division): the aggregation prologues apply it to every (edge, channel) logit
// (MRP_AGG_GB_LOGITS), and at 8x8 planes that sat on the critical path — configs[2] forward 39.5 us
// with the accurate form vs 31.9 us with post-sigmoid inputs (tools/exp_fwd_modes.py).  Error:
// exp2 and rcp are ~1 ulp; the x log2(e) product rounds to 2^-24 |x log2 e|, so sigma is within
// ~1e-7 + 3e-8 |z| relative of the exact value (tests hold the logits path to 1e-6 of torch.sigmoid).
// z -> -inf: e^-z = inf, rcp = 0; z -> +inf: 1.
__device__ __forceinline__ float sigmoid(float z) {
  const float e = __builtin_amdgcn_exp2f(-1.4426950408889634f * z);
  return __builtin_amdgcn_rcpf(1.0f + e);
}

}  // namespace mrp_math
