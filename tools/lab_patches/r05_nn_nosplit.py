# upper bound of the NN GEMM's in-kernel activation split: each B piece converted once (part 0) and the
# two small parts stored as zeros — outputs wrong by design; prices the split's VALU work
PATCH = [("compress_split.hip", """      uint32_t l0, l1, l2, h0, h1, h2;
      split2(lo, l0, l1, l2);
      split2(hi, h0, h1, h2);
      p0.x = l0, p1.x = l1, p2.x = l2, p0.y = h0, p1.y = h1, p2.y = h2;
      const uint32_t o = boff(kr + G::KR * j, fc >> 1) + 8 * (fc & 1);""", """      uint32_t l0 = cvt2(lo), h0 = cvt2(hi);
      p0.x = l0, p1.x = 0u, p2.x = 0u, p0.y = h0, p1.y = 0u, p2.y = 0u;
      const uint32_t o = boff(kr + G::KR * j, fc >> 1) + 8 * (fc & 1);""")]
