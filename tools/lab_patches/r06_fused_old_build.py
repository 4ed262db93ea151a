PATCH = [
 ("gcn_fused.hip", "      if (!(f.lab & 16)) X = mma6(wa, pp, X);", "      X = mma6(wa, pp, X);"),
 ("gcn_fused.hip", """    if (f.lab & 16) {
#pragma unroll
      for (int p = 0; p < 3; ++p) Z[p] += __builtin_bit_cast(float, as_u4(hp[p]).x ^ as_u4(wb[p]).x);
    } else {
      mma6_2(hp, wb, Z, ZL);
    }
  };""", """    mma6_2(hp, wb, Z, ZL);
  };"""),
 ("gcn_fused.hip", "    if (row < nval && !(f.lab & 8))", "    if (row < nval)"),
 ("gcn_fused.hip", """    if (f.lab & 32) {  // lab: occupy the slot for ~40 us without touching memory
      for (int i = 0; i < 20000; ++i) __builtin_amdgcn_s_sleep(1);
      return;
    }
""", ""),
]
