# the training encoder (all-X form) stores h^T after its z loop instead of in the X prologue: relu(X) of
# the wave's two hidden blocks kept in registers (32 floats) so the prologue's stores and their address
# arithmetic do not sit between the W2 requests and the first z block; h^T and z unchanged.
OLD_DECL = """  auto x_store_from = [&](int buf, int hbx, const u4 (&wsrc)[3]) {"""
NEW_DECL = """  f16v Xk[2];
  auto x_store_from = [&](int buf, int hbx, const u4 (&wsrc)[3]) {"""
OLD_ST = """    if (a.hT != nullptr && hbx % ngroups == cg && hbx < HB && e0 + r < a.E) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        a.hT[(int64_t)(hbx * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * a.hts + e0 + r] = relu(X[i]);
    }"""
NEW_ST = """    if constexpr (ALLX) {
      Xk[buf] = X;
    } else if (a.hT != nullptr && hbx % ngroups == cg && hbx < HB && e0 + r < a.E) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        a.hT[(int64_t)(hbx * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * a.hts + e0 + r] = relu(X[i]);
    }"""
OLD_END = """      if (hb + 3 < HB) z_block((hb + 3) / NWV, (hb + 3) % NWV, f3);
    }
  } else {"""
NEW_END = """      if (hb + 3 < HB) z_block((hb + 3) / NWV, (hb + 3) % NWV, f3);
    }
    if (a.hT != nullptr && e0 + r < a.E) {
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int hbx = w + q * NWV;
        if (hbx < HB && hbx % ngroups == cg) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            a.hT[(int64_t)(hbx * 32 + (i & 3) + 8 * (i >> 2) + 4 * hh) * a.hts + e0 + r] = relu(Xk[q][i]);
        }
      }
    }
  } else {"""
PATCH = [("encoder_split.hip", OLD_DECL, NEW_DECL), ("encoder_split.hip", OLD_ST, NEW_ST),
         ("encoder_split.hip", OLD_END, NEW_END)]
