# the one-launch encoder's all-X form with a deeper W2 fragment ring: RING sets (RING - 1 hidden blocks
# ahead) instead of four; the z accumulation order is unchanged (bit-identical logits).  RING from the
# environment at build time (default 6).
import os

RING = int(os.environ.get("ENC_RING", "6"))
PRO_OLD = """  W2F f0, f1, f2, f3;"""
PRO_NEW = """  W2F f0, f1, f2, f3;
  constexpr int RING = %d;
  W2F fr[RING];""" % RING
LD_OLD = """  load_w2(0, f0);
  if (1 < HB) load_w2(1, f1);
  if (2 < HB) load_w2(2, f2);
  x_store(0, w);"""
LD_NEW = """  if constexpr (ALLX) {
#pragma unroll
    for (int j = 0; j < RING - 1; ++j)
      if (j < HB) load_w2(j, fr[j]);
  } else {
    load_w2(0, f0);
    if (1 < HB) load_w2(1, f1);
    if (2 < HB) load_w2(2, f2);
  }
  x_store(0, w);"""
OLD = """#pragma unroll 1
    for (int hb = 0; hb < HB; hb += 4) {
      if (hb + 3 < HB) load_w2(hb + 3, f3);
      z_block(hb / NWV, hb % NWV, f0);
      if (hb + 4 < HB) load_w2(hb + 4, f0);
      if (hb + 1 < HB) z_block((hb + 1) / NWV, (hb + 1) % NWV, f1);
      if (hb + 5 < HB) load_w2(hb + 5, f1);
      if (hb + 2 < HB) z_block((hb + 2) / NWV, (hb + 2) % NWV, f2);
      if (hb + 6 < HB) load_w2(hb + 6, f2);
      if (hb + 3 < HB) z_block((hb + 3) / NWV, (hb + 3) % NWV, f3);
    }"""
NEW = """#pragma unroll 1
    for (int hb = 0; hb < HB; hb += RING) {
#pragma unroll
      for (int j = 0; j < RING; ++j) {
        if (hb + j + RING - 1 < HB) load_w2(hb + j + RING - 1, fr[(j + RING - 1) % RING]);
        if (hb + j < HB) z_block((hb + j) / NWV, (hb + j) % NWV, fr[j]);
      }
    }"""
PATCH = [("encoder_split.hip", PRO_OLD, PRO_NEW), ("encoder_split.hip", LD_OLD, LD_NEW),
         ("encoder_split.hip", OLD, NEW)]
