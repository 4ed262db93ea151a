# encoder_bwd_reduce's per-hidden-unit loop over the edges unrolled ENC_UNROLL times (default 8) instead of 2,
# so more of a thread's partial / h^T / pose loads are in flight at once; sums in the same order.
import os

U = int(os.environ.get("ENC_UNROLL", "8"))
PATCH = [("compress_split.hip", """#pragma unroll 2
    for (int e = threadIdx.x; e < E; e += 256) {""", """#pragma unroll %d
    for (int e = threadIdx.x; e < E; e += 256) {""" % U)]
