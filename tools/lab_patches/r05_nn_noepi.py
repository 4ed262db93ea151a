# upper bound of the NN GEMM's epilogue cost: the 16x16x32 form computes its outputs but stores none
PATCH = [("compress_split.hip", """          *dst = v;
        }
    }
    return;""", """          if (v == 1234.5f) *dst = v;
        }
    }
    return;""")]
