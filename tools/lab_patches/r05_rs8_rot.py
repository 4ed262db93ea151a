# the fused backward's reduce-scatter also at 8 lanes per plane (8x8 planes): each lane ends with one
# Gram row (8 sums) and stores it in an order rotated by its channel group's index within the wave, so
# the wave's 64 stores of one instruction meet 64 distinct LDS banks (round 5 first measured the
# unrotated form 4 % slower: 4-way conflicts)
PATCH = [("film_mean_kernels.hpp", """        rs_store<64, NTP>(vals, lir, active, Sl + pg * SLS, Dl + pg * SZ);
        reduced = true;
      }""", """        rs_store<64, NTP>(vals, lir, active, Sl + pg * SLS, Dl + pg * SZ);
        reduced = true;
      } else if (a.want_dgb && a.lpc == 8) {
        __builtin_amdgcn_sched_barrier(0);
        float vals[64];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int u = 0; u < 8; ++u) vals[i * 8 + u] = u == i ? S[i] : D[i][u];
        reduce_scatter64<8>(vals, threadIdx.x & 63);  // lane gl: vals[u] = the group's sum of row gl, slot u
        const int gl = (int)threadIdx.x & 7, rot = ((int)threadIdx.x >> 3) & 7;
        // rotate by rot (three conditional rotations: 24 selects) so that store k writes slot (k + rot) & 7
        float r1[8], r2[8], r3[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r1[k] = (rot & 1) ? vals[(k + 1) & 7] : vals[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) r2[k] = (rot & 2) ? r1[(k + 2) & 7] : r1[k];
#pragma unroll
        for (int k = 0; k < 8; ++k) r3[k] = (rot & 4) ? r2[(k + 4) & 7] : r2[k];
        if (active) {
          float* sl = Sl + grp * SLS;
          float* dl = Dl + grp * SZ + gl * NTP;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const int u = (k + rot) & 7;
            *(u == gl ? sl + gl : dl + u) = r3[k];
          }
        }
        reduced = true;
      }""")]
