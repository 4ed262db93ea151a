# the fused backward's round-4 lane reduction (all-reduce of every Gram value, lane 0 stores) at every plane size
PATCH = [("film_mean_kernels.hpp", """      if (a.want_dgb && a.lpc >= 64) {""", """      if (false) {""")]
