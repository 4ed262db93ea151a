// film_mean_bwd_13_16.hip — backward launches for graphs of 13..16 nodes (see film_mean_bwd.hip).
#include "film_mean_bwd_launch.hpp"

namespace mrp_host {

hipError_t dispatch_bwd_13_16(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st) {
  switch (nt) {
    MRP_NT_CASE(13, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(14, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(15, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(16, complete, launch_bwd_nt, a, g, st)
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mrp_host
