// film_mean_bwd_9_12.hip — backward launches for graphs of 9..12 nodes (see film_mean_bwd.hip).
#include "film_mean_bwd_launch.hpp"

namespace mrp_host {

hipError_t dispatch_bwd_9_12(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st) {
  switch (nt) {
    MRP_NT_CASE(9, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(10, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(11, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(12, complete, launch_bwd_nt, a, g, st)
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mrp_host
