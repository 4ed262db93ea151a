// film_mean_bwd_1_8.hip — backward launches for graphs of 1..8 nodes (see film_mean_bwd.hip).
#include "film_mean_bwd_launch.hpp"

namespace mrp_host {

hipError_t dispatch_bwd_1_8(int nt, bool complete, const AggArgs& a, const Geometry& g, hipStream_t st) {
  switch (nt) {
    MRP_NT_CASE(1, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(2, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(3, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(4, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(5, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(6, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(7, complete, launch_bwd_nt, a, g, st)
    MRP_NT_CASE(8, complete, launch_bwd_nt, a, g, st)
    default: return hipErrorInvalidValue;
  }
}

}  // namespace mrp_host
