// cmpc_wide_w80r.hip — the 80-column wide class with the fp64 refinement step of the converged
// active set (cmpc_wide.h wide_refine; horizons N > 10), one workgroup per list entry.
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 5
#endif
#define CMPC_WIDE_BUILD 1
#define CMPC_WIDE_REFINE 1
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w80_r(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                            hipStream_t stream, int base) {
  return launch_wide_impl<80>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid, stream, base);
}

}  // namespace cmpc
