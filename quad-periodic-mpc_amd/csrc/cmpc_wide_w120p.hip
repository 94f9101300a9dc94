// cmpc_wide_w120p.hip — the persistent launch form of the 120-column wide class (kernel template:
// cmpc_wide.h; launch_solve uses it when the class does not hold the trot size n = 6N).
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 4
#endif
#define CMPC_WIDE_BUILD 2
#ifndef CMPC_WIDE_REFINE
#define CMPC_WIDE_REFINE 0  // N <= 10; the refining persistent build: cmpc_wide_w120pr.hip
#endif
#ifndef CMPC_WIDE_PRIO
#define CMPC_WIDE_PRIO 1  // N <= 10: issue priority over the class-1 waves (config 2 +1.9 %, config 3 +0.2 %, r04_p)
#endif
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w120_persist(const float* d_recs, const KParams& P, float* d_forces,
                                  uint8_t* d_status, int32_t* d_iters, const int* in_list,
                                  const int* in_count, int* deq, int grid, hipStream_t stream, int base) {
  return launch_wide_impl<120>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                              stream, base);
}

}  // namespace cmpc
