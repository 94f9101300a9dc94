// cmpc_wide_w128p.hip — the persistent launch form of the 128-column wide class (kernel template:
// cmpc_wide.h; launch_solve uses it when the class does not hold the trot size n = 6N).
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 4
#endif
#define CMPC_WIDE_BUILD 2
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w128_persist(const float* d_recs, const KParams& P, float* d_forces,
                                  uint8_t* d_status, int32_t* d_iters, const int* in_list,
                                  const int* in_count, int* deq, int grid, hipStream_t stream, int base) {
  return launch_wide_impl<128>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                              stream, base);
}

}  // namespace cmpc
