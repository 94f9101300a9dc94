// cmpc_wide_w256.hip — wide size class with 256-column rows (kernel template: cmpc_wide.h).
#define CMPC_WIDE_BUILD 2  // launch forms built (cmpc_wide.h): persistent only
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w256(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  return launch_wide_impl<256>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                              stream, base);
}

}  // namespace cmpc
