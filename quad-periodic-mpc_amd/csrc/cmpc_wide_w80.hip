// cmpc_wide_w80.hip — wide size class with 80-column rows (kernel template: cmpc_wide.h).
// five waves per SIMD (96 VGPRs, one spilled): config 3's n 65-80 instances finish inside
// class 1's run (tail beyond class 1 0.30 -> 0.15 ms, config 3 29.2M -> 29.6M QP/s)
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 5
#endif
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w80(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream) {
  return launch_wide_impl<80>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                              stream);
}

}  // namespace cmpc
