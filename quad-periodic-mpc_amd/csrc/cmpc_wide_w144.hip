// cmpc_wide_w144.hip — wide size class with 144-column rows (n 129-144: random contact tables at N = 20) (kernel template: cmpc_wide.h).
// four waves per SIMD (128 VGPRs, 42 spilled) and 51 KB of LDS (R^-1 kept for 40 active-set
// positions, not 64): three five-wave workgroups per CU where three waves per SIMD (167 VGPRs, no
// spills) and 56 KB admitted two. Config 5 4.33 M -> 4.73 M QP/s (same-box A/B r04_c5)
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 4
#endif
#define CMPC_WIDE_BUILD 2  // launch forms built (cmpc_wide.h): persistent only
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w144(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  return launch_wide_impl<144>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                              stream, base);
}

}  // namespace cmpc
