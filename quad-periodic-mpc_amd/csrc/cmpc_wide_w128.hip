// cmpc_wide_w128.hip — wide size class with 128-column rows (kernel template: cmpc_wide.h).
// four waves per SIMD: 124 VGPRs and 38 KB of LDS (the stage buffers share P's tail), four
// four-wave workgroups per CU
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 4
#endif
#ifndef CMPC_WIDE_BUILD
#define CMPC_WIDE_BUILD 1  // one workgroup per entry here; the persistent form in cmpc_wide_w128p.hip
#endif
#include "cmpc_wide.h"

namespace cmpc {

hipError_t launch_wide_w128(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  if (deq)  // persistent form: its own unit (compiled beside this kernel it spilled registers)
    return launch_wide_w128_persist(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                                   stream, base);
  return launch_wide_impl<128>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid,
                              stream, base);
}

}  // namespace cmpc
