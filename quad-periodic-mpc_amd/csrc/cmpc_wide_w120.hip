// cmpc_wide_w120.hip — wide size class with 120-column rows (n 97-120: every trot instance at
// N = 20, n = 120; the 128-column build keeps n 121-128) (kernel template: cmpc_wide.h).
// four waves per SIMD: 118 VGPRs and 34 KB of LDS (the stage buffers share P's tail), four
// four-wave workgroups per CU
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 4
#endif
#ifndef CMPC_WIDE_BUILD
#define CMPC_WIDE_BUILD 1  // one workgroup per entry here; the persistent form in cmpc_wide_w120p.hip
#endif
#ifndef CMPC_WIDE_REFINE
#define CMPC_WIDE_REFINE 0  // N <= 10 (no refinement); the refining builds: cmpc_wide_w120r.hip, w120pr.hip
#endif
#ifndef CMPC_WIDE_PRIO
#define CMPC_WIDE_PRIO 1  // N <= 10: issue priority over the class-1 waves (config 2 +1.9 %, config 3 +0.2 %, r04_p)
#endif
#include "cmpc_wide.h"

namespace cmpc {

// the same class with the fp64 refinement step (N > 10), each launch form in its own unit
hipError_t launch_wide_w120_r(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                            hipStream_t stream, int base);
hipError_t launch_wide_w120_persist_r(const float* d_recs, const KParams& P, float* d_forces,
                                    uint8_t* d_status, int32_t* d_iters, const int* in_list,
                                    const int* in_count, int* deq, int grid, hipStream_t stream, int base);

hipError_t launch_wide_w120(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  if (P.refine)
    return deq ? launch_wide_w120_persist_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid, stream, base)
               : launch_wide_w120_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid, stream, base);
  if (deq)  // persistent form: its own unit (compiled beside this kernel it spilled registers)
    return launch_wide_w120_persist(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                                   stream, base);
  return launch_wide_impl<120>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid,
                              stream, base);
}

}  // namespace cmpc
