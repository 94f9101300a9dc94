// cmpc_wide_w80.hip — wide size class with 80-column rows (kernel template: cmpc_wide.h).
// five waves per SIMD (94 VGPRs, no spills): config 3's n 65-80 instances finish inside class 1's
// run
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 5
#endif
#ifndef CMPC_WIDE_BUILD
#define CMPC_WIDE_BUILD 1  // one workgroup per entry here; the persistent form in cmpc_wide_w80p.hip
#endif
#ifndef CMPC_WIDE_REFINE
#define CMPC_WIDE_REFINE 0  // N <= 10 (no refinement); the refining builds: cmpc_wide_w80r.hip, w80pr.hip
#endif
#ifndef CMPC_WIDE_PRIO
#define CMPC_WIDE_PRIO 1  // N <= 10: issue priority over the class-1 waves (config 2 +1.9 %, config 3 +0.2 %, r04_p)
#endif
#include "cmpc_wide.h"

namespace cmpc {

// the same class with the fp64 refinement step (N > 10), each launch form in its own unit
hipError_t launch_wide_w80_r(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                            hipStream_t stream, int base);
hipError_t launch_wide_w80_persist_r(const float* d_recs, const KParams& P, float* d_forces,
                                    uint8_t* d_status, int32_t* d_iters, const int* in_list,
                                    const int* in_count, int* deq, int grid, hipStream_t stream, int base);

hipError_t launch_wide_w80(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  if (P.refine)
    return deq ? launch_wide_w80_persist_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid, stream, base)
               : launch_wide_w80_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid, stream, base);
  if (deq)  // persistent form: its own unit (compiled beside this kernel it spilled registers)
    return launch_wide_w80_persist(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                                   stream, base);
  return launch_wide_impl<80>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid,
                              stream, base);
}

}  // namespace cmpc
