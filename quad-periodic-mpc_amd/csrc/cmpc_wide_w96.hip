// cmpc_wide_w96.hip — wide size class with 96-column rows (kernel template: cmpc_wide.h).
// five waves per SIMD, 96 VGPRs, no spills (N = 16 trot, the reference's deployed horizon: every
// instance n = 96)
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 5
#endif
#ifndef CMPC_WIDE_BUILD
#define CMPC_WIDE_BUILD 1  // one workgroup per entry here; the persistent form in cmpc_wide_w96p.hip
#endif
#ifndef CMPC_WIDE_REFINE
#define CMPC_WIDE_REFINE 0  // N <= 10 (no refinement); the refining builds: cmpc_wide_w96r.hip, w96pr.hip
#endif
#ifndef CMPC_WIDE_PRIO
#define CMPC_WIDE_PRIO 1  // N <= 10: issue priority over the class-1 waves (config 2 +1.9 %, config 3 +0.2 %, r04_p)
#endif
#include "cmpc_wide.h"

namespace cmpc {

// the same class with the fp64 refinement step (N > 10), each launch form in its own unit
hipError_t launch_wide_w96_r(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                            hipStream_t stream, int base);
hipError_t launch_wide_w96_persist_r(const float* d_recs, const KParams& P, float* d_forces,
                                    uint8_t* d_status, int32_t* d_iters, const int* in_list,
                                    const int* in_count, int* deq, int grid, hipStream_t stream, int base);

hipError_t launch_wide_w96(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                          int32_t* d_iters, const int* in_list, const int* in_count, int* deq, int grid,
                          hipStream_t stream, int base) {
  if (P.refine)
    return deq ? launch_wide_w96_persist_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid, stream, base)
               : launch_wide_w96_r(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid, stream, base);
  if (deq)  // persistent form: its own unit (compiled beside this kernel it spilled registers)
    return launch_wide_w96_persist(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, deq, grid,
                                   stream, base);
  return launch_wide_impl<96>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, nullptr, grid,
                              stream, base);
}

}  // namespace cmpc
