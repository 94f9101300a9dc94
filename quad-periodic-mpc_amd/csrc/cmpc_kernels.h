// cmpc_kernels.h — internal interface between the HIP kernels and the C-ABI host layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cmpc_solver.h"

namespace cmpc {

// Kernel-side copy of cmpc_params (by value, lands in SGPRs).
struct KParams {
  float dt;
  float mu_inv;    // fmat uses 1/mu (SolverMPC.cpp:657)
  float f_max;
  float alpha2;    // 2 * alpha (qH = 2 (B'SB + alpha I))
  float wts[12];
  int N;
  int rec_words;
  int max_iter;
  int pad;
};

// Scratch ints needed by launch_solve for max_batch instances.
inline size_t work_ints(int max_batch) { return 4 + 2 * (size_t)max_batch; }

// ev (optional): 3 events recorded around the two size-class launches
// (ev[0] before class 1, ev[1] between, ev[2] after class 2).
hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        hipStream_t stream, hipEvent_t* ev = nullptr);
// per-class launchers (cmpc_class1.hip, cmpc_class2.hip)
hipError_t launch_class1(const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         int* ovf_list, int* ovf_count, int grid, hipStream_t stream);
hipError_t launch_class2(const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         int* ovf_list, int* ovf_count, int grid, hipStream_t stream);
hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           hipStream_t stream);

}  // namespace cmpc
