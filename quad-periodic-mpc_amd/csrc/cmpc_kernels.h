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
  int max_iter;    // active-set cap; the kernels allow max_iter + 2 n
  int pad;
};

// Scratch ints needed by launch_solve for max_batch instances.
inline size_t work_ints(int max_batch) { return 4 + 3 * (size_t)max_batch; }
// Workgroups of the general class (persistent over its overflow list) and its global slabs.
inline int classg_grid(int max_batch) { return max_batch < 512 ? max_batch : 512; }
size_t classg_scratch_floats(int horizon, int grid);

// ev (optional): 3 events recorded around the size-class launches
// (ev[0] before class 1, ev[1] between class 1 and the wider classes, ev[2] after them).
hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        float* d_gscratch, hipStream_t stream, hipEvent_t* ev = nullptr);
// per-class launchers (cmpc_class1.hip, cmpc_class2.hip, cmpc_classg.hip)
hipError_t launch_class1(const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         int* ovf_list, int* ovf_count, int grid, hipStream_t stream);
// width: row width of the 2-wavefront class, 96 (class 2a) or 128 (class 2b)
hipError_t launch_class2(int width, const float* d_recs, int batch, const KParams& P,
                         float* d_forces, uint8_t* d_status, int32_t* d_iters, const int* in_list,
                         const int* in_count, int* ovf_list, int* ovf_count, int grid,
                         hipStream_t stream);
hipError_t launch_classg(const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         float* scratch, int grid, hipStream_t stream);
// config 5 estimator (cmpc_estimator.hip). d_gauss: the two normalised float Gaussian kernels
// of gaussian_filter (sigma 7: 43 taps, then sigma 27: 163 taps), built on the host exactly as
// SolverMPC.cpp:404-418 builds them.
constexpr int kGaussR7 = 21;   // ceil(3 * 7)
constexpr int kGaussR27 = 81;  // ceil(3 * 27)
constexpr int kGaussTaps = 2 * kGaussR7 + 1 + 2 * kGaussR27 + 1;
hipError_t launch_estimate(float* d_est, const float* d_logs, const float* d_fext3,
                           const float* d_time, float sim_time, float* d_records, int rec_words,
                           float* d_fext6, const float* d_gauss, int batch, hipStream_t stream);
// parity hook: full (nothing eliminated) qH [12N x 12N] / qg [12N] per instance
hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           float* scratch, int grid, hipStream_t stream);

}  // namespace cmpc
