// cmpc_launch.hip — orchestration of the size classes for one batch solve (host code).
#include "cmpc_kernels.h"

namespace cmpc {

hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        hipStream_t stream, hipEvent_t* ev) {
  // d_work layout: [0] overflow count of class 1, [1] of class 2, [4 ..) lists [max_batch] x 2
  int* cnt1 = d_work;
  int* list1 = d_work + 4;
  hipError_t e = hipMemsetAsync(d_work, 0, 4 * sizeof(int), stream);
  if (e != hipSuccess) return e;
  if (batch <= 0) return hipSuccess;
  if (ev) (void)hipEventRecord(ev[0], stream);
  // class 1: one 64-thread workgroup per instance; instances with > 64 stance variables are
  // appended to list1
  e = launch_class1(d_recs, batch, P, d_forces, d_status, d_iters, nullptr, nullptr, list1, cnt1,
                    batch, stream);
  if (e != hipSuccess) return e;
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (12 * P.N > 64) {
    // class 2: persistent grid of 128-thread workgroups over list1
    const int g2 = batch < 2048 ? batch : 2048;
    e = launch_class2(d_recs, batch, P, d_forces, d_status, d_iters, list1, cnt1, nullptr, nullptr,
                      g2, stream);
  }
  if (ev) (void)hipEventRecord(ev[2], stream);
  return e;
}

}  // namespace cmpc
