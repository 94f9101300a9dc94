// cmpc_launch.hip — orchestration of the size classes for one batch solve (host code).
//   class 1 (cmpc_class1.hip): every instance, one wavefront each; n > 64  -> list 1
//   class 2 (cmpc_class2.hip): one 128-lane workgroup per list-1 entry; n > 128 -> list 2
//   class G (cmpc_classg.hip): persistent 256-lane workgroups over list 2 (any n)
#include "cmpc_kernels.h"

namespace cmpc {

hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        float* d_gscratch, hipStream_t stream, hipEvent_t* ev) {
  // d_work layout: [0] count of list 1, [1] count of list 2, [4 ..) list 1, then list 2
  int* cnt1 = d_work;
  int* cnt2 = d_work + 1;
  int* list1 = d_work + 4;
  int* list2 = d_work + 4 + max_batch;
  hipError_t e = hipMemsetAsync(d_work, 0, 4 * sizeof(int), stream);
  if (e != hipSuccess) return e;
  if (batch <= 0) return hipSuccess;
  if (ev) (void)hipEventRecord(ev[0], stream);
  e = launch_class1(d_recs, batch, P, d_forces, d_status, d_iters, nullptr, nullptr, list1, cnt1,
                    batch, stream);
  if (e != hipSuccess) return e;
  if (ev) (void)hipEventRecord(ev[1], stream);
  if (12 * P.N > 64) {
    // one workgroup per possible list-1 entry; surplus workgroups exit after one load
    e = launch_class2(d_recs, batch, P, d_forces, d_status, d_iters, list1, cnt1, list2, cnt2, batch,
                      stream);
    if (e != hipSuccess) return e;
  }
  if (12 * P.N > 128) {
    e = launch_classg(d_recs, batch, P, d_forces, d_status, d_iters, list2, cnt2, d_gscratch,
                      classg_grid(max_batch), stream);
  }
  if (ev) (void)hipEventRecord(ev[2], stream);
  return e;
}

}  // namespace cmpc
