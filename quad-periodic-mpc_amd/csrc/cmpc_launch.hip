// cmpc_launch.hip — orchestration of the size classes for one batch solve (host code).
//   class 1 (cmpc_class1.hip): every instance, one wavefront each; n > 64  -> list 1
//   class 2a (cmpc_class2.hip, rows of 96): one 128-lane workgroup per list-1 entry; n > 96 -> list 2
//   class 2b (cmpc_class2.hip, rows of 128): one 128-lane workgroup per list-2 entry; n > 128 -> list 3
//   class G (cmpc_classg.hip): persistent 256-lane workgroups over list 3 (any n)
#include "cmpc_kernels.h"

namespace cmpc {

hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        float* d_gscratch, hipStream_t stream, hipEvent_t* ev) {
  // d_work layout: [0..2] counts of lists 1..3, [4 ..) list 1, then list 2, then list 3
  int* cnt1 = d_work;
  int* cnt2 = d_work + 1;
  int* cnt3 = d_work + 2;
  int* list1 = d_work + 4;
  int* list2 = d_work + 4 + max_batch;
  int* list3 = d_work + 4 + 2 * (size_t)max_batch;
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
    e = launch_class2(96, d_recs, batch, P, d_forces, d_status, d_iters, list1, cnt1, list2, cnt2,
                      batch, stream);
    if (e != hipSuccess) return e;
  }
  if (12 * P.N > 96) {
    e = launch_class2(128, d_recs, batch, P, d_forces, d_status, d_iters, list2, cnt2, list3, cnt3,
                      batch, stream);
    if (e != hipSuccess) return e;
  }
  if (12 * P.N > 128) {
    e = launch_classg(d_recs, batch, P, d_forces, d_status, d_iters, list3, cnt3, d_gscratch,
                      classg_grid(max_batch), stream);
  }
  if (ev) (void)hipEventRecord(ev[2], stream);
  return e;
}

}  // namespace cmpc
