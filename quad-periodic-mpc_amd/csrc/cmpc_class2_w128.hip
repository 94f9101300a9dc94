// cmpc_class2_w128.hip — size class 2 with 128-wide rows (kernel template: cmpc_class2.h).
#include "cmpc_class2.h"

namespace cmpc {

hipError_t launch_class2_w128(const float* d_recs, const KParams& P, float* d_forces,
                             uint8_t* d_status, int32_t* d_iters, const int* in_list,
                             const int* in_count, int* ovf_list, int* ovf_count, int grid,
                             hipStream_t stream) {
  return launch_class2_impl<128>(d_recs, P, d_forces, d_status, d_iters, in_list, in_count, ovf_list,
                                ovf_count, grid, stream);
}

}  // namespace cmpc
