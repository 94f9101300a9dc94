// cmpc_class1.hip — register-resident size class W=1 (n <= 64 reduced variables)
#include "cmpc_device.h"

namespace cmpc {

#ifndef CMPC_W1_WAVES_PER_EU
#define CMPC_W1_WAVES_PER_EU 2  // 2 waves/SIMD: measured best (r01: 6.1 ms vs 10.2 at 1, 9.5 at 3 with spills)
#endif
// Register-resident size classes. Class W handles instances with n <= 64 W reduced variables;
// class 1 runs one workgroup per instance over the batch, wider classes run a persistent grid
// over the overflow list of the previous class.
template <int W>
__global__ __launch_bounds__(64 * W, (W == 1 ? CMPC_W1_WAVES_PER_EU : 1)) void cmpc_solve_reg_kernel(
    const float* __restrict__ recs, int batch, KParams P, float* __restrict__ forces,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, const int* __restrict__ in_list,
    const int* __restrict__ in_count, int* __restrict__ ovf_list, int* __restrict__ ovf_count) {
  __shared__ SharedReg<W> sh;
  const int count = in_list ? *in_count : batch;
  for (int t = blockIdx.x; t < count; t += gridDim.x) {
    const int inst = in_list ? in_list[t] : t;
    solve_reg<W>(recs + (size_t)inst * P.rec_words, P, sh, forces + (size_t)inst * 12 * P.N,
                 status + inst, iters ? iters + inst : nullptr, ovf_list, ovf_count, inst);
    __syncthreads();
  }
}

hipError_t launch_class1(const float* d_recs, int batch, const KParams& P, float* d_forces,
                          uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                          int* ovf_list, int* ovf_count, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(cmpc_solve_reg_kernel<1>, dim3(grid), dim3(64), 0, stream, d_recs, batch, P,
                     d_forces, d_status, d_iters, in_list, in_count, ovf_list, ovf_count);
  return hipGetLastError();
}

}  // namespace cmpc
