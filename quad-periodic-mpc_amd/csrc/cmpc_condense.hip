// cmpc_condense.hip — parity hook: full (no elimination) qH / qg per instance
#include "cmpc_device.h"

namespace cmpc {

template <int W>
__global__ __launch_bounds__(64 * W) void cmpc_condense_kernel(const float* __restrict__ recs,
                                                               int batch, KParams P,
                                                               float* __restrict__ H,
                                                               float* __restrict__ g) {
  __shared__ Shared<W> sh;
  const int nv = 12 * P.N;
  for (int inst = blockIdx.x; inst < batch; inst += gridDim.x) {
    solve_instance<W>(recs + (size_t)inst * P.rec_words, P, sh, nullptr, nullptr, nullptr, nullptr,
                      nullptr, inst, H + (size_t)inst * nv * nv, g + (size_t)inst * nv);
    __syncthreads();
  }
}

hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  const int nv = 12 * P.N;
  if (nv <= 64)
    hipLaunchKernelGGL(cmpc_condense_kernel<1>, dim3(batch), dim3(64), 0, stream, d_recs, batch, P, d_H, d_g);
  else if (nv <= 128)
    hipLaunchKernelGGL(cmpc_condense_kernel<2>, dim3(batch), dim3(128), 0, stream, d_recs, batch, P, d_H, d_g);
  else
    return hipErrorInvalidValue;  // 12N > 128 needs the 4-wave class (not built yet)
  return hipGetLastError();
}

}  // namespace cmpc
