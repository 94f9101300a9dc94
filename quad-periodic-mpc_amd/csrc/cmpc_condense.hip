// cmpc_condense.hip — parity hook for the condensation rows (SolverMPC.cpp:96-146, 806-814) and
// the condensation stage of the JCQP paths (use_jcqp == 1 / 2): the full reduced-free qH [12N x
// 12N] and qg [12N] of every instance, all variables kept (no swing elimination), by the same
// structured recursions as the solver kernels (cmpc_common.h) — never forming A_qp, B_qp or the
// dense 13N x 13N weight matrix S. One 256-thread workgroup per instance, grid-strided; the
// symmetric H is written straight to the caller's buffer.
#include "cmpc_common.h"

namespace cmpc {
namespace {

constexpr int NTG = 256;

struct SharedC {
  float BdtT[12][16];
  float traj[12 * MAXN];
  float E[MAXN][16];
  float ZE[MAXN][16];
};

// One instance: H [n x n] row-major (n = 12 N) and g [n] of rec.
__device__ void condense_one(const float* __restrict__ rec, const KParams& P, SharedC& sh,
                             float* __restrict__ H, float* __restrict__ g) {
  const int tid = threadIdx.x;
  const int N = P.N;
  const int n = 12 * N;
  for (int t = tid; t < 12 * N; t += NTG) sh.traj[t] = rec[CMPC_REC_HDR + t];
  Model md;
  make_model(rec, P.dt, md);
  make_bdt<NTG>(rec, md, tid, sh.BdtT);
  __syncthreads();
  if (tid < N) {
    float e[13];
    state_error(rec, md, tid, &sh.traj[12 * tid], e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.E[tid][j] = e[j];
  }
  __syncthreads();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  if (tid < 64) {
    float ze[13];
#pragma unroll
    for (int j = 0; j < 13; j++) ze[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      float e[13];
#pragma unroll
      for (int j = 0; j < 13; j++) e[j] = sh.E[i][j];
      recur(md, wts, e, ze);
      if ((tid & 63) == 0) {
#pragma unroll
        for (int j = 0; j < 13; j++) sh.ZE[i][j] = ze[j];
      }
    }
  }
  __syncthreads();
  // variable v = 12 k + c (every foot-step kept): row v by the backward recursion of its column
  for (int v = tid; v < n; v += NTG) {
    const int kv = v / 12, cv = v - 12 * (v / 12);
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = sh.BdtT[cv][j];
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.ZE[kv][j];
      g[v] = 2.f * dot13(b, zk);  // qg = 2 B_qp' S (A_qp x0 + Q_qp f - X_d)
    }
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    for (int i = N - 1; i >= kv; i--) {
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = fmaf(k2, u2[j], fmaf(k, u1[j], b[j]));
      recur(md, wts, gk, z);
      for (int w = max(12 * i, v); w < 12 * i + 12; w++) {
        float bw[13];
#pragma unroll
        for (int j = 0; j < 13; j++) bw[j] = sh.BdtT[w - 12 * i][j];
        float val = 2.f * dot13(bw, z);
        if (w == v) val += P.alpha2;  // qH = 2 (B'SB + alpha I), SolverMPC.cpp:806
#ifdef CMPC_DIAG_PERTURB  // diagnostic builds only: a deliberately wrong qH (shows the parity gate fails)
        val *= 1.f + CMPC_DIAG_PERTURB;
#endif
        H[(size_t)v * n + w] = val;
        H[(size_t)w * n + v] = val;
      }
    }
  }
}

__global__ __launch_bounds__(NTG) void cmpc_condense_kernel(const float* __restrict__ recs, int batch, KParams P,
                                                            float* __restrict__ Hout, float* __restrict__ gout) {
  __shared__ SharedC sh;
  const size_t n = 12 * (size_t)P.N;
  for (int inst = blockIdx.x; inst < batch; inst += gridDim.x) {
    condense_one(recs + (size_t)inst * P.rec_words, P, sh, Hout + inst * n * n, gout + inst * n);
    __syncthreads();
  }
}

}  // namespace

hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  const int grid = batch < 2048 ? batch : 2048;
  hipLaunchKernelGGL(cmpc_condense_kernel, dim3(grid), dim3(NTG), 0, stream, d_recs, batch, P, d_H, d_g);
  return hipGetLastError();
}

}  // namespace cmpc
