// cmpc_admm.hip — batched JCQP ADMM, the use_jcqp == 1 branch of solve_mpc (SURVEY.md §8(f)
// rank 4; SolverMPC.cpp:818-838 and :1057-1062, third_party/JCQP/QpProblem.cpp:165-381).
//
// One workgroup (256 lanes, 4 wavefronts) per instance, fp64 like QpProblem<double>:
//   P = qH, q = qg (the full fp32 condensation of cmpc_batch_condense, cast to double),
//   A = fmat (20N x 12N, 5x3 friction-pyramid blocks), l = 0, u = U_b (5e10 / gait*f_max).
// computeConstraintInfos (QpProblem.cpp:255-272) picks rho per row: u > infty -> rhoInfty,
// |u - l| < eqlTol (swing fz rows) -> rho*rhoEqualityScale, else rho.
// The KKT system [P + sigma I, A'; A, -diag(1/rho)] is solved through its Schur complement
// M = P + sigma I + A' diag(rho) A (block-diagonal A'rhoA: 3x3 per foot-step), inverted once in
// LDS by Gauss-Jordan (SPD, no pivoting); per iteration xt = M^-1 (sigma xp - q + A'(rho zp - y))
// and zt = A xt, which is what solveLinearSystem's "step!" line produces. stepX / stepZ / stepY
// and the every-10-iterations residual (p + d) / 4 against _zPrev follow QpProblem.cpp:306-381.
// M (n x n doubles) is resident in LDS while n <= 120 (the full QP up to N = 10; the reduced one
// (use_jcqp == 2) while 3 x (stance foot-steps) <= 120, e.g. trot up to N = 20). Larger problems
// (the full QP at N = 11..24, the reference's deployed N = 16 included; reduced QPs with more
// stance foot-steps) keep M in a per-workgroup fp64 slab in global memory (L2-resident: 295 KB at
// n = 192) with the same arithmetic, over a persistent grid of slabs (cmpc_admm_gm_kernel).
#include "cmpc_kernels.h"

namespace cmpc {
namespace {

constexpr int kAdmmThreads = 256;
constexpr int kAdmmMaxN = 10;
constexpr int kNV = 12 * kAdmmMaxN;   // 120 variables
constexpr int kNC = 20 * kAdmmMaxN;   // 200 constraints

struct AdmmParams {
  double rho, sigma, alpha, terminate;
  int max_iter;
  int N;
  int rec_words;
  float mu_inv;
  float f_max;
  int reduced;   // use_jcqp == 2: swing legs eliminated first (SolverMPC.cpp:859-950, 984-1053)
  int out_cols;  // forces kept per instance (cmpc_batch_set_output_steps): the output stride, as
                 // the active-set kernels and cmpc_batch_rollout use it
};

// fmat row k (0..4) of a 5x3 block, column a (SolverMPC.cpp:657-664)
__device__ __forceinline__ double fcoef(int k, int a, double mi) {
  // [[mi,0,1],[-mi,0,1],[0,mi,1],[0,-mi,1],[0,0,1]]
  if (a == 2) return 1.0;
  if (k == 4) return 0.0;
  if (a == 0) return k == 0 ? mi : (k == 1 ? -mi : 0.0);
  return k == 2 ? mi : (k == 3 ? -mi : 0.0);
}

__device__ __forceinline__ double block_max(double v, double* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int s = kAdmmThreads / 2; s > 0; s >>= 1) {
    if (t < s) red[t] = fmax(red[t], red[t + s]);
    __syncthreads();
  }
  double r = red[0];
  __syncthreads();
  return r;
}

// Barrier over the workgroup that also orders M's traffic: with M in a global slab the
// workgroup-scope fences of __syncthreads do not wait for this wave's global stores nor refresh
// the CU's L1, so the agent-scope release (s_waitcnt vmcnt(0), L2 write-back) and acquire (L1
// invalidate) around it publish every store of M to the other waves of the workgroup.
template <bool GM>
__device__ __forceinline__ void msync() {
  if constexpr (GM) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  } else {
    __syncthreads();
  }
}

template <int NV, int NC>
struct AdmmShared {
  double sx[2][NV], sz[2][NV > NC ? NV : NC];
  double sy[NC], sq[NV], srhs[NV], sxt[NV], srho[NC], su[NC];
  double red[kAdmmThreads];
  int smap[4 * CMPC_MAX_HORIZON];   // compact foot-step -> foot-step (variables 3b..)
  int sinv[4 * CMPC_MAX_HORIZON];   // foot-step -> compact, -1 if eliminated
  int snb;
};

// One instance by one workgroup. M: the n x n Schur complement / its inverse, in LDS (n <= 120)
// or in this workgroup's global slab. Returns false (nothing written) when the instance's n is
// outside [n_lo, NV] — another launch owns it.
template <int NV, int NC, bool GM>
__device__ bool admm_solve(const float* __restrict__ recs, const float* __restrict__ gH,
                           const float* __restrict__ gg, const AdmmParams& ap,
                           float* __restrict__ forces, uint8_t* __restrict__ status,
                           int32_t* __restrict__ iters, int inst, double* __restrict__ M,
                           AdmmShared<NV, NC>& sh, int n_lo) {
  double(&sx)[2][NV] = sh.sx;
  auto& sz = sh.sz;
  double* sy = sh.sy;
  double* sq = sh.sq;
  double* srhs = sh.srhs;
  double* sxt = sh.sxt;
  double* srho = sh.srho;
  double* su = sh.su;
  double* red = sh.red;
  int* smap = sh.smap;
  int* sinv = sh.sinv;
  const int t = threadIdx.x;
  const int nf = 12 * ap.N;                    // full variable count = qH stride
  const float* H = gH + (size_t)inst * nf * nf;
  const float* rec = recs + (size_t)inst * ap.rec_words;
  const uint8_t* gait = reinterpret_cast<const uint8_t*>(rec + CMPC_REC_HDR + 12 * ap.N);
  const double mi = (double)ap.mu_inv;
  // Elimination (reduced mode): a foot-step whose fz row has lb = ub = 0 (gait 0) loses its three
  // variables and five rows; the kept ones stay in order (SolverMPC.cpp:859-950)
  __syncthreads();   // the previous instance of a persistent workgroup is done with sh
  if (t == 0) {
    int c = 0;
    for (int b = 0; b < 4 * ap.N; ++b) {
      const bool keep = !ap.reduced || gait[b] != 0;
      sinv[b] = keep ? c : -1;
      if (keep) smap[c++] = b;
    }
    sh.snb = c;
  }
  __syncthreads();
  const int nb = sh.snb, n = 3 * nb, m = 5 * nb;
  if (n > NV || n < n_lo) return false;   // another size class owns this instance

  // ---- setup: P + sigma I, q, u, rho; cold start (QpProblem.cpp:9-20) ----
  for (int e = t; e < n * n; e += kAdmmThreads) {
    const int i = e / n, j = e - i * n;
    const int fi = 3 * smap[i / 3] + i % 3, fj = 3 * smap[j / 3] + j % 3;
    M[e] = (double)H[(size_t)fi * nf + fj] + (i == j ? ap.sigma : 0.0);
  }
  for (int i = t; i < n; i += kAdmmThreads) {
    sq[i] = (double)gg[(size_t)inst * nf + 3 * smap[i / 3] + i % 3];
    sx[0][i] = 0.0;
    sx[1][i] = 0.0;
  }
  for (int r = t; r < m; r += kAdmmThreads) {
    const int b = r / 5, k = r - 5 * b;
    // U_b (SolverMPC.cpp:646-652): 5e10 for the four pyramid rows, gait * f_max for fz
    const double u = k < 4 ? (double)5e10f : (double)((float)gait[smap[b]] * ap.f_max);
    double rho;
    if (u > 1e10) rho = 1e-6;                        // INFINITE: rhoInfty
    else if (fabs(u) < 1e-10) rho = ap.rho * 1e3;   // EQUALITY: rho * rhoEqualityScale
    else rho = ap.rho;
    su[r] = u;
    srho[r] = rho;
    sy[r] = 0.0;
    sz[0][r] = 0.0;
    sz[1][r] = 0.0;
  }
  msync<GM>();
  // A' diag(rho) A: block-diagonal, 3x3 per foot-step b (variables 3b..3b+2, rows 5b..5b+4)
  for (int e = t; e < 9 * (n / 3); e += kAdmmThreads) {
    const int b = e / 9, a0 = (e - 9 * b) / 3, a1 = e - 9 * b - 3 * a0;
    double s = 0.0;
    for (int k = 0; k < 5; ++k) s += srho[5 * b + k] * fcoef(k, a0, mi) * fcoef(k, a1, mi);
    M[(3 * b + a0) * n + 3 * b + a1] += s;
  }
  msync<GM>();

  // ---- Gauss-Jordan inverse in place (SPD: no pivoting) ----
  for (int k = 0; k < n; ++k) {
    const double piv = 1.0 / M[k * n + k];
    for (int j = t; j < n; j += kAdmmThreads)
      if (j != k) M[k * n + j] *= piv;
    msync<GM>();
    for (int e = t; e < n * n; e += kAdmmThreads) {
      const int i = e / n, j = e - i * n;
      if (i != k && j != k) M[e] -= M[i * n + k] * M[k * n + j];
    }
    msync<GM>();
    for (int i = t; i < n; i += kAdmmThreads)
      if (i != k) M[i * n + k] *= -piv;
    if (t == 0) M[k * n + k] = piv;
    msync<GM>();
  }

  // ---- ADMM iterations (runFromDense, QpProblem.cpp:165-225) ----
  const double al = ap.alpha, sg = ap.sigma;
  int cur = 0;                 // sx[cur] / sz[cur] hold _x / _z
  int it_done = ap.max_iter;
  uint8_t st = 1;
  for (int it = 0; it < ap.max_iter; ++it) {
    const int prv = cur;       // stepSetup: swap, the old _x becomes _xPrev
    cur ^= 1;
    const double* xp = sx[prv];
    const double* zp = sz[prv];
    // rhs = sigma xp - q + A'(rho zp - y)
    for (int i = t; i < n; i += kAdmmThreads) {
      const int b = i / 3, a = i - 3 * b;
      double s = sg * xp[i] - sq[i];
      for (int k = 0; k < 5; ++k) {
        const int r = 5 * b + k;
        s += fcoef(k, a, mi) * (srho[r] * zp[r] - sy[r]);
      }
      srhs[i] = s;
    }
    __syncthreads();
    // xt = M^-1 rhs: two adjacent lanes per row, each half of the columns with four
    // independent accumulators (the LDS reads pipeline instead of one serial FMA chain), then a
    // lane-pair shuffle; M^-1 is symmetric, so lanes of a row read down a column
    // (rows beyond 128, the global-slab sizes, take further passes of the 256 lanes)
    for (int b0 = 0; b0 < 2 * n; b0 += kAdmmThreads) {
      const int tt = b0 + t;
      if (tt >= 2 * n) break;
      const int i = tt >> 1, h = tt & 1, half = n >> 1;   // n = 3 x kept foot-steps: may be odd
      const int j0 = h ? half : 0, j1 = h ? n : half;
      double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
      int j = j0;
      for (; j + 4 <= j1; j += 4) {
        a0 += M[(j + 0) * n + i] * srhs[j + 0];
        a1 += M[(j + 1) * n + i] * srhs[j + 1];
        a2 += M[(j + 2) * n + i] * srhs[j + 2];
        a3 += M[(j + 3) * n + i] * srhs[j + 3];
      }
      for (; j < j1; ++j) a0 += M[j * n + i] * srhs[j];
      double s = (a0 + a1) + (a2 + a3);
      s += __shfl_xor(s, 1);
      if (h == 0) {
        sxt[i] = s;
        sx[cur][i] = al * s + (1.0 - al) * xp[i];               // stepX
      }
    }
    __syncthreads();
    for (int r = t; r < m; r += kAdmmThreads) {                 // stepZ, stepY
      const int b = r / 5, k = r - 5 * b;
      double zt = 0.0;
      for (int a = 0; a < 3; ++a) zt += fcoef(k, a, mi) * sxt[3 * b + a];
      const double zr = al * zt + (1.0 - al) * zp[r];
      double z = zr + sy[r] / srho[r];
      if (z < 0.0) z = 0.0;
      if (z > su[r]) z = su[r];
      sz[cur][r] = z;
      sy[r] += srho[r] * (zr - z);
    }
    __syncthreads();
    if ((it + 1) % 10 == 0) {
      // p = |A x - zPrev|_inf, d = |P x + q + A' y|_inf  (calcAndDisplayResidual, dense branch)
      const double* x = sx[cur];
      double pm = 0.0, dm = 0.0;
      for (int r = t; r < m; r += kAdmmThreads) {
        const int b = r / 5, k = r - 5 * b;
        double ax = 0.0;
        for (int a = 0; a < 3; ++a) ax += fcoef(k, a, mi) * x[3 * b + a];
        pm = fmax(pm, fabs(ax - zp[r]));
      }
      for (int i = t; i < n; i += kAdmmThreads) {
        const float* Hi = H + (size_t)(3 * smap[i / 3] + i % 3) * nf;
        double a0 = 0.0, a1 = 0.0, a2 = 0.0;
        for (int c = 0; c < nb; ++c) {     // the kept columns, one foot-step (3 wide) at a time
          const float* h = Hi + 3 * smap[c];
          a0 += (double)h[0] * x[3 * c + 0];
          a1 += (double)h[1] * x[3 * c + 1];
          a2 += (double)h[2] * x[3 * c + 2];
        }
        double s = (a0 + a1) + a2 + sq[i];
        const int b = i / 3, a = i - 3 * b;
        for (int k = 0; k < 5; ++k) s += fcoef(k, a, mi) * sy[5 * b + k];
        dm = fmax(dm, fabs(s));
      }
      const double p = block_max(pm, red);
      const double d = block_max(dm, red);
      const double res = (d + p) / 4;
      if (res < ap.terminate || it + 1 >= ap.max_iter) {
        it_done = it + 1;
        st = res < ap.terminate ? 0 : 1;
        break;
      }
    }
  }
  // q_soln[i] = jcqp.getSolution()[i] (SolverMPC.cpp:1057-1062)
  // q_soln: eliminated variables 0 (reduced), else reducedProblem / jcqp.getSolution()
  // (the leading ap.out_cols of them: 12 N unless the handle keeps fewer steps)
  for (int v = t; v < ap.out_cols; v += kAdmmThreads) {
    const int c = sinv[v / 3];
    forces[(size_t)inst * ap.out_cols + v] = c < 0 ? 0.f : (float)sx[cur][3 * c + v % 3];
  }
  if (t == 0) {
    status[inst] = st;
    if (iters) iters[inst] = it_done;
  }
  return true;
}

__global__ void __launch_bounds__(kAdmmThreads)
cmpc_admm_kernel(const float* __restrict__ recs, const float* __restrict__ gH,
                 const float* __restrict__ gg, AdmmParams ap, float* __restrict__ forces,
                 uint8_t* __restrict__ status, int32_t* __restrict__ iters) {
  __shared__ double M[kNV * kNV];
  __shared__ AdmmShared<kNV, kNC> sh;
  admm_solve<kNV, kNC, false>(recs, gH, gg, ap, forces, status, iters, blockIdx.x, M, sh, 0);
}

// n > 120: M in a global fp64 slab per workgroup, persistent over the batch
constexpr int kGNV = 12 * CMPC_MAX_HORIZON;
constexpr int kGNC = 20 * CMPC_MAX_HORIZON;
__global__ void __launch_bounds__(kAdmmThreads)
cmpc_admm_gm_kernel(const float* __restrict__ recs, const float* __restrict__ gH,
                    const float* __restrict__ gg, AdmmParams ap, float* __restrict__ forces,
                    uint8_t* __restrict__ status, int32_t* __restrict__ iters, int batch,
                    double* __restrict__ slabs) {
  __shared__ AdmmShared<kGNV, kGNC> sh;
  const int nf = 12 * ap.N;
  double* M = slabs + (size_t)blockIdx.x * nf * nf;
  for (int inst = blockIdx.x; inst < batch; inst += gridDim.x)
    admm_solve<kGNV, kGNC, true>(recs, gH, gg, ap, forces, status, iters, inst, M, sh, kNV + 1);
}

}  // namespace

size_t admm_slab_doubles(int horizon) { return (size_t)144 * horizon * horizon; }

hipError_t launch_admm(const float* d_recs, const float* d_H, const float* d_g, int batch,
                       const KParams& P, const cmpc_admm_settings& s, float* d_forces,
                       uint8_t* d_status, int32_t* d_iters, double* d_slabs, int nslabs,
                       hipStream_t stream) {
  if (P.N < 1 || P.N > CMPC_MAX_HORIZON || s.max_iter < 1 || !(s.rho > 0) || !(s.alpha > 0))
    return hipErrorInvalidValue;
  if (batch == 0) return hipSuccess;
  AdmmParams ap{s.rho, s.sigma, s.alpha, s.terminate, s.max_iter, P.N, P.rec_words, P.mu_inv,
                P.f_max, s.reduced ? 1 : 0, P.out_cols};
  if (ap.out_cols < 12 || ap.out_cols > 12 * P.N) return hipErrorInvalidValue;
  const bool small_possible = s.reduced || P.N <= kAdmmMaxN;
  const bool large_possible = 12 * P.N > kNV;
  if (large_possible && (!d_slabs || nslabs < 1)) return hipErrorInvalidValue;
  if (small_possible)
    hipLaunchKernelGGL(cmpc_admm_kernel, dim3(batch), dim3(kAdmmThreads), 0, stream, d_recs, d_H,
                       d_g, ap, d_forces, d_status, d_iters);
  if (large_possible)
    hipLaunchKernelGGL(cmpc_admm_gm_kernel, dim3(batch < nslabs ? batch : nslabs),
                       dim3(kAdmmThreads), 0, stream, d_recs, d_H, d_g, ap, d_forces, d_status,
                       d_iters, batch, d_slabs);
  return hipGetLastError();
}

}  // namespace cmpc
