// cmpc_quadprog.hip — batched Goldfarb-Idnani dual active-set QP (include/cmpc_quadprog.h): the
// QuadProg++ solve_quadprog of WBIC::MakeTorque (be2r_cmpc_unitree/src/controllers/WBC/WBIC/
// WBIC.cpp:91; third_party/Goldfarb_Optimizer/QuadProg++.cc:108-507), fp64.
//
// MI355X mapping: ONE WAVEFRONT PER PROBLEM, four problems per 256-thread workgroup. WBIC's QPs
// are tiny (n <= 18 variables, 6 equalities, <= 24 inequalities), so the whole working state of
// a problem — J (n x n), R (n x n, aliased by the Cholesky factor during preprocessing) and the
// vectors — sits in that wave's slice of LDS (about 7.5 KB at n = 18, so 20 waves per CU), and
// every step of the method is lane-parallel over one index and serial over the other:
//   compute_d  lane c: d_c = sum_j J[j][c] np_j          (rows of J broadcast, column per lane)
//   update_z   lane i: z_i = sum_{j >= iq} J[i][j] d_j   (row per lane)
//   Givens     lane k rotates its row's two entries of J (add / drop) or R's two rows (drop)
//   update_r   column-oriented back substitution: lane k accumulates R[k][i] r_i
//   scalar products: a 64-lane xor-butterfly, identical on every lane
// The HBM traffic is one read of (G, g0, CE, ce0) per problem, CI / ci0 re-read per outer
// iteration from L2, and n + 1 doubles written: the kernel is latency-bound on the serial
// chain of the active-set loop, not on bandwidth or the VALU.
//
// Every operation follows oracle/quadprog_oracle.c in the same order without contraction, so
// the kernel reproduces the oracle bit for bit (tests/test_quadprog.py); the few places where
// that order differs from QuadProg++'s serial loops are listed in the oracle's header.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/cmpc_quadprog.h"

#pragma clang fp contract(off)

namespace cmpc {
void set_last_error(const char* msg);  // cmpc_abi.cpp
namespace {

constexpr double kEps = 2.220446049250313e-16;  // std::numeric_limits<double>::epsilon()
constexpr int kQpWaves = 4;

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) v = v + __shfl_xor(v, k);
  return v;
}

// first minimum in index order: (v, i) pairs; lanes without a candidate pass (inf, big)
__device__ __forceinline__ void wargmin(double& v, int& i) {
#pragma unroll
  for (int k = 32; k >= 1; k >>= 1) {
    const double ov = __shfl_xor(v, k);
    const int oi = __shfl_xor(i, k);
    if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
  }
}

// QuadProg++.cc:700-717
__device__ __forceinline__ double qp_dist(double a, double b) {
  const double a1 = fabs(a), b1 = fabs(b);
  if (a1 > b1) { const double t = b1 / a1; return a1 * sqrt(1.0 + t * t); }
  if (b1 > a1) { const double t = a1 / b1; return b1 * sqrt(1.0 + t * t); }
  return a1 * sqrt(2.0);
}

struct QpLds {
  double* J;   // [nm][ld]
  double* R;   // [nm][ld] (Cholesky factor during preprocessing)
  double *x, *z, *d, *np, *xo;   // [nm]
  double *r, *u, *uo;            // [mp]
  double* s;                     // [mm]
  int *A, *Ao;                   // [mp]
  int *iai, *iaex;               // [mm]
};

__host__ __device__ inline int qp_ld(int nm) { return nm + 1; }
__host__ __device__ inline size_t qp_wave_bytes(int nm, int pm, int mm) {
  const int mp = pm + mm;
  const size_t dbl = 2 * (size_t)nm * qp_ld(nm) + 5 * (size_t)nm + 3 * (size_t)mp + (size_t)mm;
  const size_t ints = 2 * (size_t)mp + 2 * (size_t)mm;
  return (dbl * 8 + ints * 4 + 15) & ~(size_t)15;
}

__device__ __forceinline__ double ld_dot(const double* a, const double* b, int n, int lane) {
  const double t = (lane < n) ? a[lane] * b[lane] : 0.0;
  return wsum(t);
}

// d = J' np (:509-522), lane c
__device__ __forceinline__ void qp_compute_d(const QpLds& w, int n, int ld, int lane) {
  if (lane < n) {
    double sum = 0.0;
    for (int j = 0; j < n; j++) sum += w.J[j * ld + lane] * w.np[j];
    w.d[lane] = sum;
  }
  wsync();
}

// z = J[:, iq:] d[iq:] (:524-535), lane i
__device__ __forceinline__ void qp_update_z(const QpLds& w, int n, int ld, int iq, int lane) {
  if (lane < n) {
    double sum = 0.0;
    for (int j = iq; j < n; j++) sum += w.J[lane * ld + j] * w.d[j];
    w.z[lane] = sum;
  }
  wsync();
}

// r = R^-1 d (:537-550), column-oriented: lane k keeps acc_k
__device__ __forceinline__ void qp_update_r(const QpLds& w, int ld, int iq, int lane) {
  double acc = 0.0;
  for (int i = iq - 1; i >= 0; i--) {
    if (lane == i) w.r[i] = (w.d[i] - acc) / w.R[i * ld + i];
    wsync();
    const double ri = w.r[i];
    if (lane < i) acc += w.R[lane * ld + i] * ri;
  }
  wsync();
}

// add_constraint (:552-621); returns false when the new column is degenerate
__device__ __forceinline__ bool qp_add(const QpLds& w, int n, int ld, int& iq, double& rnorm,
                                       int lane) {
  if (n - 1 >= iq + 1) {
    double carry = w.d[n - 1];   // the current d[j]
    for (int j = n - 1; j >= iq + 1; j--) {
      double cc = w.d[j - 1], ss = carry;
      const double h = qp_dist(cc, ss);
      if (fabs(h) < kEps) {
        if (lane == 0) w.d[j] = carry;
        carry = cc;
        continue;
      }
      if (lane == 0) w.d[j] = 0.0;
      ss = ss / h;
      cc = cc / h;
      double dj1;
      if (cc < 0.0) { cc = -cc; ss = -ss; dj1 = -h; } else { dj1 = h; }
      carry = dj1;
      const double xny = ss / (1.0 + cc);
      if (lane < n) {
        double* Jr = w.J + lane * ld;
        const double t1 = Jr[j - 1], t2 = Jr[j];
        const double a = t1 * cc + t2 * ss;
        Jr[j - 1] = a;
        Jr[j] = xny * (t1 + a) - t2;
      }
    }
    if (lane == 0) w.d[iq] = carry;
    wsync();
  }
  iq++;
  if (lane < iq) w.R[lane * ld + (iq - 1)] = w.d[lane];
  wsync();
  const double dl = fabs(w.d[iq - 1]);
  if (dl <= kEps * rnorm) return false;
  rnorm = fmax(rnorm, dl);
  return true;
}

// delete_constraint (:623-698)
__device__ void qp_delete(const QpLds& w, int n, int ld, int p, int& iq, int l, int lane) {
  // qq = first active position >= p holding l
  int qq = 0x7fffffff;
  for (int b = 0; b < CMPC_QP_NMAX + 1; b += 64) {  // active positions < iq <= n
    const int i = b + lane;
    const bool hit = (i >= p && i < iq && w.A[i] == l);
    const unsigned long long m = __ballot(hit);
    if (m != 0ull && qq == 0x7fffffff) qq = b + __ffsll((long long)m) - 1;
    if (b + 64 >= iq) break;
  }
  if (qq == 0x7fffffff) return;
  // shift positions qq+1 .. iq down by one (A, u: read all, then write; R columns: per row)
  {
    int a0 = 0, a1 = 0;
    double u0 = 0.0, u1 = 0.0;
    const int i0 = lane, i1 = lane + 64;
    if (i0 >= qq && i0 < iq) { a0 = w.A[i0 + 1]; u0 = w.u[i0 + 1]; }
    if (i1 >= qq && i1 < iq) { a1 = w.A[i1 + 1]; u1 = w.u[i1 + 1]; }
    wsync();
    if (i0 >= qq && i0 < iq) { w.A[i0] = a0; w.u[i0] = u0; }
    if (i1 >= qq && i1 < iq) { w.A[i1] = a1; w.u[i1] = u1; }
    if (lane == 0) { w.A[iq] = 0; w.u[iq] = 0.0; }
    if (lane < n) {
      double* Rr = w.R + lane * ld;
      for (int i = qq; i < iq - 1; i++) Rr[i] = Rr[i + 1];
      if (lane < iq) Rr[iq - 1] = 0.0;
    }
    wsync();
  }
  iq--;
  if (iq == 0) return;
  for (int j = qq; j < iq; j++) {
    double cc = w.R[j * ld + j], ss = w.R[(j + 1) * ld + j];
    const double h = qp_dist(cc, ss);
    if (fabs(h) < kEps) continue;
    cc = cc / h;
    ss = ss / h;
    wsync();
    if (lane == 0) {
      w.R[(j + 1) * ld + j] = 0.0;
      w.R[j * ld + j] = (cc < 0.0) ? -h : h;
    }
    if (cc < 0.0) { cc = -cc; ss = -ss; }
    const double xny = ss / (1.0 + cc);
    const int k = lane;
    if (k > j && k < iq) {
      const double t1 = w.R[j * ld + k], t2 = w.R[(j + 1) * ld + k];
      const double a = t1 * cc + t2 * ss;
      w.R[j * ld + k] = a;
      w.R[(j + 1) * ld + k] = xny * (t1 + a) - t2;
    }
    if (k < n) {
      double* Jr = w.J + k * ld;
      const double t1 = Jr[j], t2 = Jr[j + 1];
      const double a = t1 * cc + t2 * ss;
      Jr[j] = a;
      Jr[j + 1] = xny * (a + t1) - t2;
    }
    wsync();
  }
}

__global__ __launch_bounds__(64 * kQpWaves) void cmpc_quadprog_kernel(
    int batch, int nm, int pm, int mm, const int32_t* __restrict__ dims,
    const double* __restrict__ Gg, const double* __restrict__ g0g, const double* __restrict__ CEg,
    const double* __restrict__ ce0g, const double* __restrict__ CIg, const double* __restrict__ ci0g,
    int max_iter, double* __restrict__ xg, double* __restrict__ fg, uint8_t* __restrict__ stg,
    int32_t* __restrict__ itg) {
  extern __shared__ __align__(16) unsigned char qp_smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * kQpWaves + wave;
  if (b >= batch) return;
  const int ld = qp_ld(nm), mp = pm + mm;
  QpLds w;
  {
    unsigned char* base = qp_smem + (size_t)wave * qp_wave_bytes(nm, pm, mm);
    double* dp = reinterpret_cast<double*>(base);
    w.J = dp; dp += nm * ld;
    w.R = dp; dp += nm * ld;
    w.x = dp; dp += nm;
    w.z = dp; dp += nm;
    w.d = dp; dp += nm;
    w.np = dp; dp += nm;
    w.xo = dp; dp += nm;
    w.r = dp; dp += mp;
    w.u = dp; dp += mp;
    w.uo = dp; dp += mp;
    w.s = dp; dp += mm;
    int* ip_ = reinterpret_cast<int*>(dp);
    w.A = ip_; ip_ += mp;
    w.Ao = ip_; ip_ += mp;
    w.iai = ip_; ip_ += mm;
    w.iaex = ip_;
  }
  int n = nm, p = pm, m = mm;
  if (dims) {
    n = __builtin_amdgcn_readfirstlane(dims[3 * b]);
    p = __builtin_amdgcn_readfirstlane(dims[3 * b + 1]);
    m = __builtin_amdgcn_readfirstlane(dims[3 * b + 2]);
  }
  const double* G = Gg + (size_t)b * nm * nm;
  const double* g0 = g0g + (size_t)b * nm;
  const double* CE = CEg + (size_t)b * nm * pm;
  const double* ce0 = ce0g + (size_t)b * pm;
  const double* CI = CIg + (size_t)b * nm * mm;
  const double* ci0 = ci0g + (size_t)b * mm;
  double* xout = xg + (size_t)b * nm;
  const double inf = __builtin_inf();
  int status = CMPC_OK, iter = 0;
  double f = 0.0;
  if (n < 1 || n > nm || p < 0 || p > pm || p > n || m < 0 || m > mm) {
    status = CMPC_BAD_INPUT;
    goto done;
  }
  {
    double* L = w.R;  // the Cholesky factor lives where R will
    if (lane < n)
      for (int i = 0; i < n; i++) L[i * ld + lane] = G[i * nm + lane];
    wsync();
    const double c1 = wsum(lane < n ? L[lane * ld + lane] : 0.0);
    // cholesky_decomposition (:731-762), row i at a time, lane j >= i
    for (int i = 0; i < n; i++) {
      double sum = 0.0;
      if (lane >= i && lane < n) {
        sum = L[i * ld + lane];
        for (int k = i - 1; k >= 0; k--) sum -= L[i * ld + k] * L[lane * ld + k];
      }
      const bool bad = __ballot(lane == i && sum <= 0.0) != 0ull;
      if (bad) { status = CMPC_NOT_PD; f = inf; goto done; }
      if (lane == i) L[i * ld + i] = sqrt(sum);
      wsync();
      const double dii = L[i * ld + i];
      if (lane > i && lane < n) L[lane * ld + i] = sum / dii;
      wsync();
      if (lane > i && lane < n) L[i * ld + lane] = L[lane * ld + i];
      wsync();
    }
    // J = L^-T (:194-204): lane i forward-eliminates e_i into row i of J
    if (lane < n) {
      double* Jr = w.J + lane * ld;
      for (int rr = 0; rr < n; rr++) {
        double v = (rr == lane) ? 1.0 : 0.0;
        for (int j = 0; j < rr; j++) v -= L[rr * ld + j] * Jr[j];
        Jr[rr] = v / L[rr * ld + rr];
      }
    }
    wsync();
    const double c2 = wsum(lane < n ? w.J[lane * ld + lane] : 0.0);
    // x = -G^-1 g0 (:216-217): forward then backward elimination, serial in lane 0
    if (lane == 0) {
      double* y = w.z;
      for (int i = 0; i < n; i++) {
        double v = g0[i];
        for (int j = 0; j < i; j++) v -= L[i * ld + j] * y[j];
        y[i] = v / L[i * ld + i];
      }
      for (int i = n - 1; i >= 0; i--) {
        double v = y[i];
        for (int j = i + 1; j < n; j++) v -= L[i * ld + j] * w.x[j];
        w.x[i] = v / L[i * ld + i];
      }
    }
    wsync();
    if (lane < n) w.x[lane] = -w.x[lane];
    wsync();
    f = 0.5 * wsum(lane < n ? g0[lane] * w.x[lane] : 0.0);
    // R = 0 (:186-191), u = r = 0, A = 0
    if (lane < n)
      for (int i = 0; i < n; i++) w.R[i * ld + lane] = 0.0;
    for (int i = lane; i < mp; i += 64) { w.u[i] = 0.0; w.r[i] = 0.0; w.A[i] = 0; }
    wsync();
    double rnorm = 1.0;
    int iq = 0;
    // equality constraints (:225-266)
    for (int i = 0; i < p; i++) {
      if (lane < n) w.np[lane] = CE[lane * pm + i];
      wsync();
      qp_compute_d(w, n, ld, lane);
      qp_update_z(w, n, ld, iq, lane);
      qp_update_r(w, ld, iq, lane);
      const double zz = ld_dot(w.z, w.z, n, lane), znp = ld_dot(w.z, w.np, n, lane);
      const double npx = ld_dot(w.np, w.x, n, lane);
      double t2 = 0.0;
      if (fabs(zz) > kEps) t2 = (-npx - ce0[i]) / znp;
      if (lane < n) w.x[lane] += t2 * w.z[lane];
      if (lane < iq) w.u[lane] -= t2 * w.r[lane];
      if (lane == 0) { w.u[iq] = t2; w.A[i] = -i - 1; }
      f += 0.5 * (t2 * t2) * znp;
      wsync();
      if (!qp_add(w, n, ld, iq, rnorm, lane)) { status = CMPC_BAD_INPUT; goto done; }
    }
    for (int i = lane; i < m; i += 64) w.iai[i] = i;
    wsync();
    int ip = 0;
    double ss = 0.0;
    for (;;) {  // l1 (:272)
      if (++iter > max_iter) { status = CMPC_MAX_ITER; iter--; goto done; }
      if (lane == 0)
        for (int i = p; i < iq; i++) w.iai[w.A[i]] = -1;
      wsync();
      ss = 0.0;
      ip = 0;
      double mins = 0.0;
      for (int i0 = 0; i0 < m; i0 += 64) {
        const int i = i0 + lane;
        if (i < m) {
          w.iaex[i] = 1;
          double sum = 0.0;
          for (int j = 0; j < n; j++) sum += CI[j * mm + i] * w.x[j];
          sum += ci0[i];
          w.s[i] = sum;
          if (i0 == 0) mins = fmin(0.0, sum);
        }
      }
      const double psi = wsum(mins);  // m <= 64
      wsync();
      if (fabs(psi) <= m * kEps * c1 * c2 * 100.0) { status = CMPC_OK; goto done; }
      for (int i = lane; i < iq; i += 64) { w.uo[i] = w.u[i]; w.Ao[i] = w.A[i]; }
      if (lane < n) w.xo[lane] = w.x[lane];
      wsync();
      bool go_l1 = false;
      while (!go_l1) {  // l2 (:320)
        {
          double bv = inf;
          int bi = 0x7fffffff;
          for (int i0 = 0; i0 < m; i0 += 64) {
            const int i = i0 + lane;
            if (i < m && w.s[i] < ss && w.iai[i] != -1 && w.iaex[i] && (w.s[i] < bv)) {
              bv = w.s[i];
              bi = i;
            }
          }
          wargmin(bv, bi);
          if (bi != 0x7fffffff) { ss = bv; ip = bi; }
        }
        if (ss >= 0.0) { status = CMPC_OK; goto done; }
        if (lane < n) w.np[lane] = CI[lane * mm + ip];
        if (lane == 0) { w.u[iq] = 0.0; w.A[iq] = ip; }
        wsync();
        for (;;) {  // l2a (:349)
          if (++iter > max_iter) { status = CMPC_MAX_ITER; iter--; goto done; }
          qp_compute_d(w, n, ld, lane);
          qp_update_z(w, n, ld, iq, lane);
          qp_update_r(w, ld, iq, lane);
          // t1: first minimum of u_k / r_k over r_k > 0, k in [p, iq)
          double t1 = inf;
          int l = 0;
          {
            double bv = inf;
            int bk = 0x7fffffff;
            for (int k0 = 0; k0 < iq; k0 += 64) {
              const int k = k0 + lane;
              if (k >= p && k < iq && w.r[k] > 0.0) {
                const double qv = w.u[k] / w.r[k];
                if (qv < bv) { bv = qv; bk = k; }
              }
            }
            wargmin(bv, bk);
            if (bk != 0x7fffffff && bv < inf) { t1 = bv; l = w.A[bk]; }
          }
          const double zz = ld_dot(w.z, w.z, n, lane), znp = ld_dot(w.z, w.np, n, lane);
          double t2;
          if (fabs(zz) > kEps) {
            t2 = -w.s[ip] / znp;
            if (t2 < 0) t2 = inf;
          } else {
            t2 = inf;
          }
          const double t = fmin(t1, t2);
          if (t >= inf) { status = CMPC_INFEASIBLE; f = inf; goto done; }
          if (t2 >= inf) {  // (ii) step in dual space, drop l
            if (lane < iq) w.u[lane] -= t * w.r[lane];
            wsync();
            if (lane == 0) { w.u[iq] += t; w.iai[l] = l; }
            wsync();
            qp_delete(w, n, ld, p, iq, l, lane);
            continue;
          }
          // (iii) step in primal and dual space
          if (lane < n) w.x[lane] += t * w.z[lane];
          f += t * znp * (0.5 * t + w.u[iq]);
          wsync();
          if (lane < iq) w.u[lane] -= t * w.r[lane];
          wsync();
          if (lane == 0) w.u[iq] += t;
          wsync();
          if (fabs(t - t2) < kEps) {  // full step: add ip
            if (!qp_add(w, n, ld, iq, rnorm, lane)) {
              if (lane == 0) w.iaex[ip] = 0;
              wsync();
              qp_delete(w, n, ld, p, iq, ip, lane);
              for (int i = lane; i < m; i += 64) w.iai[i] = i;
              wsync();
              if (lane == 0)
                for (int i = p; i < iq; i++) { w.A[i] = w.Ao[i]; w.u[i] = w.uo[i]; w.iai[w.A[i]] = -1; }
              if (lane < n) w.x[lane] = w.xo[lane];
              wsync();
              break;  // goto l2
            }
            if (lane == 0) w.iai[ip] = -1;
            wsync();
            go_l1 = true;
            break;
          }
          // partial step: drop l, refresh s[ip]
          if (lane == 0) w.iai[l] = l;
          wsync();
          qp_delete(w, n, ld, p, iq, l, lane);
          if (lane == 0) {
            double sum = 0.0;
            for (int k = 0; k < n; k++) sum += CI[k * mm + ip] * w.x[k];
            w.s[ip] = sum + ci0[ip];
          }
          wsync();
        }
      }
    }
  }
done:
  wsync();
  if (lane < nm) xout[lane] = (status == CMPC_OK && lane < n) ? w.x[lane] : 0.0;
  if (lane == 0) {
    fg[b] = (status == CMPC_OK) ? f : ((status == CMPC_INFEASIBLE || status == CMPC_NOT_PD) ? inf : f);
    stg[b] = (uint8_t)status;
    if (itg) itg[b] = iter;
  }
}

}  // namespace
}  // namespace cmpc

extern "C" int cmpc_batch_quadprog(cmpc_batch* h, int n_max, int p_max, int m_max,
                                   const int32_t* d_dims, const double* d_G, const double* d_g0,
                                   const double* d_CE, const double* d_ce0, const double* d_CI,
                                   const double* d_ci0, int max_iter, double* d_x, double* d_f,
                                   uint8_t* d_status, int32_t* d_iters, int batch) {
  if (!h || batch < 0 || n_max < 1 || n_max > CMPC_QP_NMAX || p_max < 0 || p_max > n_max ||
      m_max < 1 || m_max > CMPC_QP_MMAX || max_iter < 1 ||
      (batch && (!d_G || !d_g0 || (p_max && (!d_CE || !d_ce0)) || !d_CI || !d_ci0 || !d_x ||
                 !d_f || !d_status))) {
    cmpc::set_last_error("cmpc_batch_quadprog: bad arguments");
    return -1;
  }
  if (batch == 0) return 0;
  hipStream_t stream = static_cast<hipStream_t>(cmpc_batch_stream(h));
  const size_t lds = cmpc::kQpWaves * cmpc::qp_wave_bytes(n_max, p_max, m_max);
  const int grid = (batch + cmpc::kQpWaves - 1) / cmpc::kQpWaves;
  hipLaunchKernelGGL(cmpc::cmpc_quadprog_kernel, dim3(grid), dim3(64 * cmpc::kQpWaves), lds, stream,
                     batch, n_max, p_max, m_max, d_dims, d_G, d_g0, d_CE, d_ce0, d_CI, d_ci0,
                     max_iter, d_x, d_f, d_status, d_iters);
  if (hipGetLastError() != hipSuccess) {
    cmpc::set_last_error("cmpc_batch_quadprog: launch failed");
    return -1;
  }
  return 0;
}
