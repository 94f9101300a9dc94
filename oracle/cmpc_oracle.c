/*
 * TEST INFRASTRUCTURE ONLY (see cmpc_oracle.h). Reference-faithful CPU restatement of
 * SolverMPC.cpp:566-982 for one MPC instance. Every function cites the reference lines it
 * restates. fp32 (Eigen `fpt = float`, common_types.h:14) wherever the reference is fp32; the
 * reduced QP is double as qpOASES `real_t` (Types.hpp:171).
 */
#include "cmpc_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define BIG_NUMBER 5e10f /* SolverMPC.cpp:19 */
#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ---------------------------------------------------------------------------------------- */
/* small dense helpers (row-major)                                                           */
/* ---------------------------------------------------------------------------------------- */

/* Summation order of the fp32 products of the condensation (sgemm_nn / sgemv below). Eigen's
 * GEMM/GEMV kernels (SolverMPC.cpp:806-814) sum each dot product in an order set by its blocking
 * and vector width, which the build's Eigen version and flags fix and which this container cannot
 * reproduce (no Eigen). Three orders bracket it (oracle_set_sum_order; tests and
 * scripts/branch_orders.py only):
 *   0  sequential over k, the compiler's contraction (gcc -O3 -march=x86-64-v3: FMA) — default;
 *   1  blocked k-outer: panels of 8 products summed by fused multiply-adds from zero, each panel's
 *      sum then added to the running total (a register-blocked micro-kernel's order);
 *   2  pairwise: every product rounded on its own, then summed by recursive halving. */
static int g_sum_order = 0;
void oracle_set_sum_order(int order) { g_sum_order = (order >= 0 && order <= 2) ? order : 0; }
int oracle_sum_order(void) { return g_sum_order; }

static float dot_pairwise(const float* prod, int n) {
  if (n <= 2) return n <= 0 ? 0.f : (n == 1 ? prod[0] : prod[0] + prod[1]);
  const int h = n / 2;
  return dot_pairwise(prod, h) + dot_pairwise(prod + h, n - h);
}

/* sum_p a[p * sa] * b[p * sb] in order 1 or 2 (k <= 13 * CMPC_MAX_HORIZON) */
static float dot_order(int k, const float* a, int sa, const float* b, int sb, int order) {
  if (order == 1) {
    float acc = 0.f;
    for (int p0 = 0; p0 < k; p0 += 8) {
      float panel = 0.f;
      const int pe = p0 + 8 < k ? p0 + 8 : k;
      for (int p = p0; p < pe; p++) panel = fmaf(a[(size_t)p * sa], b[(size_t)p * sb], panel);
      acc += panel;
    }
    return acc;
  }
  float prod[13 * CMPC_MAX_HORIZON];
  for (int p = 0; p < k; p++) {
    volatile float t = a[(size_t)p * sa] * b[(size_t)p * sb];  /* rounded, never contracted */
    prod[p] = t;
  }
  return dot_pairwise(prod, k);
}

/* C[m x n] = A[m x k] * B[k x n], fp32 accumulate, C zeroed first. */
static void sgemm_nn(int m, int n, int k, const float* A, const float* B, float* C) {
  if (g_sum_order != 0) {
    for (int i = 0; i < m; i++)
      for (int j = 0; j < n; j++) C[(size_t)i * n + j] = dot_order(k, A + (size_t)i * k, 1, B + j, n, g_sum_order);
    return;
  }
  memset(C, 0, sizeof(float) * (size_t)m * n);
  for (int i = 0; i < m; i++) {
    float* c = C + (size_t)i * n;
    for (int p = 0; p < k; p++) {
      const float a = A[(size_t)i * k + p];
      const float* b = B + (size_t)p * n;
      for (int j = 0; j < n; j++) c[j] += a * b[j];
    }
  }
}

/* C[m x n] = alpha * A^T * B, A stored [k x m], B [k x n]. */
static void sgemm_tn(int m, int n, int k, float alpha, const float* A, const float* B, float* C) {
  memset(C, 0, sizeof(float) * (size_t)m * n);
  for (int p = 0; p < k; p++) {
    const float* b = B + (size_t)p * n;
    for (int i = 0; i < m; i++) {
      const float a = alpha * A[(size_t)p * m + i];
      float* c = C + (size_t)i * n;
      for (int j = 0; j < n; j++) c[j] += a * b[j];
    }
  }
}

/* y[m] = A[m x n] x[n] */
static void sgemv(int m, int n, const float* A, const float* x, float* y) {
  if (g_sum_order != 0) {
    for (int i = 0; i < m; i++) y[i] = dot_order(n, A + (size_t)i * n, 1, x, 1, g_sum_order);
    return;
  }
  for (int i = 0; i < m; i++) {
    float s = 0.f;
    for (int j = 0; j < n; j++) s += A[(size_t)i * n + j] * x[j];
    y[i] = s;
  }
}

static void dmm(int m, int n, int k, const double* A, const double* B, double* C) {
  for (int i = 0; i < m; i++)
    for (int j = 0; j < n; j++) {
      double s = 0.0;
      for (int p = 0; p < k; p++) s += A[i * k + p] * B[p * n + j];
      C[i * n + j] = s;
    }
}

/* ---------------------------------------------------------------------------------------- */
/* RobotState::set (RobotState.cpp:9-50) + quat_to_rpy (SolverMPC.cpp:352-361)               */
/* ---------------------------------------------------------------------------------------- */

/* Eigen Quaternion::toRotationMatrix (w,x,y,z), no normalisation (RobotState.cpp:36, TODO at :49). */
static void quat_to_R(const float* q, float R[9]) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  const float tx = 2.f * x, ty = 2.f * y, tz = 2.f * z;
  const float twx = tx * w, twy = ty * w, twz = tz * w;
  const float txx = tx * x, txy = ty * x, txz = tz * x;
  const float tyy = ty * y, tyz = tz * y, tzz = tz * z;
  R[0] = 1.f - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
  R[3] = txy + twz;         R[4] = 1.f - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.f - (txx + tyy);
}

static void quat_to_rpy(const float* q, float rpy[3]) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  /* t_min(-2.*(...), .99999): double arithmetic, upper clamp only, stored as fpt */
  double asd = -2. * (double)(x * z - w * y);
  if (!(asd < .99999)) asd = .99999;
  const float as = (float)asd;
  rpy[0] = (float)atan2((double)(2.f * (x * y + w * z)), (double)(w * w + x * x - y * y - z * z));
  rpy[1] = (float)asin((double)as);
  rpy[2] = (float)atan2((double)(2.f * (y * z + w * x)), (double)(w * w - x * x - y * y + z * z));
}

/* Eigen 3x3 inverse via the adjugate (SolverMPC.cpp:273). */
static void inv3(const float* m, float* o) {
  const float c00 = m[4] * m[8] - m[5] * m[7];
  const float c10 = m[5] * m[6] - m[3] * m[8];
  const float c20 = m[3] * m[7] - m[4] * m[6];
  const float det = m[0] * c00 + m[1] * c10 + m[2] * c20;
  const float id = 1.f / det;
  o[0] = c00 * id; o[1] = (m[2] * m[7] - m[1] * m[8]) * id; o[2] = (m[1] * m[5] - m[2] * m[4]) * id;
  o[3] = c10 * id; o[4] = (m[0] * m[8] - m[2] * m[6]) * id; o[5] = (m[2] * m[3] - m[0] * m[5]) * id;
  o[6] = c20 * id; o[7] = (m[1] * m[6] - m[0] * m[7]) * id; o[8] = (m[0] * m[4] - m[1] * m[3]) * id;
}

/* ---------------------------------------------------------------------------------------- */
/* ct_ss_mats (SolverMPC.cpp:260-279) + Q_ct (:607-615)                                      */
/* ---------------------------------------------------------------------------------------- */
static void ct_ss_mats(const float* I_world, float m, const float* r_feet /*3x4*/, const float* R_yaw,
                       float x_drag, float* A /*13x13*/, float* B /*13x12*/) {
  memset(A, 0, sizeof(float) * 169);
  A[3 * 13 + 9] = 1.f;
  A[11 * 13 + 9] = x_drag;
  A[4 * 13 + 10] = 1.f;
  A[5 * 13 + 11] = 1.f;
  A[11 * 13 + 12] = 1.f;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) A[i * 13 + 6 + j] = R_yaw[j * 3 + i]; /* R_yaw^T */

  memset(B, 0, sizeof(float) * 156);
  float I_inv[9];
  inv3(I_world, I_inv);
  for (int b = 0; b < 4; b++) {
    const float r0 = r_feet[0 * 4 + b], r1 = r_feet[1 * 4 + b], r2 = r_feet[2 * 4 + b];
    const float cm[9] = {0.f, -r2, r1, r2, 0.f, -r0, -r1, r0, 0.f};
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++) {
        float s = 0.f;
        for (int k = 0; k < 3; k++) s += I_inv[i * 3 + k] * cm[k * 3 + j];
        B[(6 + i) * 12 + b * 3 + j] = s;
      }
    for (int i = 0; i < 3; i++) B[(9 + i) * 12 + b * 3 + i] = 1.f / m;
  }
}

/* ---------------------------------------------------------------------------------------- */
/* c2qp discretisation (SolverMPC.cpp:96-107). expm(dt*[A B Q; 0]) of the 31x31 generator.  */
/* A^3 = 0 for this A, so M^4 = 0 and the exponential is the finite series                  */
/* I + M + M^2/2 + M^3/6 — what Eigen's Pade approximant returns up to rounding (a [p/p]      */
/* Pade of exp matches the Taylor series through order 2p >= 6). Evaluated in double,        */
/* rounded to fp32.                                                                           */
/* ---------------------------------------------------------------------------------------- */
static void discretise(const float* Af, const float* Bf, float dt, float* Adt, float* Bdt, float* Qdt) {
  double A[169], BQ[13 * 18], A2[169], ABQ[13 * 18], A2BQ[13 * 18];
  for (int i = 0; i < 169; i++) A[i] = Af[i];
  for (int i = 0; i < 13; i++) {
    for (int j = 0; j < 12; j++) BQ[i * 18 + j] = Bf[i * 12 + j];
    for (int j = 0; j < 6; j++) BQ[i * 18 + 12 + j] = (i >= 6 && i < 12 && (i - 6) == j) ? 1.0 : 0.0;
  }
  dmm(13, 13, 13, A, A, A2);
  dmm(13, 18, 13, A, BQ, ABQ);
  dmm(13, 18, 13, A, ABQ, A2BQ);
  const double h = dt, h2 = h * h / 2.0, h3 = h * h * h / 6.0;
  for (int i = 0; i < 13; i++) {
    for (int j = 0; j < 13; j++) Adt[i * 13 + j] = (float)((i == j ? 1.0 : 0.0) + h * A[i * 13 + j] + h2 * A2[i * 13 + j]);
    for (int j = 0; j < 18; j++) {
      const float v = (float)(h * BQ[i * 18 + j] + h2 * ABQ[i * 18 + j] + h3 * A2BQ[i * 18 + j]);
      if (j < 12) Bdt[i * 12 + j] = v; else Qdt[i * 6 + (j - 12)] = v;
    }
  }
}

static inline uint8_t rec_gait(const float* rec, int N, int idx) {
  const uint8_t* g = (const uint8_t*)(rec + CMPC_REC_GAIT(N));
  return g[idx];
}

/* ---------------------------------------------------------------------------------------- */
/* solve_mpc up to qH/qg (SolverMPC.cpp:566-814)                                             */
/* ---------------------------------------------------------------------------------------- */
/* ---- the blocked implementation of SolverMPC.cpp:806-814 (oracle_set_impl(1)) ----------------
 * The same dense products as the naive loops (Eigen evaluates them densely: B_qp is a dense
 * MatrixXf, S a dense 13N x 13N MatrixXf), register-tiled the way a GEMM micro-kernel is: a 6 x 16
 * tile of C in vector registers, one B row panel and six A broadcasts per k. Every C element is
 * still a sequential fused multiply-add over k from zero, the order of the naive loops compiled
 * with contraction (gcc -O3 -march=x86-64-v3), so both give the same bits
 * (tests/test_oracle.py::test_blocked_condensation_bitwise). qg's matrix-vector product runs over
 * (2 S) B_qp, the transpose of (2 B_qp^T) S (each entry is the single product 2 S_jj B_ji), so the
 * vector sweep runs along rows. CPU baseline only (bench.py cpu_baseline). */
static int g_impl = 0;
void oracle_set_impl(int impl) { g_impl = impl == 1 ? 1 : 0; }

typedef float v8f __attribute__((vector_size(32)));
#define PAD16(x) (((x) + 15) & ~15)
#define PAD6(x) ((((x) + 5) / 6) * 6)

static size_t blocked_ws_floats(int N) {
  const size_t nx = 13u * N, nu = 12u * N, nxp = PAD16(nx), nup = PAD16(nu), mx6 = PAD6(nx);
  return nu * nx + nx * nxp + nu * nxp + nx * nup + nu * nup + mx6 * nx + mx6 * nup + nup + 8 * 16;
}

#define LD8(p) (*(const v8f*)(p))   /* 32-B aligned: every buffer is 64-B aligned, ld % 16 == 0 */
#define ST8(p, v) (*(v8f*)(p) = (v))

/* The same tile loop with 16-wide vectors where the host has AVX-512 (a 6 x 32 tile in twelve
 * zmm accumulators, a 6 x 16 tile for the last 16 columns): each element is still one sequential
 * fused multiply-add chain over k from zero, so both builds give the same bits. */
typedef float v16f __attribute__((vector_size(64)));
__attribute__((target("avx512f"))) static void gemm_tiled_512(int M, int Np, int K, const float* A, int lda,
                                                              const float* B, int ldb, float* C, int ldc) {
  for (int i0 = 0; i0 < M; i0 += 6) {
    const float* a0 = A + (size_t)i0 * lda;
    int j0 = 0;
    for (; j0 + 32 <= Np; j0 += 32) {
      v16f c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0}, c20 = {0}, c21 = {0};
      v16f c30 = {0}, c31 = {0}, c40 = {0}, c41 = {0}, c50 = {0}, c51 = {0};
      for (int k = 0; k < K; k++) {
        const float* bk = B + (size_t)k * ldb + j0;
        const v16f b0 = *(const v16f*)bk, b1 = *(const v16f*)(bk + 16);
        float a;
        a = a0[k];           c00 += a * b0; c01 += a * b1;
        a = a0[lda + k];     c10 += a * b0; c11 += a * b1;
        a = a0[2 * lda + k]; c20 += a * b0; c21 += a * b1;
        a = a0[3 * lda + k]; c30 += a * b0; c31 += a * b1;
        a = a0[4 * lda + k]; c40 += a * b0; c41 += a * b1;
        a = a0[5 * lda + k]; c50 += a * b0; c51 += a * b1;
      }
      float* c = C + (size_t)i0 * ldc + j0;
      *(v16f*)c = c00; *(v16f*)(c + 16) = c01; c += ldc;
      *(v16f*)c = c10; *(v16f*)(c + 16) = c11; c += ldc;
      *(v16f*)c = c20; *(v16f*)(c + 16) = c21; c += ldc;
      *(v16f*)c = c30; *(v16f*)(c + 16) = c31; c += ldc;
      *(v16f*)c = c40; *(v16f*)(c + 16) = c41; c += ldc;
      *(v16f*)c = c50; *(v16f*)(c + 16) = c51;
    }
    for (; j0 < Np; j0 += 16) {
      v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0}, c4 = {0}, c5 = {0};
      for (int k = 0; k < K; k++) {
        const v16f b0 = *(const v16f*)(B + (size_t)k * ldb + j0);
        c0 += a0[k] * b0;
        c1 += a0[lda + k] * b0;
        c2 += a0[2 * lda + k] * b0;
        c3 += a0[3 * lda + k] * b0;
        c4 += a0[4 * lda + k] * b0;
        c5 += a0[5 * lda + k] * b0;
      }
      float* c = C + (size_t)i0 * ldc + j0;
      *(v16f*)c = c0; *(v16f*)(c + ldc) = c1; *(v16f*)(c + 2 * ldc) = c2;
      *(v16f*)(c + 3 * ldc) = c3; *(v16f*)(c + 4 * ldc) = c4; *(v16f*)(c + 5 * ldc) = c5;
    }
  }
}

/* C[M x Np] = A[M x K] (row stride lda) * B[K x Np] (ldb); M % 6 == 0, Np % 16 == 0 */
static void gemm_tiled(int M, int Np, int K, const float* A, int lda, const float* B, int ldb, float* C,
                       int ldc) {
  static int wide = -1;
  if (wide < 0) wide = __builtin_cpu_supports("avx512f") ? 1 : 0;
  if (wide) {
    gemm_tiled_512(M, Np, K, A, lda, B, ldb, C, ldc);
    return;
  }
  for (int i0 = 0; i0 < M; i0 += 6) {
    const float* a0 = A + (size_t)i0 * lda;
    for (int j0 = 0; j0 < Np; j0 += 16) {
      v8f c00 = {0}, c01 = {0}, c10 = {0}, c11 = {0}, c20 = {0}, c21 = {0};
      v8f c30 = {0}, c31 = {0}, c40 = {0}, c41 = {0}, c50 = {0}, c51 = {0};
      for (int k = 0; k < K; k++) {
        const float* bk = B + (size_t)k * ldb + j0;
        const v8f b0 = LD8(bk), b1 = LD8(bk + 8);
        float a;
        a = a0[k];           c00 += a * b0; c01 += a * b1;
        a = a0[lda + k];     c10 += a * b0; c11 += a * b1;
        a = a0[2 * lda + k]; c20 += a * b0; c21 += a * b1;
        a = a0[3 * lda + k]; c30 += a * b0; c31 += a * b1;
        a = a0[4 * lda + k]; c40 += a * b0; c41 += a * b1;
        a = a0[5 * lda + k]; c50 += a * b0; c51 += a * b1;
      }
      float* c = C + (size_t)i0 * ldc + j0;
      ST8(c, c00); ST8(c + 8, c01); c += ldc;
      ST8(c, c10); ST8(c + 8, c11); c += ldc;
      ST8(c, c20); ST8(c + 8, c21); c += ldc;
      ST8(c, c30); ST8(c + 8, c31); c += ldc;
      ST8(c, c40); ST8(c + 8, c41); c += ldc;
      ST8(c, c50); ST8(c + 8, c51);
    }
  }
}

static float* align64(float* p) { return (float*)(((uintptr_t)p + 63) & ~(uintptr_t)63); }

/* qH and qg as the naive code below computes them, through gemm_tiled */
static void condense_blocked(int N, const float* Bqp, const float* w12, float alpha, const float* vec,
                             float* qH, float* qg, float* ws) {
  const int nx = 13 * N, nu = 12 * N, nxp = PAD16(nx), nup = PAD16(nu), mx6 = PAD6(nx);
  float* Bt = align64(ws);
  float* Sp = align64(Bt + (size_t)nu * nx);
  float* T = align64(Sp + (size_t)nx * nxp);
  float* Bp = align64(T + (size_t)nu * nxp);
  float* Hp = align64(Bp + (size_t)nx * nup);
  float* S2 = align64(Hp + (size_t)nu * nup);
  float* T2t = align64(S2 + (size_t)mx6 * nx);
  float* y = align64(T2t + (size_t)mx6 * nup);
  /* the dense S (SolverMPC.cpp:624-630) and 2 S, B_qp^T and B_qp with padded rows */
  memset(Sp, 0, sizeof(float) * (size_t)nx * nxp);
  memset(S2, 0, sizeof(float) * (size_t)mx6 * nx);
  for (int k = 0; k < N; k++)
    for (int i = 0; i < 12; i++) {
      const int d = 13 * k + i;
      Sp[(size_t)d * nxp + d] = w12[i];
      S2[(size_t)d * nx + d] = 2.f * w12[i];
    }
  for (int p = 0; p < nx; p++) {
    for (int i = 0; i < nu; i++) Bt[(size_t)i * nx + p] = Bqp[(size_t)p * nu + i];
    memcpy(Bp + (size_t)p * nup, Bqp + (size_t)p * nu, sizeof(float) * nu);
    for (int i = nu; i < nup; i++) Bp[(size_t)p * nup + i] = 0.f;
  }
  gemm_tiled(nu, nxp, nx, Bt, nx, Sp, nxp, T, nxp);    /* B^T S */
  gemm_tiled(nu, nup, nx, T, nxp, Bp, nup, Hp, nup);   /* (B^T S) B */
  gemm_tiled(mx6, nup, nx, S2, nx, Bp, nup, T2t, nup); /* ((2 B^T) S)^T = (2 S) B */
  for (int i = 0; i < nu; i++)
    for (int j = 0; j < nu; j++) {
      float h = Hp[(size_t)i * nup + j];
      if (i == j) h += alpha;
      qH[(size_t)i * nu + j] = 2.f * h;
    }
  for (int i0 = 0; i0 < nup; i0 += 8) {
    v8f acc = {0};
    for (int j = 0; j < nx; j++) acc += LD8(T2t + (size_t)j * nup + i0) * vec[j];
    ST8(y + i0, acc);
  }
  memcpy(qg, y, sizeof(float) * nu);
}

size_t oracle_condense_ws_bytes(int N) {
  const size_t nx = 13u * N, nu = 12u * N;
  return sizeof(float) * (169u * (N + 1) + nx * 13 + nx * nu + nx * 6 + nx * nx + nu * nx + 2 * nx +
                          blocked_ws_floats(N));
}
static size_t naive_ws_bytes(int N) {
  const size_t nx = 13u * N, nu = 12u * N;
  return sizeof(float) * (169u * (N + 1) + nx * 13 + nx * nu + nx * 6 + nx * nx + nu * nx + 2 * nx);
}

int oracle_condense(const float* rec, const cmpc_params* prm, oracle_cond* out) {
  const int N = prm->horizon;
  if (N < 1 || N > CMPC_MAX_HORIZON) return CMPC_BAD_INPUT;
  void* ws = malloc(oracle_condense_ws_bytes(N));
  const int st = oracle_condense_ws(rec, prm, out, ws);
  free(ws);
  return st;
}

int oracle_condense_ws(const float* rec, const cmpc_params* prm, oracle_cond* out, void* ws) {
  const int N = prm->horizon;
  if (N < 1 || N > CMPC_MAX_HORIZON) return CMPC_BAD_INPUT;
  const int nx = 13 * N, nu = 12 * N;

  /* RobotState::set */
  const float* p = rec + CMPC_REC_P;
  const float* v = rec + CMPC_REC_V;
  const float* q = rec + CMPC_REC_Q;
  const float* w = rec + CMPC_REC_W;
  const float* r = rec + CMPC_REC_R; /* r_feet(rs, c) = r[rs*4 + c] (RobotState.cpp:28-34) */
  float R[9];
  quat_to_R(q, R);                   /* R_yaw = R (RobotState.cpp:44) */
  const float Ibody[3] = {.07f, 0.26f, 0.242f};
  const float m = 12.0f;             /* RobotState.h:26 */

  float rpy[3];
  quat_to_rpy(q, rpy);
  float x0[13] = {rpy[2], rpy[1], rpy[0], p[0], p[1], p[2], w[0], w[1], w[2], v[0], v[1], v[2], -9.8f};

  /* I_world = R_yaw * I_body * R_yaw^T (SolverMPC.cpp:593) */
  float RI[9], Iw[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) RI[i * 3 + j] = R[i * 3 + j] * Ibody[j];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      float s = 0.f;
      for (int k = 0; k < 3; k++) s += RI[i * 3 + k] * R[j * 3 + k];
      Iw[i * 3 + j] = s;
    }

  float Act[169], Bct[156];
  ct_ss_mats(Iw, m, r, R, rec[CMPC_REC_XDRAG], Act, Bct);

  float Adt[169], Bdt[156], Qdt[78];
  discretise(Act, Bct, prm->dt, Adt, Bdt, Qdt);

  /* powerMats, A_qp, B_qp, Q_qp (SolverMPC.cpp:118-139); the N <= 19 cap is lifted. */
  /* resize_qp_mats zeroes every matrix on every call (SolverMPC.cpp:188-196) */
  float* pw = (float*)ws;
  float* Aqp = pw + 169 * (N + 1);
  float* Bqp = Aqp + nx * 13;
  float* Qqp = Bqp + (size_t)nx * nu;
  float* S = Qqp + nx * 6;
  float* T = S + (size_t)nx * nx;
  float* vec = T + (size_t)nu * nx;
  float* tmp = vec + nx;
  memset(ws, 0, naive_ws_bytes(N));
  float blk[13 * 12], qb[13 * 6];
  memset(pw, 0, sizeof(float) * 169);
  for (int i = 0; i < 13; i++) pw[i * 14] = 1.f;
  for (int k = 1; k <= N; k++) sgemm_nn(13, 13, 13, Adt, pw + 169 * (k - 1), pw + 169 * k);
  for (int rr = 0; rr < N; rr++) {
    for (int i = 0; i < 13; i++)
      for (int j = 0; j < 13; j++) Aqp[(13 * rr + i) * 13 + j] = pw[169 * (rr + 1) + i * 13 + j];
    for (int c = 0; c <= rr; c++) {
      sgemm_nn(13, 12, 13, pw + 169 * (rr - c), Bdt, blk);
      sgemm_nn(13, 6, 13, pw + 169 * (rr - c), Qdt, qb);
      for (int i = 0; i < 13; i++) {
        for (int j = 0; j < 12; j++) Bqp[(size_t)(13 * rr + i) * nu + 12 * c + j] = blk[i * 12 + j];
        for (int j = 0; j < 6; j++) Qqp[(13 * rr + i) * 6 + j] += qb[i * 6 + j];
      }
    }
  }

  /* S = diag([weights, 0] x N), dense (SolverMPC.cpp:624-630); X_d (:633-639) */
  for (int k = 0; k < N; k++)
    for (int i = 0; i < 12; i++) S[(size_t)(13 * k + i) * nx + 13 * k + i] = prm->weights[i];
  const float* traj = rec + CMPC_REC_TRAJ(N);

  const int blocked = g_impl == 1 && out && out->qH && out->qg;
  /* qH = 2 (B^T S B + alpha I) (SolverMPC.cpp:806): (B^T S) B, as Eigen evaluates it. */
  if (out && out->qH && !blocked) {
    sgemm_tn(nu, nx, nx, 1.f, Bqp, S, T);
    sgemm_nn(nu, nu, nx, T, Bqp, out->qH);
    for (int i = 0; i < nu; i++)
      for (int j = 0; j < nu; j++) {
        float h = out->qH[(size_t)i * nu + j];
        if (i == j) h += prm->alpha;
        out->qH[(size_t)i * nu + j] = 2.f * h;
      }
  }
  /* qg = 2 B^T S (A_qp x0 + Q_qp f - X_d) (SolverMPC.cpp:808-814); f = f_est only when the
   * disturbance history exceeds 500 samples (flag bit 0), else f = 0. */
  if (out && out->qg) {
    float f[6] = {0, 0, 0, 0, 0, 0};
    uint32_t flags;
    memcpy(&flags, rec + CMPC_REC_FLAGS, 4);
    if (flags & 1u) f[3] = rec[CMPC_REC_FEST3];
    sgemv(nx, 13, Aqp, x0, vec);
    sgemv(nx, 6, Qqp, f, tmp);
    for (int k = 0; k < N; k++)
      for (int i = 0; i < 13; i++) {
        const float xd = (i < 12) ? traj[12 * k + i] : 0.f;
        vec[13 * k + i] = (vec[13 * k + i] + tmp[13 * k + i]) - xd;
      }
    if (blocked) {
      condense_blocked(N, Bqp, prm->weights, prm->alpha, vec, out->qH, out->qg,
                       (float*)((char*)ws + naive_ws_bytes(N)));
    } else {
      sgemm_tn(nu, nx, nx, 2.f, Bqp, S, T); /* (2 B^T) S, a second product as in the reference */
      sgemv(nu, nx, T, vec, out->qg);
    }
  }
  if (out) {
    memcpy(out->x0, x0, sizeof(x0));
    memcpy(out->Adt, Adt, sizeof(Adt));
    memcpy(out->Bdt, Bdt, sizeof(Bdt));
    memcpy(out->Qdt, Qdt, sizeof(Qdt));
  }
  return CMPC_OK;
}

/* near_zero / near_one take fpt (SolverMPC.cpp:72-80) */
static int near_zero(float a) { return (a < 0.01f && a > -.01f); }
static int near_one(float a) { return near_zero(a - 1); }

/* ---------------------------------------------------------------------------------------- */
/* QP data + swing elimination (SolverMPC.cpp:841-950)                                       */
/* ---------------------------------------------------------------------------------------- */
size_t oracle_reduce_ws_bytes(int N) {
  const size_t nv = 12u * N, nc = 20u * N;
  return sizeof(double) * (nc * nv + 2 * nc) + sizeof(int) * (nv + nc);
}

int oracle_reduce(const float* rec, const cmpc_params* prm, const float* qH, const float* qg,
                  oracle_red* red) {
  void* ws = malloc(oracle_reduce_ws_bytes(prm->horizon));
  const int st = oracle_reduce_ws(rec, prm, qH, qg, red, ws);
  free(ws);
  return st;
}

int oracle_reduce_ws(const float* rec, const cmpc_params* prm, const float* qH, const float* qg,
                     oracle_red* red, void* ws) {
  const int N = prm->horizon;
  const int nv = 12 * N, nc = 20 * N;
  /* fmat (:657-665) and U_b (:643-655), lb = 0 (:846-849), all as double */
  double* A = (double*)ws;
  double* ub = A + (size_t)nc * nv;
  double* lb = ub + nc;
  memset(A, 0, sizeof(double) * (size_t)nc * nv);
  const float mu = 1.f / prm->mu;
  const float fb[15] = {mu, 0, 1.f, -mu, 0, 1.f, 0, mu, 1.f, 0, -mu, 1.f, 0, 0, 1.f};
  for (int i = 0; i < 4 * N; i++)
    for (int a = 0; a < 5; a++)
      for (int b = 0; b < 3; b++) A[(size_t)(5 * i + a) * nv + 3 * i + b] = fb[a * 3 + b];
  for (int k = 0; k < 4 * N; k++) {
    ub[5 * k + 0] = BIG_NUMBER;
    ub[5 * k + 1] = BIG_NUMBER;
    ub[5 * k + 2] = BIG_NUMBER;
    ub[5 * k + 3] = BIG_NUMBER;
    ub[5 * k + 4] = (float)rec_gait(rec, N, k) * prm->f_max; /* u8 * fpt */
  }
  for (int i = 0; i < nc; i++) lb[i] = 0.0f;

  char* var_elim = red->var_elim;
  char* con_elim = red->con_elim;
  memset(var_elim, 0, nv);
  memset(con_elim, 0, nc);
  int new_vars = nv, new_cons = nc;
  for (int i = 0; i < nc; i++) {
    if (!(near_zero((float)lb[i]) && near_zero((float)ub[i]))) continue;
    const double* c_row = &A[(size_t)i * nv];
    for (int j = 0; j < nv; j++) {
      if (near_one((float)c_row[j])) {
        new_vars -= 3;
        new_cons -= 5;
        const int cs = (j * 5) / 3 - 3;
        var_elim[j - 2] = 1; var_elim[j - 1] = 1; var_elim[j] = 1;
        for (int t = 0; t < 5; t++) con_elim[cs + t] = 1;
      }
    }
  }
  int* var_ind = (int*)(lb + nc);
  int* con_ind = var_ind + nv;
  int vc = 0;
  for (int i = 0; i < nv; i++) if (!var_elim[i]) var_ind[vc++] = i;
  vc = 0;
  for (int i = 0; i < nc; i++) if (!con_elim[i]) con_ind[vc++] = i;
  for (int i = 0; i < new_vars; i++) {
    const int olda = var_ind[i];
    red->g[i] = (double)qg[olda];
    for (int j = 0; j < new_vars; j++) red->H[i * new_vars + j] = (double)qH[(size_t)olda * nv + var_ind[j]];
  }
  for (int c = 0; c < new_cons; c++)
    for (int s = 0; s < new_vars; s++) {
      const float cval = (float)A[(size_t)nv * con_ind[c] + var_ind[s]]; /* :941 */
      red->A[c * new_vars + s] = cval;
    }
  for (int i = 0; i < new_cons; i++) {
    red->ub[i] = ub[con_ind[i]];
    red->lb[i] = lb[con_ind[i]];
  }
  red->nv = new_vars;
  red->nc = new_cons;
  red->nv_full = nv;
  red->nc_full = nc;
  return CMPC_OK;
}

void oracle_scatter(const oracle_red* red, const double* q_red, double* q_soln) {
  int vc = 0;
  for (int i = 0; i < red->nv_full; i++) q_soln[i] = red->var_elim[i] ? 0.0 : q_red[vc++];
}

/* ---------------------------------------------------------------------------------------- */
/* Config 5: periodic-disturbance estimation                                                 */
/* ---------------------------------------------------------------------------------------- */

/* gaussian_filter (SolverMPC.cpp:404-437): float kernel of radius ceil(3 sigma), each tap
 * exp(-0.5 i^2 / sigma^2) evaluated in double and stored as float, normalised by a float sum;
 * double accumulation with edge clamping. */
void oracle_gaussian_filter(const double* data, int n, float sigma, double* out) {
  const int radius = (int)ceil(3 * sigma);
  float kernel[2 * 81 + 1];
  float sum = 0.0f;
  for (int i = -radius; i <= radius; i++) {
    const float value = (float)exp(-0.5 * (i * i) / (double)(sigma * sigma));
    kernel[i + radius] = value;
    sum += value;
  }
  for (int i = 0; i < 2 * radius + 1; i++) kernel[i] /= sum;
  for (int i = 0; i < n; i++) {
    double acc = 0.0;
    for (int j = -radius; j <= radius; j++) {
      int idx = i + j;
      if (idx < 0) idx = 0;
      else if (idx >= n) idx = n - 1;
      acc += data[idx] * kernel[j + radius];
    }
    out[i] = acc;
  }
}

/* fit_sin (SolverMPC.cpp:478-541): |r2c| of bins 0..n/2 (here a direct DFT in double), argmax
 * over bins >= 1 (first maximum), freq = |fftfreq(n, tt[1]-tt[0])[k]|, amp = sqrt(2) std,
 * offset = mean, phase = 0; returned freq = (2 pi f) / (2 pi) as the reference computes it. */
void oracle_fit_sin(const double* tt, const double* yy, int n, double* amp, double* freq,
                    double* phase, double* offset, int* peak_bin) {
  const double dt = tt[1] - tt[0];
  int max_index = 1;
  double max_val = -1.0;
  for (int k = 1; k <= n / 2; k++) {
    double re = 0.0, im = 0.0;
    for (int t = 0; t < n; t++) {
      const double ang = 2.0 * M_PI * (double)((long)k * t % n) / (double)n;
      re += yy[t] * cos(ang);
      im -= yy[t] * sin(ang);
    }
    const double mag = sqrt(re * re + im * im);
    if (k == 1 || mag > max_val) { max_val = mag; max_index = k; }
  }
  const double guess_freq = fabs((max_index <= n / 2) ? max_index / (n * dt) : (max_index - n) / (n * dt));
  double m = 0.0;
  for (int i = 0; i < n; i++) m += yy[i];
  m /= n;
  double acc = 0.0;
  for (int i = 0; i < n; i++) acc += (yy[i] - m) * (yy[i] - m);
  const double s = sqrt(acc / n);
  const double w = 2 * M_PI * guess_freq;
  *amp = s * sqrt(2.0);
  *offset = m;
  *phase = 0.0;
  *freq = w / (2 * M_PI);
  if (peak_bin) *peak_bin = max_index;
}

/* Residual f_ext of ConvexMPCLocomotion.cpp:639-771: e = x_k - A_prev x_prev - B_prev u_prev with
 * the CONTINUOUS model of the logged step (no dt), x(12) = -9.81, u_prev = -logged forces;
 * f_ext = (-e6, -e7, e8, e9, e10, e11). x_k = (roll, pitch, yaw, p, w, v, -9.81) of the record. */
void oracle_residual(const float* log, const float* rec, float f_ext[6]) {
  float A[169], B[156];
  const float* R = log + CMPC_LOG_ROT; /* R_yaw, row-major */
  const float Ibody[3] = {0.07f, 0.26f, 0.242f};
  float RI[9], Iw[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) RI[i * 3 + j] = R[i * 3 + j] * Ibody[j];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      float s = 0.f;
      for (int k = 0; k < 3; k++) s += RI[i * 3 + k] * R[j * 3 + k];
      Iw[i * 3 + j] = s;
    }
  /* A_prev / B_prev have exactly the ct_ss_mats structure (:641-687 vs SolverMPC.cpp:260-279) */
  ct_ss_mats(Iw, 12.f, log + CMPC_LOG_R, R, log[CMPC_LOG_XDRAG], A, B);
  float x_k[13], x_prev[13], u_prev[12];
  x_k[0] = rec[CMPC_REC_RPY + 0];
  x_k[1] = rec[CMPC_REC_RPY + 1];
  x_k[2] = rec[CMPC_REC_RPY + 2];
  for (int i = 0; i < 3; i++) {
    x_k[3 + i] = rec[CMPC_REC_P + i];
    x_k[6 + i] = rec[CMPC_REC_W + i];
    x_k[9 + i] = rec[CMPC_REC_V + i];
    x_prev[0 + i] = log[CMPC_LOG_EUL + i];
    x_prev[3 + i] = log[CMPC_LOG_POS + i];
    x_prev[6 + i] = log[CMPC_LOG_ANG + i];
    x_prev[9 + i] = log[CMPC_LOG_LIN + i];
  }
  x_k[12] = -9.81f;
  x_prev[12] = -9.81f;
  for (int i = 0; i < 12; i++) u_prev[i] = -log[CMPC_LOG_FORCE + i];
  float e[13];
  for (int i = 0; i < 13; i++) {
    float ax = 0.f, bu = 0.f;
    for (int k = 0; k < 13; k++) ax += A[i * 13 + k] * x_prev[k];
    for (int k = 0; k < 12; k++) bu += B[i * 12 + k] * u_prev[k];
    e[i] = (x_k[i] - ax) - bu;
  }
  f_ext[0] = -e[6];
  f_ext[1] = -e[7];
  f_ext[2] = e[8];
  f_ext[3] = e[9];
  f_ext[4] = e[10];
  f_ext[5] = e[11];
}

/* Estimator step (SolverMPC.cpp:688-798) on a CMPC_EST_WORDS state. */
float oracle_est_step(float* st, float f3, float t, int* use_f_est) {
  int32_t count, head;
  memcpy(&count, st + CMPC_EST_COUNT, 4);
  memcpy(&head, st + CMPC_EST_HEAD, 4);
  double prm[4];
  memcpy(prm, st + CMPC_EST_PARAMS, sizeof(prm));
  st[CMPC_EST_F + head] = f3; /* diff_history.push_back(f_ext(3)) */
  st[CMPC_EST_T + head] = t;  /* time_history.push_back(simulation_time) */
  head = (head + 1) % CMPC_EST_WINDOW;
  if (count < (1 << 30)) count++;
  float f_est3 = st[CMPC_EST_FEST3];
  if (count >= CMPC_EST_WINDOW) {
    if (count <= CMPC_EST_STOP) {
      double tw[CMPC_EST_WINDOW], dw[CMPC_EST_WINDOW], b7[CMPC_EST_WINDOW], b27[CMPC_EST_WINDOW];
      for (int i = 0; i < CMPC_EST_WINDOW; i++) {
        const int idx = (head + i) % CMPC_EST_WINDOW; /* oldest first */
        tw[i] = st[CMPC_EST_T + idx];
        dw[i] = st[CMPC_EST_F + idx];
      }
      oracle_gaussian_filter(dw, CMPC_EST_WINDOW, 7.0f, b7);
      oracle_gaussian_filter(dw, CMPC_EST_WINDOW, 27.0f, b27);
      for (int i = 0; i < CMPC_EST_WINDOW; i++) b7[i] = b7[i] - b27[i];
      double amp, freq, phase, offset;
      oracle_fit_sin(tw, b7, CMPC_EST_WINDOW, &amp, &freq, &phase, &offset, NULL);
      prm[0] = offset; /* est_stat */
      prm[1] = amp;
      prm[2] = freq;
      prm[3] = phase;
    }
    /* compensatory_force = est_amp + sin(2 pi t f + phase)  ('+' as in :766), float */
    f_est3 = (float)(prm[1] + sin(2 * M_PI * t * prm[2] + prm[3]));
  }
  st[CMPC_EST_FEST3] = f_est3;
  memcpy(st + CMPC_EST_COUNT, &count, 4);
  memcpy(st + CMPC_EST_HEAD, &head, 4);
  memcpy(st + CMPC_EST_PARAMS, prm, sizeof(prm));
  if (use_f_est) *use_f_est = count > CMPC_EST_STOP;
  return f_est3;
}
