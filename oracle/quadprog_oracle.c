/* TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * CPU restatement of QuadProg++'s solve_quadprog (Goldfarb-Idnani dual active set, fp64), the QP
 * of WBIC::MakeTorque (be2r_cmpc_unitree/src/controllers/WBC/WBIC/WBIC.cpp:91):
 *
 *     min 0.5 x'Gx + g0'x   s.t.   CE'x + ce0 = 0,   CI'x + ci0 >= 0
 *
 * following be2r_cmpc_unitree/src/third_party/Goldfarb_Optimizer/QuadProg++.cc:108-507 step by
 * step (preprocessing :174-223, equality phase :225-266, step 1 :272-318, step 2 :320-347,
 * step 2a/2b/2c :349-506, add_constraint :552-621, delete_constraint :623-698, distance
 * :700-717, cholesky_decomposition :731-762, forward/backward elimination :775-801).
 *
 * The reference cannot be compiled here: QuadProg++.hh includes <eigen3/Eigen/Dense> and the
 * image has no Eigen. Parity is pinned instead by KKT certificates (tests/test_quadprog.py:
 * stationarity, primal feasibility, dual feasibility, complementarity; for a strictly convex QP
 * the KKT point is THE optimum, whatever the solver).
 *
 * Evaluation orders: where the reference's order is inherently serial and a wavefront would
 * compute it in parallel, this restatement fixes the parallel order instead, and the HIP kernel
 * (csrc/cmpc_quadprog.hip) uses exactly the same one, so kernel and oracle agree bit for bit:
 *   - scalar products and sums over a vector: a 64-wide xor-butterfly tree (qp_tsum);
 *   - update_r (:537-550): r_i = (d_i - acc_i) / R_ii with acc_i accumulated over j = iq-1 down
 *     to i+1 (the reference sums j upwards);
 *   - the argmins of step 2 and 2b (:321-328, :369-379): first minimum in index order, as the
 *     reference's strict '<' scans pick.
 * Every other loop keeps the reference's order. Compile with -ffp-contract=off.
 * An iteration cap (the reference loops until done) returns status 1.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "cmpc_oracle.h"

#define QP_EPS 2.220446049250313e-16 /* std::numeric_limits<double>::epsilon() */

/* 64-lane xor-butterfly sum of v[0..cnt) (zero padded), the kernel's wave reduction */
static double qp_tsum(const double* v, int cnt) {
  double a[64];
  for (int l = 0; l < 64; l++) a[l] = (l < cnt) ? v[l] : 0.0;
  for (int k = 32; k >= 1; k >>= 1) {
    double b[64];
    for (int l = 0; l < 64; l++) b[l] = a[l] + a[l ^ k];
    memcpy(a, b, sizeof a);
  }
  return a[0];
}

static double qp_dot(const double* x, const double* y, int n) {
  double t[64];
  for (int i = 0; i < n; i++) t[i] = x[i] * y[i];
  return qp_tsum(t, n);
}

/* QuadProg++.cc:700-717 */
static double qp_dist(double a, double b) {
  const double a1 = fabs(a), b1 = fabs(b);
  if (a1 > b1) { const double t = b1 / a1; return a1 * sqrt(1.0 + t * t); }
  if (b1 > a1) { const double t = a1 / b1; return b1 * sqrt(1.0 + t * t); }
  return a1 * sqrt(2.0);
}

typedef struct {
  int n, p, m;
  double* J;   /* n x n, row stride n */
  double* R;   /* n x n */
  double* d;
} qp_ws;

#define JJ(w, i, j) (w)->J[(i) * (w)->n + (j)]
#define RR(w, i, j) (w)->R[(i) * (w)->n + (j)]

/* compute_d (:509-522): d = J' np */
static void qp_compute_d(qp_ws* w, const double* np) {
  for (int i = 0; i < w->n; i++) {
    double sum = 0.0;
    for (int j = 0; j < w->n; j++) sum += JJ(w, j, i) * np[j];
    w->d[i] = sum;
  }
}

/* update_z (:524-535): z = J[:, iq:] d[iq:] */
static void qp_update_z(qp_ws* w, double* z, int iq) {
  for (int i = 0; i < w->n; i++) {
    double sum = 0.0;
    for (int j = iq; j < w->n; j++) sum += JJ(w, i, j) * w->d[j];
    z[i] = sum;
  }
}

/* update_r (:537-550): r = R^-1 d over the iq active positions (column-oriented order) */
static void qp_update_r(qp_ws* w, double* r, int iq) {
  double acc[64];
  for (int i = 0; i < iq; i++) acc[i] = 0.0;
  for (int i = iq - 1; i >= 0; i--) {
    r[i] = (w->d[i] - acc[i]) / RR(w, i, i);
    for (int k = 0; k < i; k++) acc[k] += RR(w, k, i) * r[i];
  }
}

/* add_constraint (:552-621); returns 0 when the new column is degenerate */
static int qp_add(qp_ws* w, int* iq, double* rnorm) {
  const int n = w->n;
  for (int j = n - 1; j >= *iq + 1; j--) {
    double cc = w->d[j - 1], ss = w->d[j];
    const double h = qp_dist(cc, ss);
    if (fabs(h) < QP_EPS) continue;
    w->d[j] = 0.0;
    ss = ss / h;
    cc = cc / h;
    if (cc < 0.0) { cc = -cc; ss = -ss; w->d[j - 1] = -h; }
    else w->d[j - 1] = h;
    const double xny = ss / (1.0 + cc);
    for (int k = 0; k < n; k++) {
      const double t1 = JJ(w, k, j - 1), t2 = JJ(w, k, j);
      JJ(w, k, j - 1) = t1 * cc + t2 * ss;
      JJ(w, k, j) = xny * (t1 + JJ(w, k, j - 1)) - t2;
    }
  }
  (*iq)++;
  for (int i = 0; i < *iq; i++) RR(w, i, *iq - 1) = w->d[i];
  if (fabs(w->d[*iq - 1]) <= QP_EPS * *rnorm) return 0;
  *rnorm = fmax(*rnorm, fabs(w->d[*iq - 1]));
  return 1;
}

/* delete_constraint (:623-698) */
static void qp_delete(qp_ws* w, int* A, double* u, int p, int* iq, int l) {
  const int n = w->n;
  int qq = -1;
  for (int i = p; i < *iq; i++)
    if (A[i] == l) { qq = i; break; }
  if (qq < 0) return;  /* cannot happen on the reference's paths */
  for (int i = qq; i < *iq - 1; i++) {
    A[i] = A[i + 1];
    u[i] = u[i + 1];
    for (int j = 0; j < n; j++) RR(w, j, i) = RR(w, j, i + 1);
  }
  A[*iq - 1] = A[*iq];
  u[*iq - 1] = u[*iq];
  A[*iq] = 0;
  u[*iq] = 0.0;
  for (int j = 0; j < *iq; j++) RR(w, j, *iq - 1) = 0.0;
  (*iq)--;
  if (*iq == 0) return;
  for (int j = qq; j < *iq; j++) {
    double cc = RR(w, j, j), ss = RR(w, j + 1, j);
    const double h = qp_dist(cc, ss);
    if (fabs(h) < QP_EPS) continue;
    cc = cc / h;
    ss = ss / h;
    RR(w, j + 1, j) = 0.0;
    if (cc < 0.0) { RR(w, j, j) = -h; cc = -cc; ss = -ss; }
    else RR(w, j, j) = h;
    const double xny = ss / (1.0 + cc);
    for (int k = j + 1; k < *iq; k++) {
      const double t1 = RR(w, j, k), t2 = RR(w, j + 1, k);
      RR(w, j, k) = t1 * cc + t2 * ss;
      RR(w, j + 1, k) = xny * (t1 + RR(w, j, k)) - t2;
    }
    for (int k = 0; k < n; k++) {
      const double t1 = JJ(w, k, j), t2 = JJ(w, k, j + 1);
      JJ(w, k, j) = t1 * cc + t2 * ss;
      JJ(w, k, j + 1) = xny * (JJ(w, k, j) + t1) - t2;
    }
  }
}

/* One problem. Dense row-major inputs with leading dimensions (QuadProg++ layout: CE is n x p,
 * CI is n x m, a constraint per column). Returns the status; *fval = objective (inf when
 * infeasible), x[0..n). */
int oracle_quadprog(int n, int p, int m, const double* Gin, int ldg, const double* g0,
                    const double* CE, int ldce, const double* ce0, const double* CI, int ldci,
                    const double* ci0, int max_iter, double* x, double* fval, int* iters_out) {
  *fval = 0.0;
  *iters_out = 0;
  if (n < 1 || n > 64 || p < 0 || p > n || m < 0 || m > 64) return CMPC_BAD_INPUT;
  const double inf = INFINITY;
  double L[64 * 64], J[64 * 64], R[64 * 64], d[64], z[64], np[64], r[128], u[128], s[128];
  double x_old[64], u_old[128];
  int A[128], A_old[128], iai[128], iaexcl[128];
  qp_ws w = {n, p, m, J, R, d};
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) L[i * n + j] = Gin[i * ldg + j];
  for (int i = 0; i < 128; i++) { u[i] = 0.0; r[i] = 0.0; A[i] = 0; }
  *iters_out = 0;
  /* :174-181 trace of G, Cholesky G = L L' (row-oriented, :731-762) */
  double tr[64];
  for (int i = 0; i < n; i++) tr[i] = L[i * n + i];
  const double c1 = qp_tsum(tr, n);
  for (int i = 0; i < n; i++) {
    double dii = 0.0;
    for (int j = i; j < n; j++) {
      double sum = L[i * n + j];
      for (int k = i - 1; k >= 0; k--) sum -= L[i * n + k] * L[j * n + k];
      if (j == i) {
        if (sum <= 0.0) { *fval = inf; return CMPC_NOT_PD; }
        dii = sqrt(sum);
        L[i * n + i] = dii;
      } else {
        L[j * n + i] = sum / dii;
      }
    }
    for (int k = i + 1; k < n; k++) L[i * n + k] = L[k * n + i];
  }
  /* :186-204 R = 0, J = L^-T by forward elimination of the unit vectors, c2 = trace J */
  for (int i = 0; i < n * n; i++) R[i] = 0.0;
  double jd[64];
  for (int i = 0; i < n; i++) {
    double y[64];
    for (int rr = 0; rr < n; rr++) {
      double v = (rr == i) ? 1.0 : 0.0;
      for (int j = 0; j < rr; j++) v -= L[rr * n + j] * y[j];
      y[rr] = v / L[rr * n + rr];
    }
    for (int j = 0; j < n; j++) J[i * n + j] = y[j];
    jd[i] = y[i];
  }
  const double c2 = qp_tsum(jd, n);
  double rnorm = 1.0;
  /* :216-219 x = -G^-1 g0 (forward then backward elimination), f = 0.5 g0'x */
  {
    double y[64];
    for (int i = 0; i < n; i++) {
      double v = g0[i];
      for (int j = 0; j < i; j++) v -= L[i * n + j] * y[j];
      y[i] = v / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
      double v = y[i];
      for (int j = i + 1; j < n; j++) v -= L[i * n + j] * x[j];
      x[i] = v / L[i * n + i];
    }
    for (int i = 0; i < n; i++) x[i] = -x[i];
  }
  double f = 0.5 * qp_dot(g0, x, n);
  /* :225-266 equality constraints */
  int iq = 0;
  for (int i = 0; i < p; i++) {
    for (int j = 0; j < n; j++) np[j] = CE[j * ldce + i];
    qp_compute_d(&w, np);
    qp_update_z(&w, z, iq);
    qp_update_r(&w, r, iq);
    double t2 = 0.0;
    const double zz = qp_dot(z, z, n), znp = qp_dot(z, np, n);
    if (fabs(zz) > QP_EPS) t2 = (-qp_dot(np, x, n) - ce0[i]) / znp;
    for (int k = 0; k < n; k++) x[k] += t2 * z[k];
    u[iq] = t2;
    for (int k = 0; k < iq; k++) u[k] -= t2 * r[k];
    f += 0.5 * (t2 * t2) * znp;
    A[i] = -i - 1;
    if (!qp_add(&w, &iq, &rnorm)) { *fval = f; return CMPC_BAD_INPUT; }
  }
  for (int i = 0; i < m; i++) iai[i] = i;
  int ip = 0, iter = 0;
  double ss = 0.0;
  for (;;) {  /* l1 (:272) */
    if (++iter > max_iter) { *fval = f; *iters_out = iter - 1; return CMPC_MAX_ITER; }
    for (int i = p; i < iq; i++) iai[A[i]] = -1;
    ss = 0.0;
    ip = 0;
    double mins[128];
    for (int i = 0; i < m; i++) {
      iaexcl[i] = 1;
      double sum = 0.0;
      for (int j = 0; j < n; j++) sum += CI[j * ldci + i] * x[j];
      sum += ci0[i];
      s[i] = sum;
      mins[i] = fmin(0.0, sum);
    }
    const double psi = qp_tsum(mins, m);
    if (fabs(psi) <= m * QP_EPS * c1 * c2 * 100.0) { *fval = f; *iters_out = iter; return CMPC_OK; }
    for (int i = 0; i < iq; i++) { u_old[i] = u[i]; A_old[i] = A[i]; }
    for (int i = 0; i < n; i++) x_old[i] = x[i];
    int go_l1 = 0;
    while (!go_l1) {  /* l2 (:320) */
      for (int i = 0; i < m; i++)
        if (s[i] < ss && iai[i] != -1 && iaexcl[i]) { ss = s[i]; ip = i; }
      if (ss >= 0.0) { *fval = f; *iters_out = iter; return CMPC_OK; }
      for (int i = 0; i < n; i++) np[i] = CI[i * ldci + ip];
      u[iq] = 0.0;
      A[iq] = ip;
      for (;;) {  /* l2a (:349) */
        if (++iter > max_iter) { *fval = f; *iters_out = iter - 1; return CMPC_MAX_ITER; }
        qp_compute_d(&w, np);
        qp_update_z(&w, z, iq);
        qp_update_r(&w, r, iq);
        int l = 0;
        double t1 = inf;
        for (int k = p; k < iq; k++)
          if (r[k] > 0.0 && u[k] / r[k] < t1) { t1 = u[k] / r[k]; l = A[k]; }
        const double zz = qp_dot(z, z, n), znp = qp_dot(z, np, n);
        double t2;
        if (fabs(zz) > QP_EPS) {
          t2 = -s[ip] / znp;
          if (t2 < 0) t2 = inf;
        } else {
          t2 = inf;
        }
        const double t = fmin(t1, t2);
        if (t >= inf) { *fval = inf; *iters_out = iter; return CMPC_INFEASIBLE; }
        if (t2 >= inf) {  /* (ii) step in dual space */
          for (int k = 0; k < iq; k++) u[k] -= t * r[k];
          u[iq] += t;
          iai[l] = l;
          qp_delete(&w, A, u, p, &iq, l);
          continue;
        }
        /* (iii) step in primal and dual space */
        for (int k = 0; k < n; k++) x[k] += t * z[k];
        f += t * znp * (0.5 * t + u[iq]);
        for (int k = 0; k < iq; k++) u[k] -= t * r[k];
        u[iq] += t;
        if (fabs(t - t2) < QP_EPS) {  /* full step: add ip */
          if (!qp_add(&w, &iq, &rnorm)) {
            iaexcl[ip] = 0;
            qp_delete(&w, A, u, p, &iq, ip);
            for (int i = 0; i < m; i++) iai[i] = i;
            for (int i = p; i < iq; i++) { A[i] = A_old[i]; u[i] = u_old[i]; iai[A[i]] = -1; }
            for (int i = 0; i < n; i++) x[i] = x_old[i];
            break;  /* goto l2 */
          }
          iai[ip] = -1;
          go_l1 = 1;
          break;
        }
        /* partial step: drop l, refresh s[ip] */
        iai[l] = l;
        qp_delete(&w, A, u, p, &iq, l);
        double sum = 0.0;
        for (int k = 0; k < n; k++) sum += CI[k * ldci + ip] * x[k];
        s[ip] = sum + ci0[ip];
      }
    }
  }
}

/* Batched driver over row-major blocks with per-instance dims (or the maxima when dims == NULL). */
void oracle_quadprog_batch(int batch, int n_max, int p_max, int m_max, const int32_t* dims,
                           const double* G, const double* g0, const double* CE, const double* ce0,
                           const double* CI, const double* ci0, int max_iter, double* x,
                           double* fval, uint8_t* status, int32_t* iters) {
  for (int b = 0; b < batch; b++) {
    const int n = dims ? dims[3 * b] : n_max, p = dims ? dims[3 * b + 1] : p_max,
              m = dims ? dims[3 * b + 2] : m_max;
    int it = 0;
    double* xb = x + (size_t)b * n_max;
    for (int i = 0; i < n_max; i++) xb[i] = 0.0;
    const int st = oracle_quadprog(n, p, m, G + (size_t)b * n_max * n_max, n_max,
                                   g0 + (size_t)b * n_max, CE + (size_t)b * n_max * p_max, p_max,
                                   ce0 + (size_t)b * p_max, CI + (size_t)b * n_max * m_max, m_max,
                                   ci0 + (size_t)b * m_max, max_iter, xb, &fval[b], &it);
    if (st != CMPC_OK)
      for (int i = 0; i < n_max; i++) xb[i] = 0.0;
    status[b] = (uint8_t)st;
    if (iters) iters[b] = it;
  }
}
