/*
 * cmpc_quadprog.h — batched Goldfarb-Idnani QP on the GPU: the drop-in for QuadProg++'s
 * solve_quadprog (be2r_cmpc_unitree/src/third_party/Goldfarb_Optimizer/QuadProg++.hh:71-77,
 * QuadProg++.cc:108-507) as WBIC::MakeTorque calls it once per control tick
 * (be2r_cmpc_unitree/src/controllers/WBC/WBIC/WBIC.cpp:91), for a batch of independent problems
 *
 *     min 0.5 x'Gx + g0'x   s.t.   CE'x + ce0 = 0,   CI'x + ci0 >= 0.
 *
 * fp64 throughout, as QuadProg++. Layout per instance b (row-major, QuadProg++'s orientation: a
 * constraint per COLUMN of CE / CI), with fixed strides from the batch maxima:
 *     G   [b][n_max][n_max]   g0  [b][n_max]
 *     CE  [b][n_max][p_max]   ce0 [b][p_max]
 *     CI  [b][n_max][m_max]   ci0 [b][m_max]
 *     x   [b][n_max] (out; entries >= n are 0)   f [b] (out: objective, +inf when infeasible)
 * d_dims: [b][3] = (n, p, m) of each instance, or NULL when every instance is (n_max, p_max,
 * m_max). WBIC's problems: n = 6 + 3 contacts, p = 6, m = 6 contacts (m = 1 with a zero row when
 * no foot is in contact, WBIC.cpp:341-345). Limits: n_max <= 32, p <= n, m_max <= 64.
 *
 * Status per instance (cmpc_solver.h codes): CMPC_OK; CMPC_INFEASIBLE (solve_quadprog returns
 * +inf); CMPC_NOT_PD (cholesky_decomposition throws); CMPC_BAD_INPUT (linearly dependent
 * equality constraints: the reference throws; or dims out of range); CMPC_MAX_ITER (the
 * reference has no cap; here max_iter active-set steps). G is not modified (the reference
 * overwrites it with its Cholesky factor). Asynchronous on the handle's stream.
 */
#ifndef CMPC_QUADPROG_H
#define CMPC_QUADPROG_H

#include "cmpc_solver.h"

#define CMPC_QP_NMAX 32
#define CMPC_QP_MMAX 64

CMPC_EXTERNC int cmpc_batch_quadprog(cmpc_batch* h, int n_max, int p_max, int m_max,
                                     const int32_t* d_dims, const double* d_G, const double* d_g0,
                                     const double* d_CE, const double* d_ce0, const double* d_CI,
                                     const double* d_ci0, int max_iter, double* d_x, double* d_f,
                                     uint8_t* d_status, int32_t* d_iters, int batch);

#endif
