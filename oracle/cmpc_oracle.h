/*
 * TEST INFRASTRUCTURE ONLY — never linked into, loaded by, or called from the product path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, as the checker.
 *
 * CPU restatement of the reference's per-instance MPC condensation and swing-leg elimination
 * (be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-982, RobotState.cpp:9-50),
 * reference-faithful: fp32 throughout, dense 13N x 13N weight matrix S, dense GEMMs in the order
 * Eigen evaluates SolverMPC.cpp:806-814. The QP itself is solved by the reference's vendored
 * qpOASES 3.2.0, compiled from /root/reference into oracle/_ref/ (see oracle/Makefile and
 * oracle/qp_ref_shim.cpp).
 *
 * Parity pinning: the QP stage is pinned by the reference's own qpOASES built here; the
 * condensation restatement cannot be pinned against the reference binary (SolverMPC.cpp needs
 * Eigen3/FFTW3/ROS headers absent in this image) and is cross-checked instead against
 * independent math (scipy.linalg.expm, forward simulation) in tests/test_oracle.py.
 */
#ifndef CMPC_ORACLE_H
#define CMPC_ORACLE_H

#include "../include/cmpc_solver.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Intermediates of one condensation (sizes for horizon N; caller-allocated, may be NULL). */
typedef struct oracle_cond {
  float x0[13];
  float Adt[13 * 13];   /* row-major */
  float Bdt[13 * 12];   /* row-major */
  float Qdt[13 * 6];    /* row-major */
  float* qH;            /* [12N * 12N] row-major, may be NULL */
  float* qg;            /* [12N] */
} oracle_cond;

/* Reduced QP exactly as handed to qpOASES (SolverMPC.cpp:841-950). */
typedef struct oracle_red {
  int nv, nc;           /* reduced sizes */
  int nv_full, nc_full;
  double* H;            /* [nv*nv] row-major (capacity 144 N^2) */
  double* g;            /* [nv] */
  double* A;            /* [nc*nv] row-major (capacity 240 N^2) */
  double* lb;           /* [nc] */
  double* ub;           /* [nc] */
  char* var_elim;       /* [12N] */
  char* con_elim;       /* [20N] */
} oracle_red;

/* Summation order of the condensation's fp32 dot products (process-wide; 0 = the default
 * sequential order, 1 = blocked k-outer panels of 8, 2 = pairwise; cmpc_oracle.c). Only the
 * summation-order spread of the fp64-branch evidence uses 1 and 2 (scripts/branch_orders.py). */
void oracle_set_sum_order(int order);
int oracle_sum_order(void);
/* Implementation of the dense qH / qg products: 0 the naive loops (default), 1 register-tiled
 * GEMMs in the same summation order, bit for bit (the CPU baseline's; cmpc_oracle.c). */
void oracle_set_impl(int impl);

/* Condense one record (layout: include/cmpc_solver.h). qH/qg computed as the reference does. */
int oracle_condense(const float* rec, const cmpc_params* prm, oracle_cond* out);

/* Same with a caller-provided workspace of oracle_condense_ws_bytes(N) bytes (no malloc). */
size_t oracle_condense_ws_bytes(int horizon);
int oracle_condense_ws(const float* rec, const cmpc_params* prm, oracle_cond* out, void* ws);

/* Elimination + reduction from a condensed (qH, qg) and the record's gait. */
int oracle_reduce(const float* rec, const cmpc_params* prm, const float* qH, const float* qg,
                  oracle_red* red);

size_t oracle_reduce_ws_bytes(int horizon);
int oracle_reduce_ws(const float* rec, const cmpc_params* prm, const float* qH, const float* qg,
                     oracle_red* red, void* ws);

/* Scatter a reduced solution back to q_soln[12N] (0 for eliminated), SolverMPC.cpp:970-982. */
void oracle_scatter(const oracle_red* red, const double* q_red, double* q_soln);

/* ---- Config 5: periodic-disturbance estimation ---------------------------------------------
 * gaussian_filter (SolverMPC.cpp:404-437), fit_sin (:478-541) with the FFTW r2c magnitudes
 * evaluated by a direct DFT, the estimator step (:688-798) on a CMPC_EST_WORDS state with the
 * device layout, and the caller's residual (ConvexMPCLocomotion.cpp:639-771). */
void oracle_gaussian_filter(const double* data, int n, float sigma, double* out);
void oracle_fit_sin(const double* tt, const double* yy, int n, double* amp, double* freq,
                    double* phase, double* offset, int* peak_bin);
void oracle_residual(const float* log, const float* rec, float f_ext[6]);
/* Pushes (f3, t); returns f_est(3); *use_f_est = (count > 500), the qg switch of :808. */
float oracle_est_step(float* state, float f3, float t, int* use_f_est);


/* QuadProg++ solve_quadprog restatement (quadprog_oracle.c, built into _build/libqp_oracle.so
 * with -ffp-contract=off). Returns the CMPC_* status; fval = +inf when infeasible. */
int oracle_quadprog(int n, int p, int m, const double* G, int ldg, const double* g0,
                    const double* CE, int ldce, const double* ce0, const double* CI, int ldci,
                    const double* ci0, int max_iter, double* x, double* fval, int* iters_out);
void oracle_quadprog_batch(int batch, int n_max, int p_max, int m_max, const int32_t* dims,
                           const double* G, const double* g0, const double* CE, const double* ce0,
                           const double* CI, const double* ci0, int max_iter, double* x,
                           double* fval, uint8_t* status, int32_t* iters);

#ifdef __cplusplus
}
#endif
#endif
