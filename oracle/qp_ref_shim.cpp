/*
 * TEST INFRASTRUCTURE ONLY (checker + CPU baseline; see cmpc_oracle.h).
 *
 * C wrapper around the reference's vendored qpOASES 3.2.0
 * (be2r_cmpc_unitree/src/third_party/qpOASES), compiled from its sources under /root/reference
 * by oracle/Makefile into oracle/_ref/libcmpc_ref.so. Nothing of qpOASES is copied into this
 * repository; this file only calls it exactly as SolverMPC.cpp:952-982 does:
 *   QProblem(new_vars, new_cons); Options::setToMPC(); printLevel = PL_NONE;
 *   init(H_red, g_red, A_red, NULL, NULL, lb_red, ub_red, nWSR = 100); getPrimalSolution(q_red).
 *
 * ref_solve_batch() chains the fp32 condensation restatement (cmpc_oracle.c) with that qpOASES
 * call per instance: the reference's whole solve_mpc() on one CPU thread per worker.
 */
#include <qpOASES.hpp>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "cmpc_oracle.h"

extern "C" int qpref_solve(int nv, int nc, const double* H, const double* g, const double* A,
                           const double* lb, const double* ub, int nwsr_max, double* x,
                           int* nwsr_out, int* rval_init) {
  qpOASES::QProblem problem_red(nv, nc);
  qpOASES::Options op;
  op.setToMPC();
  op.printLevel = qpOASES::PL_NONE;
  problem_red.setOptions(op);
  qpOASES::int_t nWSR = nwsr_max;
  int rval = problem_red.init(H, g, A, NULL, NULL, lb, ub, nWSR);
  int rval2 = problem_red.getPrimalSolution(x);
  if (nwsr_out) *nwsr_out = (int)nWSR;
  if (rval_init) *rval_init = rval;
  return rval2;
}

namespace {
struct Scratch {
  std::vector<float> qH, qg;
  std::vector<double> H, g, A, lb, ub, q_red;
  std::vector<char> var_elim, con_elim;
  std::vector<unsigned char> ws_cond, ws_red;
  explicit Scratch(int N)
      : qH(144 * N * N), qg(12 * N), H(144 * N * N), g(12 * N), A(240 * N * N), lb(20 * N),
        ub(20 * N), q_red(12 * N), var_elim(12 * N), con_elim(20 * N),
        ws_cond(oracle_condense_ws_bytes(N)), ws_red(oracle_reduce_ws_bytes(N)) {}
};

int solve_one(const float* rec, const cmpc_params* prm, Scratch& s, double* q_soln, int* nwsr) {
  oracle_cond c;
  c.qH = s.qH.data();
  c.qg = s.qg.data();
  int st = oracle_condense_ws(rec, prm, &c, s.ws_cond.data());
  if (st != CMPC_OK) return st;
  oracle_red red;
  red.H = s.H.data(); red.g = s.g.data(); red.A = s.A.data();
  red.lb = s.lb.data(); red.ub = s.ub.data();
  red.var_elim = s.var_elim.data(); red.con_elim = s.con_elim.data();
  oracle_reduce_ws(rec, prm, s.qH.data(), s.qg.data(), &red, s.ws_red.data());
  int rinit = 0;
  std::fill(s.q_red.begin(), s.q_red.end(), 0.0);
  if (red.nv == 0) {
    /* every leg in swing: the reference still calls QProblem(0, 0), which qpOASES rejects
     * ("invalid arguments", failed-to-solve print); q_soln is all zeros either way. */
    oracle_scatter(&red, s.q_red.data(), q_soln);
    if (nwsr) *nwsr = 0;
    return CMPC_OK;
  }
  int r2 = qpref_solve(red.nv, red.nc, red.H, red.g, red.A, red.lb, red.ub,
                       prm->max_iter > 0 ? prm->max_iter : 100, s.q_red.data(), nwsr, &rinit);
  oracle_scatter(&red, s.q_red.data(), q_soln);
  if (r2 != qpOASES::SUCCESSFUL_RETURN) return CMPC_MAX_ITER;
  if (rinit == qpOASES::RET_MAX_NWSR_REACHED) return CMPC_MAX_ITER;
  if (rinit != qpOASES::SUCCESSFUL_RETURN) return CMPC_INFEASIBLE;
  return CMPC_OK;
}
}  // namespace

/* The reference pipeline over a batch of records (layout include/cmpc_solver.h), nthreads
 * std::threads with one private scratch each (the reference itself is non-reentrant). */
extern "C" int ref_solve_batch(const float* records, int batch, const cmpc_params* prm,
                               double* q_soln, int* status, int* nwsr, int nthreads) {
  const int N = prm->horizon;
  const int stride = CMPC_REC_WORDS(N);
  const int nv = 12 * N;
  std::atomic<int> next(0);
  auto worker = [&]() {
    Scratch s(N);
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= batch) break;
      int nw = 0;
      const int st = solve_one(records + (size_t)i * stride, prm, s, q_soln + (size_t)i * nv, &nw);
      if (status) status[i] = st;
      if (nwsr) nwsr[i] = nw;
    }
  };
  nthreads = std::max(1, nthreads);
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; t++) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  return 0;
}

/* Config 5: per instance the residual of the logged previous step (ConvexMPCLocomotion.cpp:639-771)
 * and one estimator step (SolverMPC.cpp:688-798) ahead of the solve, as the reference runs them
 * inside each solveDenseMPC -> solve_mpc call. records / est_states are updated in place
 * (f_est(3) + use-f_est flag into the record, as qg reads them at SolverMPC.cpp:808-811). */
extern "C" int ref_pipeline_c5_batch(float* records, const float* logs, float* est_states,
                                     int batch, const cmpc_params* prm, float sim_time,
                                     double* q_soln, int* status, int nthreads) {
  const int N = prm->horizon;
  const int stride = CMPC_REC_WORDS(N);
  const int nv = 12 * N;
  std::atomic<int> next(0);
  auto worker = [&]() {
    Scratch s(N);
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= batch) break;
      float* rec = records + (size_t)i * stride;
      float fext[6];
      oracle_residual(logs + (size_t)i * CMPC_LOG_WORDS, rec, fext);
      int use = 0;
      const float f3 = oracle_est_step(est_states + (size_t)i * CMPC_EST_WORDS, fext[3], sim_time, &use);
      rec[CMPC_REC_FEST3] = f3;
      const uint32_t flags = use ? 1u : 0u;
      std::memcpy(rec + CMPC_REC_FLAGS, &flags, 4);
      int nw = 0;
      const int st = solve_one(rec, prm, s, q_soln ? q_soln + (size_t)i * nv : s.q_red.data(), &nw);
      if (status) status[i] = st;
    }
  };
  nthreads = std::max(1, nthreads);
  std::vector<std::thread> pool;
  for (int t = 1; t < nthreads; t++) pool.emplace_back(worker);
  worker();
  for (auto& t : pool) t.join();
  return 0;
}
