// cmpc_assemble.hip — the batched controller loop around the solver:
//   * cmpc_assemble_kernel: on-device MPC input assembly (rank 1, below);
//   * cmpc_rollout_kernel: the single-rigid-body step x+ = Adt x + Bdt u0 + Qdt xi that closes
//     the loop in a batched MPC simulator (rank 2, at the end of this file).
//
// One thread advances one instance's locomotion controller by one control tick, doing exactly
// the MPC-input side of ConvexMPCLocomotion::run (be2r_cmpc_unitree/src/controllers/convexMPC/
// ConvexMPCLocomotion.cpp):
//   _SetupCommand           :100-123  first-order command filter (filter 0.1), yaw/roll/pitch_des 0
//   setIterations           Gait.cpp:218-226  _iteration = (counter / iters) % P
//   v_des_world             :210-211  rBody^T v_des_robot (omniMode: v_des_robot)
//   rpy_int / rpy_comp      :218-230  integral pitch / roll compensation, clamped to +-0.25
//   world_position_desired  :237-257  += dt v_des_world (not standing); first run: = position
//   foot placement          :276-331  swingTimeRemaining, Raibert / capture-point foothold Pf with
//                           the pfx_rel / pfy_rel clamps, interleave offsets, yaw correction
//   iterationCounter++      :334
//   getMpcTable             Gait.cpp:159-188 (rows i < N; periodic for N > P)
//   updateMPCIfNeeded       :511-586  every `iters` ticks: the trajAll reference
//   solveDenseMPC inputs    :619-633, :786-790, :806-818  p = (x, y, z_groundtruth), r = pFoot - p,
//                           x_drag = x_comp_integral, then the x_comp_integral update
//   swing / stance          :337-431  getSwingState, firstSwing, Bezier pDesFootWorld
// and, when an MPC step is due, writes the instance's solve record (include/cmpc_solver.h) for
// cmpc_batch_solve: the record the reference would hand to update_problem_data_floats.
//
// The work is a few hundred scalar flops per instance: the kernel is HBM-bound (224 B of state
// read + written, one 16-B-aligned record written per due instance). Floating-point
// contraction is off so results are bit-identical to the fp32 restatement in oracle/oracle.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cmpc_common.h"

#pragma clang fp contract(off)

namespace cmpc {
namespace {

__global__ __launch_bounds__(256) void cmpc_assemble_kernel(float* __restrict__ loco, LocoParams lp,
                                                            float* __restrict__ recs,
                                                            uint8_t* __restrict__ due, int batch) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch) return;
  float* s = loco + (size_t)i * CMPC_LOCO_WORDS;
  const float dt = lp.dt;
  const int iters = lp.iters_between_mpc;
  const int N = lp.horizon;
  const uint32_t flags = __float_as_uint(s[CMPC_LOCO_FLAGS]);
  const bool omni = flags & CMPC_LOCO_OMNI, standing = flags & CMPC_LOCO_STANDING,
             pronk = flags & CMPC_LOCO_PRONK;
  const float pos0 = s[CMPC_LOCO_POS + 0], pos1 = s[CMPC_LOCO_POS + 1], pos2 = s[CMPC_LOCO_POS + 2];
  const float vw0 = s[CMPC_LOCO_VW + 0], vw1 = s[CMPC_LOCO_VW + 1];
  const float rpy0 = s[CMPC_LOCO_RPY + 0], rpy1 = s[CMPC_LOCO_RPY + 1], rpy2 = s[CMPC_LOCO_RPY + 2];

  // _SetupCommand (:114-122): _x_vel_des = _x_vel_des (1 - filter) + x_vel_cmd filter
  const float filter = 0.1f;
  const float vdx = s[CMPC_LOCO_VDES + 0] * (1.f - filter) + s[CMPC_LOCO_CMD + 0] * filter;
  const float vdy = s[CMPC_LOCO_VDES + 1] * (1.f - filter) + s[CMPC_LOCO_CMD + 1] * filter;
  const float yaw_rate = s[CMPC_LOCO_CMD + 2];
  const float roll_des = 0.f, pitch_des = 0.f, yaw_des = 0.f;
  s[CMPC_LOCO_VDES + 0] = vdx;
  s[CMPC_LOCO_VDES + 1] = vdy;

  // setIterations (Gait.cpp:218-226)
  const int counter = __float_as_int(s[CMPC_LOCO_COUNTER]);
  const int P = __float_as_int(s[CMPC_LOCO_GAIT + 0]);
  const int iteration = (counter / iters) % P;

  // v_des_world = rBody^T v_des_robot; rBody^T is quaternionToRotationMatrix before its
  // transposeInPlace (common/Math/orientation_tools.h:195-211)
  const float e0 = s[CMPC_LOCO_Q + 0], e1 = s[CMPC_LOCO_Q + 1], e2 = s[CMPC_LOCO_Q + 2],
              e3 = s[CMPC_LOCO_Q + 3];
  float vdw0 = vdx, vdw1 = vdy;
  if (!omni) {
    const float R00 = 1.f - 2.f * (e2 * e2 + e3 * e3), R01 = 2.f * (e1 * e2 - e0 * e3),
                R02 = 2.f * (e1 * e3 + e0 * e2);
    const float R10 = 2.f * (e1 * e2 + e0 * e3), R11 = 1.f - 2.f * (e1 * e1 + e3 * e3),
                R12 = 2.f * (e2 * e3 - e0 * e1);
    vdw0 = R00 * vdx + R01 * vdy + R02 * 0.f;
    vdw1 = R10 * vdx + R11 * vdy + R12 * 0.f;
  }

  // rpy_int / rpy_comp (:218-230)
  float ri0 = s[CMPC_LOCO_RPYINT + 0], ri1 = s[CMPC_LOCO_RPYINT + 1];
  if (fabsf(vw0) > .2f) ri1 += dt * (pitch_des - rpy1) / vw0;
  if (fabsf(vw1) > 0.1f) ri0 += dt * (roll_des - rpy0) / vw1;
  ri0 = fminf(fmaxf(ri0, -.25f), .25f);
  ri1 = fminf(fmaxf(ri1, -.25f), .25f);
  const float comp1 = vw0 * ri1;
  const float comp0 = vw1 * ri0 * (pronk ? 0.f : 1.f);
  s[CMPC_LOCO_RPYINT + 0] = ri0;
  s[CMPC_LOCO_RPYINT + 1] = ri1;

  // world_position_desired (:237-257)
  float wx = s[CMPC_LOCO_WPD + 0], wy = s[CMPC_LOCO_WPD + 1];
  if (!standing) {
    wx += dt * vdw0;
    wy += dt * vdw1;
  }
  uint32_t nflags = flags;
  float pfoot[4][3];
#pragma unroll
  for (int l = 0; l < 4; l++)
#pragma unroll
    for (int k = 0; k < 3; k++) pfoot[l][k] = s[CMPC_LOCO_PFOOT + 3 * l + k];
  if (flags & CMPC_LOCO_FIRST) {
    wx = pos0;
    wy = pos1;
    nflags &= ~(uint32_t)CMPC_LOCO_FIRST;
    // :258-271 setInitialPosition / setFinalPosition(pFoot[i])
#pragma unroll
    for (int t = 0; t < 12; t++) {
      s[CMPC_LOCO_P0 + t] = pfoot[t / 3][t % 3];
      s[CMPC_LOCO_PF + t] = pfoot[t / 3][t % 3];
    }
  }

  // foot placement (:276-331): swingTimeRemaining and the foothold Pf of every leg
  const int off[4] = {__float_as_int(s[CMPC_LOCO_GAIT + 1]), __float_as_int(s[CMPC_LOCO_GAIT + 2]),
                      __float_as_int(s[CMPC_LOCO_GAIT + 3]), __float_as_int(s[CMPC_LOCO_GAIT + 4])};
  const int dur[4] = {__float_as_int(s[CMPC_LOCO_GAIT + 5]), __float_as_int(s[CMPC_LOCO_GAIT + 6]),
                      __float_as_int(s[CMPC_LOCO_GAIT + 7]), __float_as_int(s[CMPC_LOCO_GAIT + 8])};
  const float dtm0 = dt * (float)iters;                  // recompute_timing (:95-99, :207)
  const float swing_time = dtm0 * (float)(P - dur[0]);   // Gait.cpp:252-256 (_swing)
  const float stance_time = dtm0 * (float)dur[0];        // Gait.cpp:263-267 (_stance)
  {
    const float R00 = 1.f - 2.f * (e2 * e2 + e3 * e3), R01 = 2.f * (e1 * e2 - e0 * e3),
                R02 = 2.f * (e1 * e3 + e0 * e2);
    const float R10 = 2.f * (e1 * e2 + e0 * e3), R11 = 1.f - 2.f * (e1 * e1 + e3 * e3),
                R12 = 2.f * (e2 * e3 - e0 * e1);
    const float side[4] = {-1.f, 1.f, -1.f, 1.f};
    const float ily[4] = {-0.08f, 0.08f, 0.02f, -0.02f};
    const float igain = -0.2f;
    const float v_abs = fabsf(vdx);
    const float th = -yaw_rate * stance_time / 2.f;      // coordinateRotation(Z, th) (:307)
    // sin / cos through double, rounded once: the correctly rounded float (glibc's sinf / cosf
    // are correctly rounded too), so the kernel and the oracle agree bit for bit
    const float cth = (float)cos((double)th), sth = (float)sin((double)th);
    const float hz = 0.5f * pos2 / 9.81f;
#pragma unroll
    for (int l = 0; l < 4; l++) {
      float swrem = s[CMPC_LOCO_SWREM + l];
      swrem = (flags & (CMPC_LOCO_FSWING0 << l)) ? swing_time : swrem - dt;
      s[CMPC_LOCO_SWREM + l] = swrem;
      const float hx = (l == 0 || l == 1) ? lp.hip_x : -lp.hip_x;
      const float hy = (l == 1 || l == 3) ? lp.hip_y : -lp.hip_y;
      float prf0 = hx + 0.f, prf1 = hy + side[l] * lp.abad_link, prf2 = 0.f + 0.f;
      prf1 = prf1 + ily[l] * v_abs * igain;
      const float py0 = cth * prf0 + sth * prf1 + 0.f * prf2;
      const float py1 = -sth * prf0 + cth * prf1 + 0.f * prf2;
      const float py2 = 0.f * prf0 + 0.f * prf1 + 1.f * prf2;
      const float t0 = py0 + vdx * swrem, t1 = py1 + vdy * swrem, t2 = py2 + 0.f * swrem;
      const float pf0 = pos0 + (R00 * t0 + R01 * t1 + R02 * t2);
      const float pf1 = pos1 + (R10 * t0 + R11 * t1 + R12 * t2);
      // :318-322; the double literals promote the first terms to double
      float pfx = (float)((double)vw0 * (0.5 + (double)lp.bonus_swing) * (double)stance_time +
                          (double)(0.03f * (vw0 - vdw0)) + (double)(hz * (vw1 * yaw_rate)));
      float pfy = (float)((double)vw1 * 0.5 * (double)stance_time * (double)dtm0 +
                          (double)(0.03f * (vw1 - vdw1)) + (double)(hz * (-vw0 * yaw_rate)));
      pfx = fminf(fmaxf(pfx, -0.3f), 0.3f);
      pfy = fminf(fmaxf(pfy, -0.3f), 0.3f);
      s[CMPC_LOCO_PF + 3 * l + 0] = pf0 + pfx;
      s[CMPC_LOCO_PF + 3 * l + 1] = pf1 + pfy;
      s[CMPC_LOCO_PF + 3 * l + 2] = 0.f;
    }
  }

  // iterationCounter++ (:334); updateMPCIfNeeded (:514) tests the incremented counter
  const int nc = counter + 1;
  s[CMPC_LOCO_COUNTER] = __int_as_float(nc);
  const bool mpc = (nc % iters) == 0;
  const float dtMPC = dt * (float)iters;
  float xci = s[CMPC_LOCO_XCI];
  if (mpc) {
    float* rec = recs + (size_t)i * lp.rec_words;
    float traj0[12];
    if (standing) {  // :529-533
      traj0[0] = roll_des; traj0[1] = pitch_des; traj0[2] = s[CMPC_LOCO_STAND + 2];
      traj0[3] = s[CMPC_LOCO_STAND + 0]; traj0[4] = s[CMPC_LOCO_STAND + 1];
    } else {  // :537-566, desired xy kept within 0.1 of the measured position
      const float max_pos_error = .1f;
      float xs = wx, ys = wy;
      if (xs - pos0 > max_pos_error) xs = pos0 + max_pos_error;
      if (pos0 - xs > max_pos_error) xs = pos0 - max_pos_error;
      if (ys - pos1 > max_pos_error) ys = pos1 + max_pos_error;
      if (pos1 - ys > max_pos_error) ys = pos1 - max_pos_error;
      wx = xs;
      wy = ys;
      traj0[0] = comp0; traj0[1] = comp1; traj0[2] = yaw_des; traj0[3] = xs; traj0[4] = ys;
    }
    traj0[5] = s[CMPC_LOCO_HEIGHT];
    traj0[6] = 0.f; traj0[7] = 0.f;
    traj0[8] = standing ? 0.f : yaw_rate;
    traj0[9] = standing ? 0.f : vdw0;
    traj0[10] = standing ? 0.f : vdw1;
    traj0[11] = 0.f;
    float* traj = rec + CMPC_REC_TRAJ(N);
    float px = traj0[3], py = traj0[4], pyaw = rpy2;
    for (int k = 0; k < N; k++) {  // :568-585
#pragma unroll
      for (int j = 0; j < 12; j++) traj[12 * k + j] = traj0[j];
      if (!standing) {
        if (k > 0) {
          px = px + dtMPC * vdw0;
          py = py + dtMPC * vdw1;
          pyaw = pyaw + dtMPC * yaw_rate;
        }
        traj[12 * k + 2] = pyaw;
        traj[12 * k + 3] = px;
        traj[12 * k + 4] = py;
      }
    }
    // getMpcTable (Gait.cpp:159-188) with the _iteration of this tick
    uint32_t* gw = reinterpret_cast<uint32_t*>(rec + CMPC_REC_GAIT(N));
    for (int k = 0; k < N; k++) {
      const int it = (k + iteration + 1) % P;
      uint32_t word = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) {
        int prog = it - __float_as_int(s[CMPC_LOCO_GAIT + 1 + j]);
        if (prog < 0) prog += P;
        if (prog < __float_as_int(s[CMPC_LOCO_GAIT + 5 + j])) word |= 1u << (8 * j);
      }
      gw[k] = word;
    }
    // solveDenseMPC inputs (:619-633, :786-790)
    const float zgt = s[CMPC_LOCO_ZGT];
    rec[CMPC_REC_P + 0] = pos0;
    rec[CMPC_REC_P + 1] = pos1;
    rec[CMPC_REC_P + 2] = zgt;
#pragma unroll
    for (int k = 0; k < 3; k++) {
      rec[CMPC_REC_V + k] = s[CMPC_LOCO_VW + k];
      rec[CMPC_REC_W + k] = s[CMPC_LOCO_WW + k];
      rec[CMPC_REC_RPY + k] = s[CMPC_LOCO_RPY + k];
    }
#pragma unroll
    for (int k = 0; k < 4; k++) rec[CMPC_REC_Q + k] = s[CMPC_LOCO_Q + k];
    const float pp[3] = {pos0, pos1, pos2};
#pragma unroll
    for (int t = 0; t < 12; t++) rec[CMPC_REC_R + t] = s[CMPC_LOCO_PFOOT + 3 * (t % 4) + t / 4] - pp[t / 4];
    rec[CMPC_REC_XDRAG] = xci;  // update_x_drag(x_comp_integral) precedes the update (:809)
    rec[CMPC_REC_FEST3] = 0.f;
    rec[CMPC_REC_FLAGS] = 0.f;
    rec[31] = 0.f;
    // x_comp_integral (:802, :813-818): pz_err uses p[2] = z_groundtruth
    const float pz_err = zgt - s[CMPC_LOCO_HEIGHT];
    if (vw0 > 0.3f || vw0 < -0.3f) xci += lp.x_drag_gain * pz_err * dtMPC / vw0;
    s[CMPC_LOCO_XCI] = xci;
  }
  s[CMPC_LOCO_WPD + 0] = wx;
  s[CMPC_LOCO_WPD + 1] = wy;

  // swing / stance of each foot (:337-338, :350-431): getSwingState (Gait.cpp:102-135) at the
  // phase of setIterations (Gait.cpp:218-226, pre-increment counter), then the Bezier swing
  // (FootSwingTrajectory.cpp:17-42, Interpolation.h:30-37)
  const float phase = (float)(counter % (iters * P)) / (float)(iters * P);
#pragma unroll
  for (int l = 0; l < 4; l++) {
    const float offf = (float)off[l] / (float)P, durf = (float)dur[l] / (float)P;
    float so = offf + durf;
    if (so > 1.f) so = so - 1.f;
    const float sd = 1.f - durf;
    float prog = phase - so;
    if (prog < 0.f) prog = prog + 1.f;
    prog = (prog >= sd) ? 0.f : prog / sd;
    s[CMPC_LOCO_SWST + l] = prog;
    const uint32_t fbit = CMPC_LOCO_FSWING0 << l;
    const bool first_before = (nflags & fbit) != 0u;
    if (prog > 0.f) {
      float a[3];
      if (first_before) {
        nflags &= ~fbit;
#pragma unroll
        for (int k = 0; k < 3; k++) { a[k] = pfoot[l][k]; s[CMPC_LOCO_P0 + 3 * l + k] = a[k]; }
      } else {
#pragma unroll
        for (int k = 0; k < 3; k++) a[k] = s[CMPC_LOCO_P0 + 3 * l + k];
      }
      const float b0 = s[CMPC_LOCO_PF + 3 * l + 0], b1 = s[CMPC_LOCO_PF + 3 * l + 1],
                  b2 = s[CMPC_LOCO_PF + 3 * l + 2];
      const float x = prog;
      const float bez = x * x * x + 3.f * (x * x * (1.f - x));
      float pd0 = a[0] + bez * (b0 - a[0]);
      float pd1 = a[1] + bez * (b1 - a[1]);
      float u, y0, yf;
      if (x < 0.5f) { u = x * 2.f; y0 = a[2]; yf = a[2] + lp.swing_height; }
      else { u = x * 2.f - 1.f; y0 = a[2] + lp.swing_height; yf = b2; }
      const float bz = u * u * u + 3.f * (u * u * (1.f - u));
      const float pd2 = y0 + bz * (yf - y0);
      s[CMPC_LOCO_PDES + 3 * l + 0] = pd0;
      s[CMPC_LOCO_PDES + 3 * l + 1] = pd1;
      s[CMPC_LOCO_PDES + 3 * l + 2] = pd2;
      if (flags & CMPC_LOCO_SIMFEET) {
        s[CMPC_LOCO_PFOOT + 3 * l + 0] = pd0;
        s[CMPC_LOCO_PFOOT + 3 * l + 1] = pd1;
        s[CMPC_LOCO_PFOOT + 3 * l + 2] = pd2;
      }
    } else {
      nflags |= fbit;  // firstSwing = true (:413)
      if ((flags & CMPC_LOCO_SIMFEET) && !first_before) s[CMPC_LOCO_PFOOT + 3 * l + 2] = 0.f;
    }
  }
  s[CMPC_LOCO_FLAGS] = __uint_as_float(nflags);
  due[i] = mpc ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------
// Rollout: advance each due instance by one MPC step with its own prediction model, the
// discretised single rigid body of solve_mpc (RobotState::set + ct_ss_mats + c2qp,
// SolverMPC.cpp:96-146, 260-279, 566-620; cmpc_common.h), driven by the step-0 forces of the
// solve and an optional disturbance xi (the f_ext layout [tau(3), f(3)] of Q_ct,
// SolverMPC.cpp:607-615):
//   x+ = Adt x0 + Bdt u0 + Qdt xi,  Qdt = dt Q + dt^2/2 A Q + dt^3/6 A^2 Q (A^3 = 0),
// with x0 = [rpy, p, w, v, -9.8] from the record. The new rpy / p / w / v are written back to
// the controller state (quaternion from ZYX Euler angles, z_groundtruth = p_z). Feet: with
// CMPC_LOCO_SIMFEET the assemble kernel moves them (swing feet on their Bezier trajectory, touch
// down at the foothold Pf, stance feet fixed in the world) and the rollout leaves them alone;
// without it they keep their offset from the body in x and y. One thread per instance.
__global__ __launch_bounds__(256) void cmpc_rollout_kernel(float* __restrict__ loco,
                                                           const float* __restrict__ recs,
                                                           const float* __restrict__ forces,
                                                           const float* __restrict__ xi6,
                                                           const uint8_t* __restrict__ due,
                                                           LocoParams lp, float dt, int batch) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch || (due && !due[i])) return;
  const float* rec = recs + (size_t)i * lp.rec_words;
  const float* u = forces + (size_t)i * lp.out_cols;  // step 0: 12 forces, leg * 3 + axis
  Model md;
  make_model(rec, dt, md);
  float BdtT[12][16];
#pragma unroll
  for (int c = 0; c < 12; c++) make_bdt<12>(rec, md, c, BdtT);
  float x0[13];
  {
    const float qw = rec[CMPC_REC_Q + 0], qx = rec[CMPC_REC_Q + 1], qy = rec[CMPC_REC_Q + 2],
                qz = rec[CMPC_REC_Q + 3];
    float as = -2.f * (qx * qz - qw * qy);
    as = fminf(as, 0.99999f);  // quat_to_rpy (SolverMPC.cpp:352-361)
    x0[0] = atan2f(2.f * (qy * qz + qw * qx), qw * qw - qx * qx - qy * qy + qz * qz);
    x0[1] = asinf(as);
    x0[2] = atan2f(2.f * (qx * qy + qw * qz), qw * qw + qx * qx - qy * qy - qz * qz);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      x0[3 + k] = rec[CMPC_REC_P + k];
      x0[6 + k] = rec[CMPC_REC_W + k];
      x0[9 + k] = rec[CMPC_REC_V + k];
    }
    x0[12] = -9.8f;
  }
  float x1[13];
  n1_mul(md, x0, x1);  // Adt x0 = x0 + N1 x0
#pragma unroll
  for (int j = 0; j < 13; j++) x1[j] = x0[j] + x1[j];
#pragma unroll
  for (int c = 0; c < 12; c++) {
    const float uc = u[c];
#pragma unroll
    for (int j = 0; j < 13; j++) x1[j] = x1[j] + BdtT[c][j] * uc;
  }
  if (xi6) {
    const float* xi = xi6 + (size_t)i * 6;
    float y[13], Ay[13], AAy[13];
#pragma unroll
    for (int j = 0; j < 13; j++) y[j] = (j >= 6 && j < 12) ? xi[j - 6] : 0.f;
    // A y: rows 0..2 = R^T y[6..8] (n1r = dt R^T), rows 3..5 = y[9..11], row 11 = x_drag y[9]
#pragma unroll
    for (int j = 0; j < 13; j++) Ay[j] = 0.f;
#pragma unroll
    for (int r = 0; r < 3; r++)
      Ay[r] = md.R[0 * 3 + r] * y[6] + md.R[1 * 3 + r] * y[7] + md.R[2 * 3 + r] * y[8];
    Ay[3] = y[9];
    Ay[4] = y[10];
    Ay[5] = y[11];
    Ay[11] = md.xdrag * y[9];
#pragma unroll
    for (int j = 0; j < 13; j++) AAy[j] = 0.f;
    AAy[5] = Ay[11];  // A (A y): rows 3..5 <- (A y)[9..11], rows 0..2 <- R^T (A y)[6..8] = 0
    const float dt2 = dt * dt * 0.5f, dt3 = dt * dt * dt / 6.f;
#pragma unroll
    for (int j = 0; j < 13; j++) x1[j] = x1[j] + (dt * y[j] + dt2 * Ay[j] + dt3 * AAy[j]);
  }
  float* s = loco + (size_t)i * CMPC_LOCO_WORDS;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    s[CMPC_LOCO_RPY + k] = x1[k];
    s[CMPC_LOCO_POS + k] = x1[3 + k];
    s[CMPC_LOCO_WW + k] = x1[6 + k];
    s[CMPC_LOCO_VW + k] = x1[9 + k];
  }
  s[CMPC_LOCO_ZGT] = x1[5];
  if (!(__float_as_uint(s[CMPC_LOCO_FLAGS]) & CMPC_LOCO_SIMFEET)) {
#pragma unroll
    for (int l = 0; l < 4; l++) {
      s[CMPC_LOCO_PFOOT + 3 * l + 0] += x1[3] - x0[3];
      s[CMPC_LOCO_PFOOT + 3 * l + 1] += x1[4] - x0[4];
    }
  }
  // ZYX Euler -> quaternion (w, x, y, z)
  const float cr = cosf(0.5f * x1[0]), sr = sinf(0.5f * x1[0]);
  const float cp = cosf(0.5f * x1[1]), sp = sinf(0.5f * x1[1]);
  const float cy = cosf(0.5f * x1[2]), sy = sinf(0.5f * x1[2]);
  s[CMPC_LOCO_Q + 0] = cr * cp * cy + sr * sp * sy;
  s[CMPC_LOCO_Q + 1] = sr * cp * cy - cr * sp * sy;
  s[CMPC_LOCO_Q + 2] = cr * sp * cy + sr * cp * sy;
  s[CMPC_LOCO_Q + 3] = cr * cp * sy - sr * sp * cy;
}

// Compact records -> solve records (include/cmpc_solver.h CMPC_CREC_*): the header as is, trajAll
// per updateMPCIfNeeded (ConvexMPCLocomotion.cpp:554-585) from its step-0 row — every step the
// step-0 row, except trajAll[12 k + 2/3/4] = trajAll[12 (k-1) + 2/3/4] + dtMPC x (yaw rate, v_x,
// v_y), fp32 product then fp32 sum as the caller computes them (this unit does not contract) —
// and the gait words as is. One thread per output word, so the stores coalesce; the <= 20-step
// recurrence is recomputed per word (the product is the same every step, so computing it once
// rounds identically).
__global__ __launch_bounds__(256) void cmpc_expand_kernel(const uint32_t* __restrict__ crec,
                                                          uint32_t* __restrict__ recs, int batch, int N,
                                                          int cw, int rw, float dt) {
  const long long gid = (long long)blockIdx.x * 256 + threadIdx.x;
  if (gid >= (long long)batch * rw) return;
  const int i = (int)(gid / rw), w = (int)(gid - (long long)i * rw);
  const uint32_t* c = crec + (size_t)i * cw;
  uint32_t v = 0u;
  if (w < CMPC_REC_HDR) {
    v = c[w];
  } else if (w < CMPC_REC_GAIT(N)) {
    const int k = (w - CMPC_REC_HDR) / 12, j = (w - CMPC_REC_HDR) % 12;
    v = c[CMPC_CREC_TRAJ0 + j];
    const int rate = (j == 2) ? 8 : (j == 3) ? 9 : (j == 4) ? 10 : -1;
    if (rate >= 0 && k > 0) {
      const float d = dt * __uint_as_float(c[CMPC_CREC_TRAJ0 + rate]);
      float x = __uint_as_float(v);
      for (int s = 1; s <= k; s++) x = x + d;
      v = __float_as_uint(x);
    }
  } else if (w < CMPC_REC_GAIT(N) + N) {
    v = c[CMPC_CREC_GAIT + (w - CMPC_REC_GAIT(N))];
  }
  recs[(size_t)i * rw + w] = v;
}

}  // namespace

hipError_t launch_assemble(float* d_loco, const LocoParams& lp, float* d_recs, uint8_t* d_due,
                           int batch, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_assemble_kernel, dim3((batch + 255) / 256), dim3(256), 0, stream, d_loco,
                     lp, d_recs, d_due, batch);
  return hipGetLastError();
}

hipError_t launch_rollout(float* d_loco, const float* d_recs, const float* d_forces,
                          const float* d_xi6, const uint8_t* d_due, const LocoParams& lp, float dt,
                          int batch, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_rollout_kernel, dim3((batch + 255) / 256), dim3(256), 0, stream, d_loco,
                     d_recs, d_forces, d_xi6, d_due, lp, dt, batch);
  return hipGetLastError();
}

hipError_t launch_expand(const float* d_compact, float* d_recs, int batch, int N, int rec_words, float dt,
                         hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  const long long words = (long long)batch * rec_words;
  hipLaunchKernelGGL(cmpc_expand_kernel, dim3((unsigned)((words + 255) / 256)), dim3(256), 0, stream,
                     reinterpret_cast<const uint32_t*>(d_compact), reinterpret_cast<uint32_t*>(d_recs), batch,
                     N, CMPC_CREC_WORDS(N), rec_words, dt);
  return hipGetLastError();
}

}  // namespace cmpc
