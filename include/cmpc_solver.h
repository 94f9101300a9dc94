/*
 * cmpc_solver.h — C ABI of the MI355X-native batched convex-MPC solver (libcmpc_hip.so).
 *
 * Two surfaces live here:
 *
 *  1. The reference's single-instance SolverMPC interface, unchanged, so the be2r_cmpc_unitree
 *     FSM links against this library instead of SolverMPC.cpp + convexMPC_interface.cpp +
 *     RobotState.cpp (reference: be2r_cmpc_unitree/src/controllers/convexMPC/convexMPC_interface.h:44-52).
 *     Same names, same argument meaning, same call protocol
 *       setup_problem -> update_x_drag -> update_solver_settings -> update_problem_data_floats
 *       -> get_solution(0..11)
 *     (ConvexMPCLocomotion.cpp:807-836). The solve runs on the GPU through the batched path with
 *     batch = 1.
 *
 *  2. A new reentrant batched API (cmpc_batch_*): one handle per stream, a batch of independent
 *     MPC instances packed as fixed-stride fp32 records (layout below), forces + status out.
 *
 * No torch types cross this boundary: plain pointers and sizes only.
 */
#ifndef CMPC_SOLVER_H
#define CMPC_SOLVER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
#define CMPC_EXTERNC extern "C"
#else
#define CMPC_EXTERNC
#endif

/* ------------------------------------------------------------------------------------------ */
/* Instance record layout (fp32 words).                                                       */
/* One record = one solve_mpc() call's per-instance data (SolverMPC.cpp:566-655).             */
/* ------------------------------------------------------------------------------------------ */
#define CMPC_REC_P        0   /* p[3]      body position (world)          update_data_t.p      */
#define CMPC_REC_V        3   /* v[3]      body velocity (world)          update_data_t.v      */
#define CMPC_REC_Q        6   /* q[4]      orientation quaternion w,x,y,z update_data_t.q      */
#define CMPC_REC_W        10  /* w[3]      angular velocity (world)       update_data_t.w      */
#define CMPC_REC_R        13  /* r[12]     foot offsets, axis-major 3x4:  r[axis*4 + leg]      */
#define CMPC_REC_RPY      25  /* roll, pitch, yaw (stored, unused by the solve, as reference)  */
#define CMPC_REC_XDRAG    28  /* x_drag    A(11,9) coefficient            update_x_drag()      */
#define CMPC_REC_FEST3    29  /* f_est(3): compensation force fed into qg (config 5)           */
#define CMPC_REC_FLAGS    30  /* bit-cast uint32: bit0 = use f_est in qg (history > 500)       */
#define CMPC_REC_HDR      32  /* header words; traj follows                                    */
/* traj[12*N] fp32 at CMPC_REC_HDR, then gait[4*N] uint8 (step-major, leg-minor) packed into
 * N words, then padding to a 16-byte multiple. */
#define CMPC_REC_TRAJ(N)   (CMPC_REC_HDR)
#define CMPC_REC_GAIT(N)   (CMPC_REC_HDR + 12 * (N))
#define CMPC_REC_WORDS(N)  ((CMPC_REC_HDR + 13 * (N) + 3) & ~3)

/* Compact record (cmpc_batch_expand): what the caller computes trajAll from
 * (ConvexMPCLocomotion.cpp:554-585) instead of trajAll itself — the header as above, trajAll's
 * step-0 row (12 words: trajInitial with [2] = the measured yaw), the gait words, padding to a
 * 16-byte multiple. 56 words (224 B) at N = 10 against 164 (656 B): what a root GPU sends each
 * peer per instance in the config-4 sharding (parallel.RootPipeline record_format="compact"). */
#define CMPC_CREC_TRAJ0    (CMPC_REC_HDR)
#define CMPC_CREC_GAIT     (CMPC_REC_HDR + 12)
#define CMPC_CREC_WORDS(N) ((CMPC_REC_HDR + 12 + (N) + 3) & ~3)

#define CMPC_MAX_HORIZON  20  /* reference caps at 19 (SolverMPC.cpp:113-116); lifted to 20 for config 5;
                                 longer horizons are rejected (cmpc_batch_create / set_params -2) */

/* ------------------------------------------------------------------------------------------ */
/* Config 5: periodic-disturbance estimation (fp32 words).                                    */
/* LogData record: the previous step's logged state, forces and model, as the caller receives */
/* it from /log_data (unitree_legged_msgs/msg/LogData.msg; read at                            */
/* ConvexMPCLocomotion.cpp:639-771). geometry_msgs doubles are stored as fp32, the precision */
/* the reference casts them to.                                                               */
/* ------------------------------------------------------------------------------------------ */
#define CMPC_LOG_POS      0   /* pos_act x,y,z                                                  */
#define CMPC_LOG_EUL      3   /* euler_act x,y,z (roll, pitch, yaw)                             */
#define CMPC_LOG_ANG      6   /* vel_act.angular x,y,z                                          */
#define CMPC_LOG_LIN      9   /* vel_act.linear x,y,z                                           */
#define CMPC_LOG_FORCE    12  /* foot_force{0..3}_{x,y,z}, leg-major                            */
#define CMPC_LOG_XDRAG    24  /* x_drag                                                         */
#define CMPC_LOG_R        25  /* r_{x,y,z}_{1..4}, axis-major 3x4                               */
#define CMPC_LOG_ROT      37  /* R_00 .. R_22, row-major                                        */
#define CMPC_LOG_WORDS    48
/* Estimator state of one instance: the reference's globals time_history / diff_history /
 * est_* / f_est (SolverMPC.cpp:390-398, 555-563), with the unbounded histories replaced by a
 * ring of the last CMPC_EST_WINDOW samples (only that window is ever read). */
#define CMPC_EST_WINDOW   400 /* window_size (SolverMPC.cpp:704)                                */
#define CMPC_EST_STOP     500 /* re-estimation stops above this count (SolverMPC.cpp:707)       */
#define CMPC_EST_F        0   /* f_ext[3] samples, ring [400]                                   */
#define CMPC_EST_T        400 /* simulation_time samples, ring [400]                            */
#define CMPC_EST_COUNT    800 /* int32: samples pushed so far (= time_history.size(), capped)   */
#define CMPC_EST_HEAD     801 /* int32: ring slot of the next sample (= the oldest one)         */
#define CMPC_EST_FEST3    802 /* f_est(3), the compensation force                               */
#define CMPC_EST_PARAMS   804 /* double[4]: est_stat, est_amp, est_freq, est_phase              */
#define CMPC_EST_WORDS    816

/* ------------------------------------------------------------------------------------------ */
/* Batched input assembly: locomotion-controller state (fp32 words).  */
/* The inputs and persistent state of ConvexMPCLocomotion::run's MPC side                     */
/* (ConvexMPCLocomotion.cpp:100-123, 204-257, 334-339, 511-586, 612-633, 786-818).            */
/* Words marked "state" are read and written back by cmpc_batch_assemble; int32 words are     */
/* bit-cast into the fp32 array.                                                               */
/* ------------------------------------------------------------------------------------------ */
#define CMPC_LOCO_POS      0   /* seResult.position[3]                                         */
#define CMPC_LOCO_ZGT      3   /* ground_truth_position[2]: p[2] of the solve (:628)           */
#define CMPC_LOCO_Q        4   /* seResult.orientation (w,x,y,z)                               */
#define CMPC_LOCO_RPY      8   /* seResult.rpy[3]                                              */
#define CMPC_LOCO_VW       11  /* seResult.vWorld[3]                                           */
#define CMPC_LOCO_WW       14  /* seResult.omegaWorld[3]                                       */
#define CMPC_LOCO_PFOOT    17  /* pFoot[4][3], world frame, leg-major (:234)                   */
#define CMPC_LOCO_CMD      29  /* x_vel_cmd, y_vel_cmd, _yaw_turn_rate (scaled sticks, :108-114)*/
#define CMPC_LOCO_HEIGHT   32  /* _body_height                                                 */
#define CMPC_LOCO_VDES     33  /* state: filtered _x_vel_des, _y_vel_des (:116-117)            */
#define CMPC_LOCO_WPD      35  /* state: world_position_desired x, y (:239, :537-552)          */
#define CMPC_LOCO_RPYINT   37  /* state: rpy_int[0], rpy_int[1] (:218-228)                     */
#define CMPC_LOCO_XCI      39  /* state: x_comp_integral (:809-818)                            */
#define CMPC_LOCO_COUNTER  40  /* state, int32: iterationCounter                               */
#define CMPC_LOCO_GAIT     41  /* int32: OffsetDurationGait P, offsets[4], durations[4]        */
#define CMPC_LOCO_FLAGS    50  /* state, uint32: CMPC_LOCO_OMNI | STANDING | PRONK | FIRST     */
#define CMPC_LOCO_STAND    51  /* stand_traj x, y, yaw (:146-151; stand_traj[0], [1], [5])     */
/* foot placement and swing (:276-331, :350-402; FootSwingTrajectory.cpp:17-42)                  */
#define CMPC_LOCO_SWREM    56  /* state: swingTimeRemaining[4] (:287-296)                       */
#define CMPC_LOCO_SWST     60  /* out: gait->getSwingState() of the tick (Gait.cpp:102-135)      */
#define CMPC_LOCO_P0       64  /* state: footSwingTrajectories[l]._p0 [4][3] (:262, :378)       */
#define CMPC_LOCO_PF       76  /* state: footSwingTrajectories[l]._pf [4][3], the foothold Pf   */
#define CMPC_LOCO_PDES     88  /* state: footSwingTrajectories[l]._p [4][3] = pDesFootWorld     */
#define CMPC_LOCO_WORDS    104
#define CMPC_LOCO_OMNI     1u  /* omniMode: v_des is already in the world frame (:211)         */
#define CMPC_LOCO_STANDING 2u  /* current_gait == 4: stand trajectory (:527-533)               */
#define CMPC_LOCO_PRONK    4u  /* gaitNumber == 8 (pacing): roll compensation off (:230)      */
#define CMPC_LOCO_FIRST    8u  /* firstRun: world_position_desired = position (:249-256)       */
#define CMPC_LOCO_SIMFEET  16u /* simulator feet (not in the reference): after each tick a     */
                               /* swinging foot is at its pDesFootWorld, a foot entering stance */
                               /* touches down (z = 0) and stance feet stay fixed in the world; */
                               /* cmpc_batch_rollout then leaves the feet alone                 */
#define CMPC_LOCO_FSWING0  256u/* firstSwing[l] is bit (8 + l) (:75, :289, :376, :413)          */

/* Batch-shared controller constants. */
typedef struct cmpc_loco_params {
  float dt;               /* control tick (s); dtMPC = dt * iters_between_mpc                   */
  int   iters_between_mpc;/* _iterationsBetweenMPC                                             */
  float x_drag_gain;      /* _dyn_params->cmpc_x_drag                                          */
  int   pad;
  float hip_x, hip_y;     /* quadruped._abadLocation x, y: getHipLocation(l) = (+-x, +-y, 0)    */
                          /* (Quadruped.h:95-102; A1: 0.1805, 0.047, MiniCheetah.h:30-31)       */
  float abad_link;        /* quadruped._abadLinkLength (A1: 0.0838)                             */
  float swing_height;     /* _dyn_params->Swing_traj_height (ros_config.yaml:62: 0.17)          */
  float bonus_swing;      /* _dyn_params->cmpc_bonus_swing (ros_config.yaml:70: 0)              */
  float pad2[3];
} cmpc_loco_params;

/* Per-instance status (batched API). The reference has no status: on qpOASES failure it prints
 * "failed to solve!" and leaves stale forces (SolverMPC.cpp:964-968). Documented deviation:
 * forces are zero when status != CMPC_OK. */
enum {
  CMPC_OK = 0,
  CMPC_MAX_ITER = 1,      /* active-set iteration cap (reference nWSR = 100) reached          */
  CMPC_INFEASIBLE = 2,    /* friction-pyramid QP infeasible                                    */
  CMPC_NOT_PD = 3,        /* Hessian factorisation failed                                      */
  CMPC_BAD_INPUT = 4      /* horizon out of range / non-finite input                           */
};

/* Batch-shared problem parameters (problem_setup + the update_data_t scalars that the caller
 * keeps constant across instances: ConvexMPCLocomotion.cpp:617,623,807). */
typedef struct cmpc_params {
  float dt;           /* dtMPC (s)                                                              */
  float mu;           /* friction coefficient; fmat uses 1/mu (SolverMPC.cpp:657-660)           */
  float f_max;        /* ub(fz) = gait * f_max                                                  */
  int   horizon;      /* N, 1..CMPC_MAX_HORIZON                                                 */
  float weights[12];  /* diagonal state weights (13th = 0)                                      */
  float alpha;        /* force regularisation: qH = 2(B'SB + alpha I)                          */
  int   max_iter;     /* active-set iteration cap (reference: nWSR = 100)                       */
} cmpc_params;

typedef struct cmpc_batch cmpc_batch;

/* ------------------------------------------------------------------------------------------ */
/* 1. Reference single-instance interface (convexMPC_interface.h:44-52)                       */
/* ------------------------------------------------------------------------------------------ */
/* Replaces convexMPC_interface.cpp:44-67 (+ resize_qp_mats, SolverMPC.cpp:149-250). */
CMPC_EXTERNC void setup_problem(double dt, int horizon, double mu, double f_max);
/* Replaces convexMPC_interface.cpp:96-107 (double-precision variant, yaw only). */
CMPC_EXTERNC void update_problem_data(double* p, double* v, double* q, double* w, double* r,
                                      double yaw, double* weights, double* state_trajectory,
                                      double alpha, int* gait);
/* Replaces convexMPC_interface.cpp:156-162: q_soln[index], 0 before the first solve. */
CMPC_EXTERNC double get_solution(int index);
/* Replaces convexMPC_interface.cpp:109-130 (use_jcqp thresholds >1.5 -> 2, >0.5 -> 1). */
CMPC_EXTERNC void update_solver_settings(int max_iter, double rho, double sigma,
                                         double solver_alpha, double terminate, double use_jcqp);
/* Replaces convexMPC_interface.cpp:132-149 -> solve_mpc (SolverMPC.cpp:566-1089). */
CMPC_EXTERNC void update_problem_data_floats(float* p, float* v, float* q, float* w, float* r,
                                             float roll, float pitch, float yaw, float* weights,
                                             float* state_trajectory, float alpha, int* gait);
#ifdef __cplusplus
/* C++ linkage, as the reference (convexMPC_interface.h:52; symbol _Z13update_x_dragf). */
void update_x_drag(float x_drag);
#endif

/* Globals the reference solver reads but its caller defines (ConvexMPCLocomotion.cpp:610,
 * be2r_cmpc_unitree_node.cpp:6). Weak definitions in the library; the host program's strong
 * definitions take precedence. f_ext has Eigen::Matrix<float,6,1> layout (6 floats). */
CMPC_EXTERNC float f_ext[6];
CMPC_EXTERNC float simulation_time;
/* The solver's own estimator globals (SolverMPC.h:72-74, SolverMPC.cpp:390-392, 772-798):
 * f_est(3) = the compensation force of the last update_problem_data* call (fed into qg once more
 * than 500 samples were pushed), f_est_smoothed = 0.95 f_est_smoothed + 0.05 f_est, and
 * f_est_static(3) = 0.97 f_est_static(3) + 0.03 f_ext(3). Eigen::Matrix<float,6,1> layout. The
 * estimator step itself runs on the device (the kernel of cmpc_batch_estimate, one instance). */
CMPC_EXTERNC float f_est[6];
CMPC_EXTERNC float f_est_smoothed[6];
CMPC_EXTERNC float f_est_static[6];

/* ------------------------------------------------------------------------------------------ */
/* 2. Batched, reentrant API                                                                   */
/* ------------------------------------------------------------------------------------------ */
CMPC_EXTERNC int cmpc_record_words(int horizon);
/* Create a handle bound to the current HIP device; stream may be NULL (a private stream is
 * created). Scratch for max_batch instances is allocated here, never inside solve. */
CMPC_EXTERNC int cmpc_batch_create(cmpc_batch** out, const cmpc_params* prm, int max_batch,
                                   void* hip_stream);
CMPC_EXTERNC int cmpc_batch_set_params(cmpc_batch* h, const cmpc_params* prm);
CMPC_EXTERNC void cmpc_batch_destroy(cmpc_batch* h);
/* Device-resident solve: d_records [batch * cmpc_record_words(N)] fp32, d_forces
 * [batch * 12N] fp32 (step-major, leg*3+axis), d_status [batch] uint8, d_iters [batch] int32
 * (may be NULL). Asynchronous on the handle's stream. Returns 0 or a negative error. */
CMPC_EXTERNC int cmpc_batch_solve(cmpc_batch* h, const float* d_records, int batch,
                                  float* d_forces, uint8_t* d_status, int32_t* d_iters);
/* Forces kept per instance: the first `steps` horizon steps (12 x steps floats per instance,
 * stride of d_forces / forces of the two solves below and of cmpc_batch_rollout), 0 = every step
 * (12N, the default). A caller that reads only get_solution(0..11) as ConvexMPCLocomotion.cpp:
 * 832-845 does can keep step 0 (48 B instead of 480 B per instance at N = 10). New API. */
CMPC_EXTERNC int cmpc_batch_set_output_steps(cmpc_batch* h, int steps);
/* The fp64 refinement of the converged working set in the wide size classes:
 * 1 (default) from N = 11, 0 off (every horizon solved in fp32 only, as the reference's own fp32
 * condensation: ~11 % faster at N = 16, but at N >= 16 a few all-stance instances then miss
 * qpOASES by more than 1e-4). New API. */
CMPC_EXTERNC int cmpc_batch_set_refine(cmpc_batch* h, int on);
/* Compact records (CMPC_CREC_*) -> solve records for the handle's horizon: trajAll[12 k + j] =
 * the step-0 row, except j = 2, 3, 4 (yaw, x, y) = the previous step's + dtMPC x (yaw rate, v_x,
 * v_y) of the step-0 row, in fp32 as updateMPCIfNeeded computes it (ConvexMPCLocomotion.cpp:
 * 554-585, dtMPC = the handle's dt). Bit for bit the records a caller builds itself. d_compact
 * [batch * CMPC_CREC_WORDS(N)], d_records [batch * cmpc_record_words(N)]. Asynchronous on the
 * handle's stream. New API. */
CMPC_EXTERNC int cmpc_batch_expand(cmpc_batch* h, const float* d_compact, float* d_records, int batch);
/* Same, host buffers in and out (H2D + solve + D2H on the handle's stream, synchronous). */
CMPC_EXTERNC int cmpc_batch_solve_host(cmpc_batch* h, const float* records, int batch,
                                       float* forces, uint8_t* status, int32_t* iters);
/* Parity hook for the condensation rows (SolverMPC.cpp:96-146, 806-814): full 12N x 12N qH
 * (row-major) and qg per instance, all variables kept (no swing elimination). */
CMPC_EXTERNC int cmpc_batch_condense(cmpc_batch* h, const float* d_records, int batch,
                                     float* d_H, float* d_g);
/* JCQP ADMM settings: update_solver_settings(max_iter, rho, sigma, solver_alpha, terminate, .)
 * (convexMPC_interface.cpp:109-129 -> QpProblemSettings, JCQP/QpProblem.h:15-28). */
typedef struct cmpc_admm_settings {
  int    max_iter;    /* maxIterations (ros_config.yaml jcqp_max_iter: 10000)                   */
  double rho;         /* jcqp_rho 1e-7                                                           */
  double sigma;       /* jcqp_sigma 1e-8                                                         */
  double alpha;       /* over-relaxation, jcqp_alpha 1.5                                         */
  double terminate;   /* (|Ax - z|_inf + |Px + q + A'y|_inf) / 4 threshold, jcqp_terminate 0.1  */
  int    reduced;     /* 0: use_jcqp == 1 (full QP); 1: use_jcqp == 2 (swing legs eliminated)    */
} cmpc_admm_settings;
/* use_jcqp == 1 (SolverMPC.cpp:818-838, 1057-1062): the full QP (P = qH, q = qg from
 * cmpc_batch_condense, A = fmat, l = 0, u = U_b) solved by JCQP's ADMM in fp64, one workgroup
 * per instance, any horizon. With s->reduced (use_jcqp == 2, SolverMPC.cpp:984-1053) the swing
 * legs are eliminated first. QPs of up to 120 variables keep the inverted KKT Schur complement in
 * LDS; larger ones (N > 10) in per-workgroup fp64 global slabs (min(max_batch, 512) x (12N)^2
 * doubles: 151 MB at N = 16, 236 MB at N = 20), allocated by the handle's FIRST cmpc_batch_admm
 * call and kept from then on (handles that never run ADMM never pay for them): make that first
 * call outside stream capture, and expect an allocation failure to surface there. d_forces
 * [batch * out_cols] = the solution as float (0 for eliminated variables), the leading steps the
 * handle keeps (cmpc_batch_set_output_steps; 12N by default), so cmpc_batch_rollout reads ADMM
 * forces with the same stride as the active-set solve's; d_status 0 = residual
 * below terminate, 1 = max_iter reached; d_iters (may be NULL). */
CMPC_EXTERNC int cmpc_batch_admm(cmpc_batch* h, const float* d_records, const float* d_H,
                                 const float* d_g, int batch, const cmpc_admm_settings* s,
                                 float* d_forces, uint8_t* d_status, int32_t* d_iters);
/* Config 5, one estimator step for every instance (SolverMPC.cpp:688-811 per instance, the
 * residual of ConvexMPCLocomotion.cpp:639-771 first when d_logs is given):
 *   f_ext  = residual(d_logs[i], d_records[i])          if d_logs  (written to d_fext6 if set)
 *            (0, 0, 0, d_fext3[i], 0, 0)                 otherwise
 *   push (f_ext[3], t_i) into d_est[i], t_i = d_time ? d_time[i] : sim_time;
 *   400 <= count <= 500: band-pass (Gaussian sigma 7 minus sigma 27), DFT peak, sine fit;
 *   count >= 400: f_est(3) = est_amp + sin(2 pi t_i est_freq + est_phase);
 *   d_records[i]: CMPC_REC_FEST3 = f_est(3), CMPC_REC_FLAGS bit 0 = (count > 500).
 * d_est: batch * CMPC_EST_WORDS words, zero-initialised by the caller before the first step.
 * Asynchronous on the handle's stream; run it before cmpc_batch_solve on the same records. */
CMPC_EXTERNC int cmpc_batch_estimate(cmpc_batch* h, float* d_est, const float* d_logs,
                                     const float* d_fext3, const float* d_time, float sim_time,
                                     float* d_records, float* d_fext6, int batch);
/* One control tick of every instance's locomotion controller (batched
 * ConvexMPCLocomotion::run MPC side): updates the state words of d_loco [batch *
 * CMPC_LOCO_WORDS]; where an MPC step is due (iterationCounter % iters_between_mpc == 0 after
 * the increment) writes the instance's solve record d_records[i] (the arguments the reference
 * passes to update_problem_data_floats: p, v, q, w, r, rpy, trajAll, gait table, x_drag) and
 * d_due[i] = 1, else leaves the record and sets d_due[i] = 0. Gait rows i < N use
 * (i + _iteration + 1) mod P, i.e. the table repeats for N > P where the reference would read
 * past its P-row table. Asynchronous on the handle's stream. */
CMPC_EXTERNC int cmpc_batch_assemble(cmpc_batch* h, float* d_loco, const cmpc_loco_params* lp,
                                     float* d_records, uint8_t* d_due, int batch);
/* Closes the loop of a batched MPC simulator: for every instance with d_due[i] != 0 (all when
 * d_due is NULL), advances the single-rigid-body state of its record by one MPC step with its
 * own prediction model and the step-0 forces of the solve (d_forces[i][0..11]), plus an
 * optional disturbance d_xi6[i] = [tau(3), f(3)] through Qdt (Q_ct of SolverMPC.cpp:607-615):
 *   x+ = Adt x0 + Bdt u0 + Qdt xi   (the discretisation of c2qp, SolverMPC.cpp:96-146)
 * and writes rpy / p / w / v (+ the quaternion, z_groundtruth = p_z) into d_loco[i]; the feet
 * move with the body in x, y (footstep relocation is not simulated). The step is the handle's
 * dt (dtMPC). Asynchronous on the handle's stream. */
CMPC_EXTERNC int cmpc_batch_rollout(cmpc_batch* h, float* d_loco, const float* d_records,
                                    const float* d_forces, const float* d_xi6,
                                    const uint8_t* d_due, int batch);
/* Measurement hooks: record HIP events on the handle's stream around the next `steps` solves;
 * read back per-solve ms pairs [class 1's launch, the time after it until the wide size classes
 * have joined] and the number of instances the last solve listed for the wide classes
 * (n > 64). Synchronises. */
CMPC_EXTERNC int cmpc_batch_enable_timing(cmpc_batch* h, int steps);
/* The same on every `every`-th solve only (the first of each group of `every`), `steps` of them:
 * a timed loop then pays the event packets on a fraction of its solves. */
CMPC_EXTERNC int cmpc_batch_enable_timing_every(cmpc_batch* h, int steps, int every);
CMPC_EXTERNC int cmpc_batch_read_timing(cmpc_batch* h, float* ms, int* steps_recorded,
                                        int* class1_overflow);
/* Stream the handle runs on (hipStream_t). */
CMPC_EXTERNC void* cmpc_batch_stream(cmpc_batch* h);
/* Last HIP error string for this thread (diagnostics). */
CMPC_EXTERNC const char* cmpc_last_error(void);

#endif /* CMPC_SOLVER_H */
