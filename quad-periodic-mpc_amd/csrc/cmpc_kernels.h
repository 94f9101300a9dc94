// cmpc_kernels.h — internal interface between the HIP kernels and the C-ABI host layer.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/cmpc_solver.h"

namespace cmpc {

// Launch-placement knobs of the A/B experiments: read from the environment only
// in a diagnostic build (-DCMPC_DIAG_KNOBS=1, scripts/build_diag_variant.sh); the product build
// always runs the measured defaults.
inline int diag_knob(const char* name, int dflt) {
#if defined(CMPC_DIAG_KNOBS) && CMPC_DIAG_KNOBS
  const char* v = getenv(name);
  return v ? atoi(v) : dflt;
#else
  (void)name;
  return dflt;
#endif
}

// Kernel-side copy of cmpc_params (by value, lands in SGPRs).
struct KParams {
  float dt;
  float mu_inv;    // fmat uses 1/mu (SolverMPC.cpp:657)
  float f_max;
  float alpha2;    // 2 * alpha (qH = 2 (B'SB + alpha I))
  float wts[12];
  int N;
  int rec_words;
  int max_iter;    // active-set cap; the kernels allow max_iter + 2 n
  int refine;      // wide classes: one fp64 refinement step of the converged active set (N > 10)
  int out_cols;    // forces written per instance: 12 x the leading horizon steps kept
                   // (cmpc_batch_set_output_steps; 12 N by default)
  // the step's fp64 powers for that refinement (scalar registers, not per-lane conversions)
  double dt64, dth64, dt3_64;  // dt, dt^2 / 2, dt^3 / 6
};

// Kernel-side copy of cmpc_loco_params + the handle's horizon / record stride.
struct LocoParams {
  float dt;
  int iters_between_mpc;
  float x_drag_gain;
  int horizon;
  int rec_words;
  float hip_x, hip_y, abad_link, swing_height, bonus_swing;  // foot placement (cmpc_loco_params)
  int out_cols;    // rollout: the forces' stride (the handle's KParams::out_cols)
};

// Scratch ints needed by launch_solve for max_batch instances.
// d_work: [0] instances above class 1's build, [1 + list] lengths of the class lists, then the
// lists of max_batch entries each. Instance lists of the classify pass: 80, 96, 128, 192, 256,
// 5: class 1's own instances from N = 11 (n <= its row width; up to N = 10 it runs over the whole
// batch), 144, and 7: class-1 instances with 60 < n <= 64 (the 64-wide class-1 build beside the
// 60-wide one); 8: the 120-column wide build (97 <= n <= 120; the 128 build keeps 121..128).
// 9: the tail class (cmpc_tail.hip, N <= 10: 64 < n <= 72, one wavefront each); 10: the instances
// it hands to the 80-column wide class (an active set past 64 positions).
// d_work = [2 headers of kHdr ints: cnt[0] total, cnt[1 + list] list lengths, cnt[kDeq + list] the
// persistent wide workgroups' dequeue counters] [kLists lists of max_batch]. The solves alternate
// over the two headers: each classify pass zeroes the header the next solve uses (the previous
// solve, which used it, has joined by then), so no memset precedes a solve (zeroed at create)
constexpr int kLists = 11;
constexpr int kHdr = 32;
constexpr int kDeq = 16;  // cnt[kDeq + list]: dequeue counter of a persistent class's workgroups
constexpr int kHdrBatch = 31;  // cnt[kHdrBatch]: the batch of the solve that counted into the header
static_assert(1 + kLists <= kDeq && kDeq + kLists <= kHdrBatch && kHdrBatch < kHdr,
              "list lengths, dequeue counters and the batch tag fit the header");
inline size_t work_ints(int max_batch) { return 2 * kHdr + kLists * (size_t)max_batch; }
// Side streams and events of one handle: the wider size classes run concurrently with class 1
// (they are latency-bound: few instances, long serial solves). Three side streams (the third
// carries only the tail class at N <= 10 below 131072 instances): with the handle's own stream
// that is the four hardware queues a process gets by default (GPU_MAX_HW_QUEUES = 4), so no side
// stream shares a queue with class 1. A process with two handles (parallel.RootPipeline's two
// solver lanes) has eight streams over those four queues: the lanes' streams alias in pairs; the
// lanes alternate pieces, so at most one lane's class 1 runs at a time.
constexpr int kSideStreams = 3;
struct LaunchCtx {
  hipStream_t side[kSideStreams] = {nullptr, nullptr, nullptr};
  hipEvent_t fork = nullptr;
  hipEvent_t classified = nullptr;  // the classify pass (on side 0) is done
  hipEvent_t join[kSideStreams] = {nullptr, nullptr, nullptr};
  int hdr = 0;       // header (0 / 1) of d_work the next solve's lists count into
  // class counts of an earlier solve (a header as the classify kernel left it, copied by a later
  // classify pass): host-mapped pinned memory, read by launch_solve to size the wide classes' grids
  int* h_hint = nullptr;
  int* d_hint = nullptr;
  int last_hdr = 0;  // header of the last solve (its cnt[0] for cmpc_batch_read_timing)
};
// ev (optional): 3 events recorded on `stream`: ev[0] before class 1, ev[1] after it, ev[2]
// after the wider classes (side streams) have joined.
hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        hipStream_t stream, LaunchCtx& ctx, hipEvent_t* ev = nullptr);
// per-class launchers (cmpc_class1.hip, cmpc_wide_w*.hip)
hipError_t launch_class1(int nv, const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         int* ovf_list, int* ovf_count, int grid, hipStream_t stream);
// wide classes, two lanes per row, NV/32 wavefronts (cmpc_wide_w{80,96,120,128,144,192,256}.hip)
#define CMPC_DECL_WIDE(W)                                                                          \
  hipError_t launch_wide_w##W(const float* d_recs, const KParams& P, float* d_forces,             \
                              uint8_t* d_status, int32_t* d_iters, const int* in_list,            \
                              const int* in_count, int* deq, int grid, hipStream_t stream,     \
                              int base = 0);
CMPC_DECL_WIDE(80)
CMPC_DECL_WIDE(96)
CMPC_DECL_WIDE(120)
CMPC_DECL_WIDE(128)
CMPC_DECL_WIDE(80_persist)
CMPC_DECL_WIDE(96_persist)
CMPC_DECL_WIDE(120_persist)
CMPC_DECL_WIDE(128_persist)
CMPC_DECL_WIDE(144)
CMPC_DECL_WIDE(192)
CMPC_DECL_WIDE(256)
#undef CMPC_DECL_WIDE
// the tail class (cmpc_tail.hip): 8 tail rows beside class 1's 64 (n <= 72), one wavefront per
// instance over its list, one workgroup per possible entry; an instance whose active set outgrows
// 64 positions is appended to ovf_list (batched) or, with ovf_list == nullptr, gets status
// kHandoffStatus (single-instance path: the host re-launches it in the wide class,
// launch_single(..., allow_tail = false))
constexpr uint8_t kHandoffStatus = 0xFE;
// rest_grid > 0: `grid` covers the first entries only (a predicted count), and a looping kernel of
// rest_grid workgroups follows on the stream for any entries past it
hipError_t launch_tail(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                       int32_t* d_iters, const int* in_list, const int* in_count, int* ovf_list,
                       int* ovf_count, int grid, hipStream_t stream, int rest_grid = 0);
// the reduced sizes the tail class takes from the 80-column wide class: 64 < n <= 72 at N <= 10
// (the horizons without the fp64 refinement of the wide classes; with the refinement switched
// off, cmpc_batch_set_refine(0), the longer horizons keep the 80-column class, whose parity the
// refine-off tests cover)
__host__ __device__ inline bool tail_class(const KParams& P, int n) {
  return !P.refine && P.N <= 10 && n > 64 && n <= 72;
}
// the tail class in its self-classifying form (no classify list): grid workgroups scan the batch
// in chunks of `chunk` instances and solve its tail-class instances, launched ahead of class 1
hipError_t launch_tail_self(const float* d_recs, int batch, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, int* ovf_list, int* ovf_count, int grid, int chunk,
                            hipStream_t stream);
hipError_t launch_single(const float* d_rec, int n, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* d_one, hipStream_t stream,
                         bool allow_tail = true);
// config 5 estimator (cmpc_estimator.hip). d_gauss: the two normalised float Gaussian kernels
// of gaussian_filter (sigma 7: 43 taps, then sigma 27: 163 taps), built on the host exactly as
// SolverMPC.cpp:404-418 builds them.
constexpr int kGaussR7 = 21;   // ceil(3 * 7)
constexpr int kGaussR27 = 81;  // ceil(3 * 27)
constexpr int kGaussTaps = 2 * kGaussR7 + 1 + 2 * kGaussR27 + 1;
// d_fest_out (optional): f_est(3) of instance i also to d_fest_out[i] (the single-instance ABI
// reads it back with the forces)
hipError_t launch_estimate(float* d_est, const float* d_logs, const float* d_fext3,
                           const float* d_time, float sim_time, float* d_records, int rec_words,
                           float* d_fext6, const float* d_gauss, int batch, hipStream_t stream,
                           float* d_fest_out = nullptr);
// batched input assembly (cmpc_assemble.hip): one control tick per instance
hipError_t launch_assemble(float* d_loco, const LocoParams& lp, float* d_recs, uint8_t* d_due,
                           int batch, hipStream_t stream);
// compact records (CMPC_CREC_*) -> solve records, trajAll expanded per ConvexMPCLocomotion.cpp:554-585
hipError_t launch_expand(const float* d_compact, float* d_recs, int batch, int N, int rec_words, float dt,
                         hipStream_t stream);
// single-rigid-body step of every due instance with its solved step-0 forces (cmpc_assemble.hip)
hipError_t launch_rollout(float* d_loco, const float* d_recs, const float* d_forces,
                          const float* d_xi6, const uint8_t* d_due, const LocoParams& lp, float dt,
                          int batch, hipStream_t stream);
// parity hook and JCQP condensation: full (nothing eliminated) qH [12N x 12N] / qg [12N] per
// instance (cmpc_condense.hip)
hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           hipStream_t stream);

// use_jcqp == 1 / 2: batched JCQP ADMM over the full / reduced condensed QP (cmpc_admm.hip).
// Instances whose QP has n > 120 variables run on nslabs persistent workgroups with M in
// d_slabs (nslabs * admm_slab_doubles(N) doubles); may be NULL when no such instance can occur.
size_t admm_slab_doubles(int horizon);
constexpr int kAdmmSlabs = 512;
hipError_t launch_admm(const float* d_recs, const float* d_H, const float* d_g, int batch,
                       const KParams& P, const cmpc_admm_settings& s, float* d_forces,
                       uint8_t* d_status, int32_t* d_iters, double* d_slabs, int nslabs,
                       hipStream_t stream);

}  // namespace cmpc
