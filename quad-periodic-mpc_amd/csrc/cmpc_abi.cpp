// cmpc_abi.cpp — the C ABI of libcmpc_hip.so (declared in include/cmpc_solver.h).
//
//  * cmpc_batch_*: reentrant batched API, one handle per HIP stream, device scratch allocated
//    at create time (never inside solve, so a caller may capture solve into a hipGraph).
//  * setup_problem / update_problem_data(_floats) / update_solver_settings / update_x_drag /
//    get_solution: the reference's single-instance interface (convexMPC_interface.h:44-52) with
//    the same call protocol and semantics, implemented over a batch-1 handle.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <mutex>
#include <utility>
#include <string>
#include <vector>

#include "../../include/cmpc_solver.h"
#include "cmpc_kernels.h"

namespace {
thread_local std::string g_last_error;

int fail(const char* what, hipError_t e) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return -(int)e - 1000;
}
}  // namespace

struct cmpc_batch {
  cmpc_params prm;
  cmpc::KParams kp;
  int out_steps = 0;             // cmpc_batch_set_output_steps (0: every step)
  int refine = 1;                // cmpc_batch_set_refine (1: from N = 11, 0: off)
  int max_batch = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  int* d_work = nullptr;
  float* d_gauss = nullptr;      // gaussian_filter kernels of the config-5 estimator
  double* d_admm_slabs = nullptr;  // ADMM inverses of QPs with n > 120 (cmpc_admm.hip)
  size_t admm_slab_doubles = 0;
  int admm_nslabs = 0;
  bool admm_used = false;        // slabs are allocated on the first ADMM call, not at create
  bool staged = false;           // every allocation of ensure_staging succeeded
  float* d_admm_H = nullptr;     // condensed qH / qg staging of the single-instance ADMM path
  // staging for the host-pointer entry point (allocated lazily, sized max_batch)
  float* d_rec = nullptr;
  float* d_forces = nullptr;
  uint8_t* d_status = nullptr;
  int32_t* d_iters = nullptr;
  // single-instance fast path of cmpc_batch_solve_host: the one-entry instance list {1, 0}, the
  // instance's forces + status word (one D2H), pinned host staging of record and result
  int* d_one = nullptr;
  float* d_single_out = nullptr;
  float* h_pin = nullptr;
  // side streams + fork/join events for the wider size classes (cmpc_launch.hip)
  cmpc::LaunchCtx ctx;
  bool pooled_sides = false;     // ctx.side came from the process-wide pool (acquire_sides)
  // optional per-launch timing (cmpc_batch_enable_timing)
  std::vector<hipEvent_t> ev;
  int ev_steps = 0, ev_next = 0;
  int ev_every = 1, ev_solves = 0;  // events on every ev_every-th solve (cmpc_batch_enable_timing_every)
};

#ifndef CMPC_REFINE_FROM_N
#define CMPC_REFINE_FROM_N 11  // first horizon whose wide classes refine (diagnostic builds move it)
#endif

// Side streams come from a process-wide pool and go back to it when a handle is destroyed; a new
// handle takes the oldest free set. The runtime maps streams onto a few hardware queues
// (GPU_MAX_HW_QUEUES = 4 by default) as they are created, and a set created while other streams
// were alive can share a hardware queue with the caller's stream: its side classes then queue
// behind class 1 (32768 instances 0.90 -> 1.17-1.25 ms per solve, 65536 1.48 -> 1.83 ms;
// scripts/stream_probe.py, profiles/r05_ab/r05_q .. r05_t). With the oldest free set first, one
// handle at a time always runs on the first handle's streams. Pooled per device.
namespace {
struct SideSet {
  int dev;
  bool busy;
  std::array<hipStream_t, cmpc::kSideStreams> s;
};
struct SidePool {
  std::mutex mu;
  std::vector<SideSet> sets;  // in creation order
};
SidePool& side_pool() {
  static SidePool* p = new SidePool();  // never destroyed: the streams live as long as the process
  return *p;
}
hipError_t acquire_sides(std::array<hipStream_t, cmpc::kSideStreams>& out, int prio) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(side_pool().mu);
  for (auto& set : side_pool().sets) {
    if (set.dev == dev && !set.busy) {
      set.busy = true;
      out = set.s;
      return hipSuccess;
    }
  }
  SideSet set{dev, true, {}};
  for (int j = 0; j < cmpc::kSideStreams; j++) {
    e = hipStreamCreateWithPriority(&set.s[j], hipStreamNonBlocking, prio);
    if (e != hipSuccess) {
      for (int k = 0; k < j; k++) (void)hipStreamDestroy(set.s[k]);
      return e;
    }
  }
  side_pool().sets.push_back(set);
  out = set.s;
  return hipSuccess;
}
void release_sides(const std::array<hipStream_t, cmpc::kSideStreams>& s) {
  std::lock_guard<std::mutex> lk(side_pool().mu);
  for (auto& set : side_pool().sets)
    if (set.s[0] == s[0]) set.busy = false;
}
}  // namespace

static cmpc::KParams make_kparams(const cmpc_params& p) {
  cmpc::KParams k{};
  k.dt = p.dt;
  k.mu_inv = 1.f / p.mu;  // fpt mu = 1.f / setup->mu (SolverMPC.cpp:657)
  k.f_max = p.f_max;
  k.alpha2 = 2.f * p.alpha;
  for (int i = 0; i < 12; i++) k.wts[i] = p.weights[i];
  k.N = p.horizon;
  k.rec_words = CMPC_REC_WORDS(p.horizon);
  k.max_iter = p.max_iter > 0 ? p.max_iter : 100;
  // the fp32 pipelines of the reference and of this solver are within ~1e-5 of the exact optimum
  // at N <= 10 and drift to ~1e-4 beyond: the refinement runs from N = 11
  k.refine = p.horizon >= CMPC_REFINE_FROM_N ? 1 : 0;
  k.dt64 = (double)k.dt;
  k.dth64 = 0.5 * k.dt64 * k.dt64;
  k.dt3_64 = k.dt64 * k.dt64 * k.dt64 / 6.0;
  k.out_cols = 12 * p.horizon;
  return k;
}

extern "C" int cmpc_record_words(int horizon) { return CMPC_REC_WORDS(horizon); }

// The float kernel of gaussian_filter (SolverMPC.cpp:404-418): taps exp(-0.5 i^2 / sigma^2)
// evaluated in double, stored as float, normalised by their float sum.
static void gauss_kernel(float sigma, int radius, float* out) {
  float sum = 0.0f;
  for (int i = -radius; i <= radius; i++) {
    const float value = std::exp(-0.5 * (i * i) / (sigma * sigma));
    out[i + radius] = value;
    sum += value;
  }
  for (int i = 0; i < 2 * radius + 1; i++) out[i] /= sum;
}

extern "C" const char* cmpc_last_error(void) { return g_last_error.c_str(); }
namespace cmpc {
void set_last_error(const char* msg) { g_last_error = msg; }  // for the other translation units
}  // namespace cmpc

// the ADMM kernel keeps M^-1 of QPs with more than 120 variables in per-workgroup fp64 slabs:
// min(max_batch, kAdmmSlabs) of (12N)^2 doubles (151 MB at N = 16, 236 MB at N = 20). They are
// allocated by the first cmpc_batch_admm call of a handle (and kept across set_params from then
// on), so handles that only run the default qpOASES-equivalent solve never pay for them; the
// solve kernels themselves never allocate.
static int ensure_admm_slabs(cmpc_batch* h) {
  if (!h->admm_used || h->max_batch <= 0 || 12 * h->prm.horizon <= 120) return 0;
  const int ns = h->max_batch < cmpc::kAdmmSlabs ? h->max_batch : cmpc::kAdmmSlabs;
  const size_t need = (size_t)ns * cmpc::admm_slab_doubles(h->prm.horizon);
  if (need <= h->admm_slab_doubles && h->admm_nslabs >= ns) return 0;
  if (h->d_admm_slabs) (void)hipFree(h->d_admm_slabs);
  h->d_admm_slabs = nullptr;
  h->admm_slab_doubles = 0;
  h->admm_nslabs = 0;
  hipError_t e = hipMalloc(&h->d_admm_slabs, need * sizeof(double));
  if (e != hipSuccess) return fail("hipMalloc(ADMM slabs)", e);
  h->admm_slab_doubles = need;
  h->admm_nslabs = ns;
  return 0;
}

extern "C" int cmpc_batch_set_params(cmpc_batch* h, const cmpc_params* prm) {
  if (!h || !prm) return -1;
  if (prm->horizon < 1 || prm->horizon > CMPC_MAX_HORIZON) {
    g_last_error = "horizon out of range";
    return -2;
  }
  h->prm = *prm;
  h->kp = make_kparams(*prm);
  if (h->out_steps > 0 && h->out_steps < prm->horizon) h->kp.out_cols = 12 * h->out_steps;
  if (!h->refine) h->kp.refine = 0;
  return ensure_admm_slabs(h);
}

extern "C" int cmpc_batch_set_refine(cmpc_batch* h, int on) {
  if (!h || on < 0 || on > 1) {
    g_last_error = "cmpc_batch_set_refine: bad arguments";
    return -1;
  }
  h->refine = on;
  h->kp.refine = (on && h->prm.horizon >= CMPC_REFINE_FROM_N) ? 1 : 0;
  return 0;
}

extern "C" int cmpc_batch_set_output_steps(cmpc_batch* h, int steps) {
  if (!h || steps < 0) {
    g_last_error = "cmpc_batch_set_output_steps: bad arguments";
    return -1;
  }
  h->out_steps = steps;
  h->kp.out_cols = 12 * ((steps > 0 && steps < h->prm.horizon) ? steps : h->prm.horizon);
  return 0;
}

extern "C" int cmpc_batch_create(cmpc_batch** out, const cmpc_params* prm, int max_batch,
                                 void* hip_stream) {
  if (!out || !prm || max_batch < 1) return -1;
  auto* h = new cmpc_batch();
  if (int r = cmpc_batch_set_params(h, prm); r != 0) {
    delete h;
    return r;
  }
  h->max_batch = max_batch;
  hipError_t e;
  if (hip_stream) {
    h->stream = (hipStream_t)hip_stream;
  } else {
    e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete h; return fail("hipStreamCreate", e); }
    h->own_stream = true;
  }
  // side streams at the highest priority: their few, long class-2 solves are dispatched ahead
  // of class 1's queue, so they finish inside class 1's run instead of forming a tail
  int prio_lo = 0, prio_hi = 0;
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (cmpc::diag_knob("CMPC_SIDE_PRIORITY", 1) == 0) prio_hi = prio_lo;
  {
    std::array<hipStream_t, cmpc::kSideStreams> sides{};
    e = acquire_sides(sides, prio_hi);
    if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("side streams", e); }
    for (int j = 0; j < cmpc::kSideStreams; j++) h->ctx.side[j] = sides[j];
    h->pooled_sides = true;
  }
  // The fork / classified / join events order queues of this one device only: every producer and
  // consumer of the data they guard is a kernel on this GPU, whose dispatch packets carry their own
  // device-scope acquire / release (the per-XCD L2s written back and invalidated at kernel
  // boundaries), and the caller's copies to the host order after the join on its stream. So these
  // events are recorded without the system-scope fence HIP adds by default (an L2 writeback and
  // invalidate per record, five records per solve): config 2 +3 to +4 %, 32768 instances +0.5 to
  // +1 %, config 3 +1 % (profiles/r06_s2/env_ab.log; device scope instead: within noise).
  // CMPC_EVENT_SCOPE (A/B): 0 HIP's default (system scope), 1 device scope, 2 no system fence
  const int ev_scope = cmpc::diag_knob("CMPC_EVENT_SCOPE", 2);
  const unsigned ev_flags = hipEventDisableTiming | (ev_scope == 1 ? hipEventReleaseToDevice
                                                     : ev_scope == 2 ? hipEventDisableSystemFence : 0u);
  for (int j = 0; j < cmpc::kSideStreams; j++) {
    e = hipEventCreateWithFlags(&h->ctx.join[j], ev_flags);
    if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("side events", e); }
  }
  e = hipEventCreateWithFlags(&h->ctx.fork, ev_flags);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&h->ctx.classified, ev_flags);
  if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("fork event", e); }
  // the class-count hint (cmpc_launch.hip): pinned, mapped, zero (no hint) until a classify pass
  // copies a finished solve's header into it
  e = hipHostMalloc(reinterpret_cast<void**>(&h->ctx.h_hint), sizeof(int) * cmpc::kHdr, hipHostMallocMapped);
  if (e == hipSuccess) {
    std::memset(h->ctx.h_hint, 0, sizeof(int) * cmpc::kHdr);
    e = hipHostGetDevicePointer(reinterpret_cast<void**>(&h->ctx.d_hint), h->ctx.h_hint, 0);
  }
  if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("hint buffer", e); }
  e = hipMalloc(&h->d_work, sizeof(int) * cmpc::work_ints(max_batch));
  if (e == hipSuccess) e = hipMemset(h->d_work, 0, sizeof(int) * 2 * cmpc::kHdr);  // both list headers
  if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("hipMalloc(work)", e); }
  {
    float taps[cmpc::kGaussTaps];
    gauss_kernel(7.0f, cmpc::kGaussR7, taps);
    gauss_kernel(27.0f, cmpc::kGaussR27, taps + 2 * cmpc::kGaussR7 + 1);
    e = hipMalloc(&h->d_gauss, sizeof(taps));
    if (e == hipSuccess) e = hipMemcpy(h->d_gauss, taps, sizeof(taps), hipMemcpyHostToDevice);
    if (e != hipSuccess) { cmpc_batch_destroy(h); return fail("gauss taps", e); }
  }
  *out = h;
  return 0;
}

static void free_staging(cmpc_batch* h);

extern "C" void cmpc_batch_destroy(cmpc_batch* h) {
  if (!h) return;
  if (h->d_work) (void)hipFree(h->d_work);
  if (h->d_gauss) (void)hipFree(h->d_gauss);
  if (h->d_admm_slabs) (void)hipFree(h->d_admm_slabs);
  free_staging(h);
  for (auto e : h->ev) (void)hipEventDestroy(e);
  if (h->pooled_sides) {
    // back to the pool once every side stream is idle (the next handle may fork on them at once)
    std::array<hipStream_t, cmpc::kSideStreams> sides{};
    for (int j = 0; j < cmpc::kSideStreams; j++) {
      sides[j] = h->ctx.side[j];
      (void)hipStreamSynchronize(sides[j]);
    }
    release_sides(sides);
  }
  for (int j = 0; j < cmpc::kSideStreams; j++)
    if (h->ctx.join[j]) (void)hipEventDestroy(h->ctx.join[j]);
  if (h->ctx.fork) (void)hipEventDestroy(h->ctx.fork);
  if (h->ctx.classified) (void)hipEventDestroy(h->ctx.classified);
  if (h->own_stream && h->stream) (void)hipStreamSynchronize(h->stream);
  if (h->ctx.h_hint) (void)hipHostFree(h->ctx.h_hint);  // (the classify kernels writing it are done)
  if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
  delete h;
}

extern "C" void* cmpc_batch_stream(cmpc_batch* h) { return h ? (void*)h->stream : nullptr; }

extern "C" int cmpc_batch_solve(cmpc_batch* h, const float* d_records, int batch, float* d_forces,
                                uint8_t* d_status, int32_t* d_iters) {
  if (!h || batch < 0 || batch > h->max_batch || (!d_records && batch) || (!d_forces && batch) ||
      (!d_status && batch)) {
    g_last_error = "cmpc_batch_solve: bad arguments";
    return -1;
  }
  hipEvent_t* ev = nullptr;
  if (h->ev_steps > 0 && h->ev_next < h->ev_steps && h->ev_solves++ % h->ev_every == 0)
    ev = &h->ev[3 * h->ev_next++];
  // (A HIP graph of this launch sequence, replayed while the arguments repeat, measured config 3
  // 41.8 M -> 32.5 M and config 2 14.7 M -> 9.8 M QP/s: the replay lost the overlap of class 1
  // with the side-stream classes, profiles/r04_ab/r04_m*. Direct launches only.)
  const hipError_t e = cmpc::launch_solve(d_records, batch, h->kp, d_forces, d_status, d_iters, h->d_work,
                                          h->max_batch, h->stream, h->ctx, ev);
  if (e != hipSuccess) return fail("launch_solve", e);
  return 0;
}

extern "C" int cmpc_batch_estimate(cmpc_batch* h, float* d_est, const float* d_logs,
                                   const float* d_fext3, const float* d_time, float sim_time,
                                   float* d_records, float* d_fext6, int batch) {
  if (!h || batch < 0 || batch > h->max_batch || (batch && (!d_est || !d_records)) ||
      (batch && !d_logs && !d_fext3)) {
    g_last_error = "cmpc_batch_estimate: bad arguments";
    return -1;
  }
  hipError_t e = cmpc::launch_estimate(d_est, d_logs, d_fext3, d_time, sim_time, d_records,
                                       h->kp.rec_words, d_fext6, h->d_gauss, batch, h->stream);
  if (e != hipSuccess) return fail("launch_estimate", e);
  return 0;
}

extern "C" int cmpc_batch_assemble(cmpc_batch* h, float* d_loco, const cmpc_loco_params* lp,
                                   float* d_records, uint8_t* d_due, int batch) {
  if (!h || !lp || batch < 0 || batch > h->max_batch ||
      (batch && (!d_loco || !d_records || !d_due)) || !(lp->dt > 0.f) ||
      lp->iters_between_mpc < 1) {
    g_last_error = "cmpc_batch_assemble: bad arguments";
    return -1;
  }
  cmpc::LocoParams kp{lp->dt,        lp->iters_between_mpc, lp->x_drag_gain,  h->kp.N,
                      h->kp.rec_words, lp->hip_x,            lp->hip_y,        lp->abad_link,
                      lp->swing_height, lp->bonus_swing,     h->kp.out_cols};
  hipError_t e = cmpc::launch_assemble(d_loco, kp, d_records, d_due, batch, h->stream);
  if (e != hipSuccess) return fail("launch_assemble", e);
  return 0;
}

extern "C" int cmpc_batch_expand(cmpc_batch* h, const float* d_compact, float* d_records, int batch) {
  if (!h || batch < 0 || batch > h->max_batch || (batch && (!d_compact || !d_records))) {
    g_last_error = "cmpc_batch_expand: bad arguments";
    return -1;
  }
  hipError_t e = cmpc::launch_expand(d_compact, d_records, batch, h->kp.N, h->kp.rec_words, h->kp.dt, h->stream);
  if (e != hipSuccess) return fail("launch_expand", e);
  return 0;
}

extern "C" int cmpc_batch_rollout(cmpc_batch* h, float* d_loco, const float* d_records,
                                  const float* d_forces, const float* d_xi6, const uint8_t* d_due,
                                  int batch) {
  if (!h || batch < 0 || batch > h->max_batch || (batch && (!d_loco || !d_records || !d_forces))) {
    g_last_error = "cmpc_batch_rollout: bad arguments";
    return -1;
  }
  cmpc::LocoParams kp{h->kp.dt, 1, 0.f, h->kp.N, h->kp.rec_words, 0.f, 0.f, 0.f, 0.f, 0.f, h->kp.out_cols};
  hipError_t e = cmpc::launch_rollout(d_loco, d_records, d_forces, d_xi6, d_due, kp, h->kp.dt,
                                      batch, h->stream);
  if (e != hipSuccess) return fail("launch_rollout", e);
  return 0;
}

extern "C" int cmpc_batch_enable_timing(cmpc_batch* h, int steps) {
  return cmpc_batch_enable_timing_every(h, steps, 1);
}

extern "C" int cmpc_batch_enable_timing_every(cmpc_batch* h, int steps, int every) {
  if (!h || steps < 0 || every < 1) return -1;
  h->ev_every = every;
  h->ev_solves = 0;
  for (auto e : h->ev) (void)hipEventDestroy(e);
  h->ev.assign(3 * (size_t)steps, nullptr);
  // recorded without the system-scope fence too (timing only; CMPC_EVENT_SCOPE as above)
  const unsigned tflags = cmpc::diag_knob("CMPC_EVENT_SCOPE", 2) == 2 ? hipEventDisableSystemFence : 0u;
  for (auto& e : h->ev)
    if (hipError_t r = hipEventCreateWithFlags(&e, tflags); r != hipSuccess) return fail("hipEventCreate", r);
  h->ev_steps = steps;
  h->ev_next = 0;
  return 0;
}

extern "C" int cmpc_batch_read_timing(cmpc_batch* h, float* ms, int* steps_recorded,
                                      int* class1_overflow) {
  if (!h) return -1;
  hipError_t e = hipStreamSynchronize(h->stream);
  if (e != hipSuccess) return fail("sync", e);
  for (int i = 0; i < h->ev_next; i++) {
    float a = 0.f, b = 0.f;
    (void)hipEventElapsedTime(&a, h->ev[3 * i], h->ev[3 * i + 1]);
    (void)hipEventElapsedTime(&b, h->ev[3 * i + 1], h->ev[3 * i + 2]);
    ms[2 * i] = a;
    ms[2 * i + 1] = b;
  }
  (void)hipGetLastError();  // an unrecorded event must not poison the next launch's check
  if (steps_recorded) *steps_recorded = h->ev_next;
  if (class1_overflow) {
    int c = 0;
    e = hipMemcpy(&c, h->d_work + h->ctx.last_hdr * cmpc::kHdr, sizeof(int), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return fail("D2H", e);
    *class1_overflow = c;
  }
  h->ev_next = 0;
  return 0;
}

extern "C" int cmpc_batch_condense(cmpc_batch* h, const float* d_records, int batch, float* d_H,
                                   float* d_g) {
  if (!h || batch < 0 || batch > h->max_batch) return -1;
  hipError_t e = cmpc::launch_condense(d_records, batch, h->kp, d_H, d_g, h->stream);
  if (e != hipSuccess) return fail("launch_condense", e);
  return 0;
}

extern "C" int cmpc_batch_admm(cmpc_batch* h, const float* d_records, const float* d_H,
                               const float* d_g, int batch, const cmpc_admm_settings* s,
                               float* d_forces, uint8_t* d_status, int32_t* d_iters) {
  if (!h || !s || batch < 0 || batch > h->max_batch ||
      (batch && (!d_records || !d_H || !d_g || !d_forces || !d_status))) {
    g_last_error = "cmpc_batch_admm: bad arguments";
    return -1;
  }
  if (!h->admm_used) {
    h->admm_used = true;
    if (int r = ensure_admm_slabs(h)) { h->admm_used = false; return r; }
  }
  hipError_t e = cmpc::launch_admm(d_records, d_H, d_g, batch, h->kp, *s, d_forces, d_status,
                                   d_iters, h->d_admm_slabs, h->admm_nslabs, h->stream);
  if (e != hipSuccess) return fail("launch_admm", e);
  return 0;
}

static void free_staging(cmpc_batch* h) {
  if (h->d_rec) (void)hipFree(h->d_rec);
  if (h->d_forces) (void)hipFree(h->d_forces);
  if (h->d_status) (void)hipFree(h->d_status);
  if (h->d_iters) (void)hipFree(h->d_iters);
  if (h->d_admm_H) (void)hipFree(h->d_admm_H);
  if (h->d_one) (void)hipFree(h->d_one);
  if (h->d_single_out) (void)hipFree(h->d_single_out);
  if (h->h_pin) (void)hipHostFree(h->h_pin);
  h->d_rec = h->d_forces = h->d_admm_H = h->d_single_out = h->h_pin = nullptr;
  h->d_status = nullptr;
  h->d_iters = nullptr;
  h->d_one = nullptr;
  h->staged = false;
}

// staging of the host-pointer entry points, allocated on first use; all or nothing (a failed
// allocation frees what was allocated, so a later call retries instead of using null buffers)
static int ensure_staging(cmpc_batch* h) {
  if (h->staged) return 0;
  const size_t words = (size_t)CMPC_REC_WORDS(CMPC_MAX_HORIZON) * h->max_batch;
  const size_t nv = 12 * (size_t)CMPC_MAX_HORIZON;  // qH / qg of one instance (single ADMM path)
  const int one[2] = {1, 0};
  hipError_t e;
  const char* what = "hipMalloc";
  // d_rec: 4 words past the last record for the single-instance ABI's (f_ext[3], simulation_time)
  if ((e = hipMalloc(&h->d_rec, (words + 4) * sizeof(float))) == hipSuccess &&
      (e = hipMalloc(&h->d_forces, (size_t)12 * CMPC_MAX_HORIZON * h->max_batch * sizeof(float))) == hipSuccess &&
      (e = hipMalloc(&h->d_status, (size_t)h->max_batch)) == hipSuccess &&
      (e = hipMalloc(&h->d_iters, sizeof(int32_t) * h->max_batch)) == hipSuccess &&
      (e = hipMalloc(&h->d_admm_H, (nv * nv + nv) * sizeof(float))) == hipSuccess &&
      (e = hipMalloc(&h->d_one, sizeof(one))) == hipSuccess &&
      (e = hipMalloc(&h->d_single_out, (12 * CMPC_MAX_HORIZON + 4) * sizeof(float))) == hipSuccess &&
      (what = "hipHostMalloc",
       e = hipHostMalloc(reinterpret_cast<void**>(&h->h_pin),
                         (CMPC_REC_WORDS(CMPC_MAX_HORIZON) + 4 + 12 * CMPC_MAX_HORIZON + 4) * sizeof(float))) == hipSuccess &&
      (what = "H2D", e = hipMemcpy(h->d_one, one, sizeof(one), hipMemcpyHostToDevice)) == hipSuccess) {
    h->staged = true;
    return 0;
  }
  free_staging(h);
  return fail(what, e);
}

// reduced size n = 3 x (stance foot-steps) of one record: eliminated iff |gait * f_max| < 0.01,
// the test of the classify pass and of every solver kernel (SolverMPC.cpp:869-894)
static int host_reduced_size(const float* rec, int N, float f_max) {
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(rec + CMPC_REC_GAIT(N));
  int nfs = 0;
  for (int t = 0; t < 4 * N; t++) {
    const float ub = (float)gait[t] * f_max;
    nfs += (ub < 0.01f && ub > -0.01f) ? 0 : 1;
  }
  return 3 * nfs;
}

// The tail classes hand an instance whose active set outgrows 64 positions to the 80-column wide
// class (cmpc_tail.hip); on the single-instance path that shows as the status byte kHandoffStatus:
// re-launch the record (already on the device) in the wide class and read the result again
static int single_handoff(cmpc_batch* h, int n, float* pin_out, int N, int32_t* iters = nullptr) {
  uint8_t st = 0;
  std::memcpy(&st, pin_out + 12 * N, 1);
  if (st != cmpc::kHandoffStatus) return 0;
  float* d_out = h->d_single_out;
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_out + 12 * N);
  hipError_t e;
  if ((e = cmpc::launch_single(h->d_rec, n, h->kp, d_out, d_st, h->d_iters, h->d_one, h->stream, false)) !=
      hipSuccess)
    return fail("launch_single", e);
  if ((e = hipMemcpyAsync(pin_out, d_out, (12 * N + 1) * sizeof(float), hipMemcpyDeviceToHost, h->stream)) !=
      hipSuccess)
    return fail("D2H", e);
  if (iters && (e = hipMemcpyAsync(iters, h->d_iters, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    return fail("D2H", e);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail("sync", e);
  return 0;
}

// batch == 1 from host memory: one kernel of the instance's class, pinned copies, one D2H
static int solve_single_host(cmpc_batch* h, const float* record, float* forces, uint8_t* status,
                             int32_t* iters) {
  const int N = h->prm.horizon;
  const size_t rw = (size_t)CMPC_REC_WORDS(N);
  const int n = host_reduced_size(record, N, h->prm.f_max);
  float* pin_rec = h->h_pin;
  float* pin_out = h->h_pin + CMPC_REC_WORDS(CMPC_MAX_HORIZON) + 4;
  std::memcpy(pin_rec, record, rw * sizeof(float));
  float* d_out = h->d_single_out;
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_out + 12 * N);
  hipError_t e;
  if ((e = hipMemcpyAsync(h->d_rec, pin_rec, rw * sizeof(float), hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return fail("H2D", e);
  if ((e = cmpc::launch_single(h->d_rec, n, h->kp, d_out, d_st, h->d_iters, h->d_one, h->stream)) !=
      hipSuccess)
    return fail("launch_single", e);
  if ((e = hipMemcpyAsync(pin_out, d_out, (12 * N + 1) * sizeof(float), hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    return fail("D2H", e);
  if (iters && (e = hipMemcpyAsync(iters, h->d_iters, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    return fail("D2H", e);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail("sync", e);
  if (int r = single_handoff(h, n, pin_out, N, iters)) return r;
  std::memcpy(forces, pin_out, h->kp.out_cols * sizeof(float));
  if (status) std::memcpy(status, pin_out + 12 * N, 1);
  return 0;
}

extern "C" int cmpc_batch_solve_host(cmpc_batch* h, const float* records, int batch, float* forces,
                                     uint8_t* status, int32_t* iters) {
  if (!h || batch < 0 || batch > h->max_batch) return -1;
  if (batch == 0) return 0;
  if (int r = ensure_staging(h)) return r;
  const int N = h->prm.horizon;
  const size_t rw = (size_t)CMPC_REC_WORDS(N);
  // one instance (the reference ABI's operating mode): the fast path, unless per-launch timing
  // is on (it brackets the batched launch sequence)
  if (batch == 1 && h->ev_steps == 0) return solve_single_host(h, records, forces, status, iters);
  hipError_t e;
  if ((e = hipMemcpyAsync(h->d_rec, records, rw * batch * sizeof(float), hipMemcpyHostToDevice, h->stream)) != hipSuccess)
    return fail("H2D", e);
  if (int r = cmpc_batch_solve(h, h->d_rec, batch, h->d_forces, h->d_status, h->d_iters)) return r;
  if ((e = hipMemcpyAsync(forces, h->d_forces, sizeof(float) * h->kp.out_cols * batch, hipMemcpyDeviceToHost,
                          h->stream)) != hipSuccess)
    return fail("D2H", e);
  if (status && (e = hipMemcpyAsync(status, h->d_status, batch, hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    return fail("D2H", e);
  if (iters && (e = hipMemcpyAsync(iters, h->d_iters, sizeof(int32_t) * batch, hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    return fail("D2H", e);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail("sync", e);
  return 0;
}

// =============================================================================================
// Reference single-instance interface (convexMPC_interface.cpp + the solve_mpc globals).
// =============================================================================================
extern "C" {
// Defined by the reference's caller (ConvexMPCLocomotion.cpp:610; be2r_cmpc_unitree_node.cpp:6);
// weak here so the library also loads on its own. The host program's definitions win.
__attribute__((weak)) float f_ext[6] = {0, 0, 0, 0, 0, 0};
__attribute__((weak)) float simulation_time = 0.f;
// The solver's own globals (SolverMPC.h:72-74, SolverMPC.cpp:390-392; Eigen::Matrix<float,6,1>
// layout): the compensation force of the last call and its two smoothed copies
float f_est[6] = {0, 0, 0, 0, 0, 0};
float f_est_smoothed[6] = {0, 0, 0, 0, 0, 0};
float f_est_static[6] = {0, 0, 0, 0, 0, 0};
}

namespace {
struct SingleState {
  std::mutex mu;
  cmpc_params cfg{};              // problem_configuration (convexMPC_interface.cpp:10)
  bool configured = false;        // the last setup_problem asked for a horizon in 1..CMPC_MAX_HORIZON
  // update_data_t fields (convexMPC_interface.h:23-41)
  float p[3]{}, v[3]{}, q[4]{}, w[3]{}, r[12]{};
  float roll = 0, pitch = 0, yaw = 0, alpha = 0, x_drag = 0;
  float weights[12]{};
  std::vector<float> traj;
  std::vector<unsigned char> gait;
  int max_iterations = 0, use_jcqp = 0;
  double rho = 0, sigma = 0, solver_alpha = 0, terminate = 0;
  // solve_mpc state
  std::vector<double> q_soln;
  int has_solved = 0;
  cmpc_batch* h = nullptr;
  int h_horizon = -1;
  // periodic-disturbance estimator state (SolverMPC.cpp:390-398, 555-563, 688-798): histories,
  // count and fit on the device (cmpc_estimator.hip ring of the last 400 samples); f_est,
  // f_est_smoothed and f_est_static are the exported globals below
  float* d_est = nullptr;
};
SingleState g;

// The estimator state of the single-instance ABI lives on the device (one CMPC_EST_WORDS slot,
// cmpc_estimator.hip): the same kernel as the batched config-5 path runs the reference's per-call
// estimator step (SolverMPC.cpp:688-798) ahead of the solve, so one implementation serves both.
int ensure_single_est(SingleState& s) {
  if (s.d_est) return 0;
  hipError_t e = hipMalloc(&s.d_est, CMPC_EST_WORDS * sizeof(float));
  if (e == hipSuccess) e = hipMemset(s.d_est, 0, CMPC_EST_WORDS * sizeof(float));
  if (e != hipSuccess) {
    if (s.d_est) (void)hipFree(s.d_est);
    s.d_est = nullptr;
    return fail("hipMalloc(estimator state)", e);
  }
  return 0;
}

// One instance through condense + ADMM on the handle's stream; the record is already in h->d_rec
// (staged with the estimator step), host forces out.
int admm_device(cmpc_batch* h, int N, const cmpc_admm_settings& as, float* forces, uint8_t* st) {
  const size_t n = 12 * (size_t)N;
  float* dH = h->d_admm_H;
  float* dg = dH + n * n;
  hipError_t e;
  int rc = cmpc_batch_condense(h, h->d_rec, 1, dH, dg);
  if (!rc) rc = cmpc_batch_admm(h, h->d_rec, dH, dg, 1, &as, h->d_forces, h->d_status, nullptr);
  if (!rc && (e = hipMemcpyAsync(forces, h->d_forces, n * sizeof(float), hipMemcpyDeviceToHost,
                                 h->stream)) != hipSuccess)
    rc = fail("D2H", e);
  if (!rc && (e = hipMemcpyAsync(st, h->d_status, 1, hipMemcpyDeviceToHost, h->stream)) != hipSuccess)
    rc = fail("D2H", e);
  if (!rc && (e = hipStreamSynchronize(h->stream)) != hipSuccess) rc = fail("sync", e);
  return rc;
}

// One solve_mpc call (SolverMPC.cpp:566-1089) of the single-instance ABI on the batch-1 handle:
// one H2D of the record with (f_ext[3], simulation_time) behind it, the estimator step on the
// device (writes f_est(3) and the use-f_est flag into the device record), then exactly one
// solver kernel of the record's size class (launch_single) or, for use_jcqp, condense + ADMM; one
// D2H of forces, status word and f_est(3).
int solve_single_device(SingleState& s, const float* rec, int N, float* forces, uint8_t* st) {
  cmpc_batch* h = s.h;
  if (int r = ensure_staging(h)) return r;
  if (int r = ensure_single_est(s)) return r;
  const size_t rw = (size_t)CMPC_REC_WORDS(N);
  float* pin_rec = h->h_pin;
  float* pin_out = h->h_pin + CMPC_REC_WORDS(CMPC_MAX_HORIZON) + 4;
  std::memcpy(pin_rec, rec, rw * sizeof(float));
  pin_rec[rw] = f_ext[3];            // diff_history.push_back(f_ext(3))  (SolverMPC.cpp:692)
  pin_rec[rw + 1] = simulation_time; // time_history.push_back(simulation_time)  (:698)
  float* d_out = h->d_single_out;    // [forces 12N][status word][f_est(3)]
  uint8_t* d_st = reinterpret_cast<uint8_t*>(d_out + 12 * N);
  hipError_t e;
  if ((e = hipMemcpyAsync(h->d_rec, pin_rec, (rw + 2) * sizeof(float), hipMemcpyHostToDevice, h->stream)) !=
      hipSuccess)
    return fail("H2D", e);
  if ((e = cmpc::launch_estimate(s.d_est, nullptr, h->d_rec + rw, h->d_rec + rw + 1, 0.f, h->d_rec, (int)rw,
                                 nullptr, h->d_gauss, 1, h->stream, d_out + 12 * N + 1)) != hipSuccess)
    return fail("launch_estimate", e);
  if (s.use_jcqp == 1 || s.use_jcqp == 2) {
    // use_jcqp == 1 (SolverMPC.cpp:818-838, 1057-1062): ADMM over the full QP; use_jcqp == 2
    // (:984-1053): over the reduced one; any horizon (QPs beyond 120 variables keep M^-1 in a
    // global slab)
    cmpc_admm_settings as{s.max_iterations, s.rho, s.sigma, s.solver_alpha, s.terminate,
                          s.use_jcqp == 2 ? 1 : 0};
    if (int r = admm_device(h, N, as, forces, st)) return r;
    if ((e = hipMemcpy(&f_est[3], d_out + 12 * N + 1, sizeof(float), hipMemcpyDeviceToHost)) != hipSuccess)
      return fail("D2H", e);
    return 0;
  }
  const int n = host_reduced_size(rec, N, h->prm.f_max);
  if ((e = cmpc::launch_single(h->d_rec, n, h->kp, d_out, d_st, h->d_iters, h->d_one, h->stream)) != hipSuccess)
    return fail("launch_single", e);
  if ((e = hipMemcpyAsync(pin_out, d_out, (12 * N + 2) * sizeof(float), hipMemcpyDeviceToHost, h->stream)) !=
      hipSuccess)
    return fail("D2H", e);
  if ((e = hipStreamSynchronize(h->stream)) != hipSuccess) return fail("sync", e);
  if (int r = single_handoff(h, n, pin_out, N)) return r;  // (f_est(3) at pin_out[12 N + 1] stays)
  std::memcpy(forces, pin_out, 12 * N * sizeof(float));
  std::memcpy(st, pin_out + 12 * N, 1);
  std::memcpy(&f_est[3], pin_out + 12 * N + 1, sizeof(float));
  return 0;
}

void solve_single(SingleState& s) {
  const int N = s.cfg.horizon;
  if (N < 1 || N > CMPC_MAX_HORIZON) {
    std::fprintf(stderr, "[cmpc] horizon %d out of range\n", N);
    return;
  }
  if (!s.h || s.h_horizon != N) {
    if (s.h) cmpc_batch_destroy(s.h);
    s.h = nullptr;
    if (cmpc_batch_create(&s.h, &s.cfg, 1, nullptr) != 0) {
      std::fprintf(stderr, "[cmpc] %s\n", cmpc_last_error());
      return;
    }
    s.h_horizon = N;
  }
  cmpc_params prm = s.cfg;
  for (int i = 0; i < 12; i++) prm.weights[i] = s.weights[i];
  prm.alpha = s.alpha;
  prm.max_iter = 100;  // nWSR = 100 (SolverMPC.cpp:854)
  if (std::memcmp(&prm, &s.h->prm, sizeof(prm)) != 0 && cmpc_batch_set_params(s.h, &prm) != 0) {
    std::fprintf(stderr, "[cmpc] %s\n", cmpc_last_error());
    return;
  }

  // the record; f_est(3) and the use-f_est flag are written by the device estimator step
  std::vector<float> rec(CMPC_REC_WORDS(N), 0.f);
  std::memcpy(&rec[CMPC_REC_P], s.p, sizeof(s.p));
  std::memcpy(&rec[CMPC_REC_V], s.v, sizeof(s.v));
  std::memcpy(&rec[CMPC_REC_Q], s.q, sizeof(s.q));
  std::memcpy(&rec[CMPC_REC_W], s.w, sizeof(s.w));
  std::memcpy(&rec[CMPC_REC_R], s.r, sizeof(s.r));
  rec[CMPC_REC_RPY + 0] = s.roll;
  rec[CMPC_REC_RPY + 1] = s.pitch;
  rec[CMPC_REC_RPY + 2] = s.yaw;
  rec[CMPC_REC_XDRAG] = s.x_drag;
  std::memcpy(&rec[CMPC_REC_TRAJ(N)], s.traj.data(), sizeof(float) * 12 * N);
  std::memcpy(&rec[CMPC_REC_GAIT(N)], s.gait.data(), 4 * N);

  std::vector<float> forces(12 * N);
  uint8_t st = 0;
  if (solve_single_device(s, rec.data(), N, forces.data(), &st) != 0) {
    std::fprintf(stderr, "[cmpc] %s\n", cmpc_last_error());
    return;
  }
  // SolverMPC.cpp:783, 798 (f_est itself came back with the forces)
  for (int i = 0; i < 6; i++) f_est_smoothed[i] = 0.95f * f_est_smoothed[i] + 0.05f * f_est[i];
  f_est_static[3] = 0.97f * f_est_static[3] + 0.03f * f_ext[3];
  const bool admm = (s.use_jcqp == 1 || s.use_jcqp == 2);
  // a failed qpOASES-equivalent solve prints as the reference does (SolverMPC.cpp:965-968) and
  // stores what the kernel wrote for it (zeros for every force); a failed ADMM
  // solve keeps the previous solution. The reference keeps JCQP's solution whatever its residual
  // (status 0 or 1).
  if (admm ? (st != 0 && st != 1) : (st != CMPC_OK)) {
    std::printf("failed to solve!\n");
    if (admm) return;
  }
  s.q_soln.assign(12 * N, 0.0);
  for (int i = 0; i < 12 * N; i++) s.q_soln[i] = forces[i];
  s.has_solved = 1;
}
}  // namespace

extern "C" void setup_problem(double dt, int horizon, double mu, double f_max) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.cfg.dt = (float)dt;
  g.cfg.horizon = horizon;
  g.cfg.mu = (float)mu;
  g.cfg.f_max = (float)f_max;
  // resize_qp_mats (SolverMPC.cpp:149-250). The staging holds the largest horizon the solver
  // admits, whatever is asked here, so no later copy depends on this call's horizon.
  g.traj.assign(12 * CMPC_MAX_HORIZON, 0.f);
  g.gait.assign(4 * CMPC_MAX_HORIZON, 0);
  g.configured = horizon >= 1 && horizon <= CMPC_MAX_HORIZON;
  if (!g.configured)
    // the reference throws from c2qp above 19 (SolverMPC.cpp:113-116) on the next solve; here
    // every update_problem_data* call refuses until a valid setup_problem and get_solution keeps
    // returning the previous solution
    std::fprintf(stderr, "[cmpc] setup_problem: horizon %d outside 1..%d; solves are refused and "
                 "the previous solution is kept\n", horizon, CMPC_MAX_HORIZON);
  else if (horizon > 19)
    std::fprintf(stderr, "[cmpc] horizon %d > 19: reference c2qp would throw; cap lifted\n", horizon);
}

namespace {
// update_problem_data* before a valid setup_problem: nothing is copied (the staging holds
// CMPC_MAX_HORIZON steps) and nothing is solved
bool refuse_update(const char* who) {
  if (g.configured) return false;
  std::fprintf(stderr, "[cmpc] %s: horizon %d not configured (setup_problem with 1..%d first); "
               "previous solution kept\n", who, g.cfg.horizon, CMPC_MAX_HORIZON);
  return true;
}
}  // namespace

extern "C" void update_solver_settings(int max_iter, double rho, double sigma, double solver_alpha,
                                       double terminate, double use_jcqp) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.max_iterations = max_iter;
  g.rho = rho;
  g.sigma = sigma;
  g.solver_alpha = solver_alpha;
  g.terminate = terminate;
  g.use_jcqp = use_jcqp > 1.5 ? 2 : (use_jcqp > 0.5 ? 1 : 0);
  // use_jcqp == 1 / 2 run the ADMM kernel (full / reduced QP)
}

extern "C" void update_problem_data_floats(float* p, float* v, float* q, float* w, float* r, float roll,
                                           float pitch, float yaw, float* weights, float* state_trajectory,
                                           float alpha, int* gait) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (refuse_update("update_problem_data_floats")) return;
  const int N = g.cfg.horizon;
  g.alpha = alpha;
  g.roll = roll;
  g.pitch = pitch;
  g.yaw = yaw;
  for (int i = 0; i < 4 * N; i++) g.gait[i] = (unsigned char)gait[i];  // mint_to_u8
  std::memcpy(g.p, p, sizeof(float) * 3);
  std::memcpy(g.v, v, sizeof(float) * 3);
  std::memcpy(g.q, q, sizeof(float) * 4);
  std::memcpy(g.w, w, sizeof(float) * 3);
  std::memcpy(g.r, r, sizeof(float) * 12);
  std::memcpy(g.weights, weights, sizeof(float) * 12);
  std::memcpy(g.traj.data(), state_trajectory, sizeof(float) * 12 * N);
  solve_single(g);
}

extern "C" void update_problem_data(double* p, double* v, double* q, double* w, double* r, double yaw,
                                    double* weights, double* state_trajectory, double alpha, int* gait) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (refuse_update("update_problem_data")) return;
  const int N = g.cfg.horizon;
  for (int i = 0; i < 3; i++) { g.p[i] = (float)p[i]; g.v[i] = (float)v[i]; g.w[i] = (float)w[i]; }
  for (int i = 0; i < 4; i++) g.q[i] = (float)q[i];
  for (int i = 0; i < 12; i++) { g.r[i] = (float)r[i]; g.weights[i] = (float)weights[i]; }
  g.yaw = (float)yaw;
  for (int i = 0; i < 12 * N; i++) g.traj[i] = (float)state_trajectory[i];
  g.alpha = (float)alpha;
  for (int i = 0; i < 4 * N; i++) g.gait[i] = (unsigned char)gait[i];
  solve_single(g);
}

void update_x_drag(float x_drag) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.x_drag = x_drag;
}

extern "C" double get_solution(int index) {
  std::lock_guard<std::mutex> lk(g.mu);
  if (!g.has_solved) return 0.f;
  // the reference reads q_soln[index] unchecked (convexMPC_interface.cpp:156-162); past the last
  // solve's 12N values this returns 0
  if (index < 0 || (size_t)index >= g.q_soln.size()) return 0.0;
  return g.q_soln[index];
}
