// cmpc_launch.hip — orchestration of the size classes for one batch solve.
//   classify (this file): n = 3 x stance foot-steps per instance (SolverMPC.cpp:869-894), the
//     instances with n > 64 appended to the list of their class;
//   class 1 (cmpc_class1.hip): every instance, one wavefront each; exits when n > 64;
//   wide classes (cmpc_wide.h: two lanes per row, NV/32 wavefronts; NV = 80, 96, 120, 128, 144,
//     192, 256; n <= 12 N <= 240 at CMPC_MAX_HORIZON = 20) each over its own list, on two side
//     streams forked after classify, so they run concurrently with class 1 and with each
//     other. At N = 10 they are a latency-bound tail (few, long solves); at N = 16..20 the 128-
//     and 192-column classes carry the batch and run side by side on the two streams.
#include <math.h>
#include <stdlib.h>

#include "cmpc_kernels.h"

namespace cmpc {

namespace {

// one thread per instance; wave-aggregated appends to the class lists. One-wave workgroups: beside
// class 1 (whose one-wave workgroups take every wave slot as it frees) a 4-wave workgroup waited
// for four free slots at once, and the pass took 1.0 ms instead of 0.05
__global__ __launch_bounds__(64) void cmpc_classify_kernel(const float* __restrict__ recs, int batch,
                                                           KParams P, int* __restrict__ cnt,
                                                           int* __restrict__ lists, int max_batch,
                                                           int c1_max, int* __restrict__ next_hdr,
                                                           int c1_listed, int tail,
                                                           int* __restrict__ host_hint,
                                                           unsigned list_mask, int header_duty) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  if (header_duty && blockIdx.x == 0 && threadIdx.x < kHdr) {
    // the next solve's counters: before zeroing them, the previous solve's final counts (the
    // header alternates) go to the host-mapped hint buffer (launch_solve sizes later grids by them)
    if (host_hint) host_hint[threadIdx.x] = next_hdr[threadIdx.x];
    next_hdr[threadIdx.x] = 0;
  }
  if (header_duty && blockIdx.x == 0 && threadIdx.x == 0) cnt[kHdrBatch] = batch;  // this solve's batch: the hint's scale
  int cls = -1;
  if (i < batch) {
    const uint32_t* g =
        reinterpret_cast<const uint32_t*>(recs + (size_t)i * P.rec_words + CMPC_REC_GAIT(P.N));
    int nfs = 0;
    for (int k = 0; k < P.N; k++) {
      const uint32_t w = g[k];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        // eliminated iff |gait * f_max| < 0.01, exactly as the solver kernels test it
        const float ub = (float)((w >> (8 * j)) & 0xffu) * P.f_max;
        nfs += (ub < 0.01f && ub > -0.01f) ? 0 : 1;
      }
    }
    const int n = 3 * nfs;
    // c1_listed (N >= 11, where few instances have n <= 64): class 1 runs over list 5 instead of
    // the whole batch, so the rest never stage their records only to exit
    // tail (N <= 10): 64 < n <= 72 in the one-wave tail class (list 9) instead of the 80-column
    // wide class (list 0)
    cls = (n <= c1_max) ? (c1_listed ? 5 : -1) : (n <= 64) ? 7 : (n <= 80) ? ((tail && n <= 72) ? 9 : 0)
        : (n <= 96) ? 1 : (n <= 120) ? 8
        : (n <= 128) ? 2 : (n <= 144) ? 6 : (n <= 192) ? 3 : 4;
  }
  const unsigned long long any = __ballot(cls >= 0);
  if (any == 0ull) return;
  const unsigned long long wide = __ballot(cls >= 0 && cls != 5);  // cnt[0]: n above class 1's build
  if (header_duty && lane == 0 && wide) atomicAdd(&cnt[0], __popcll(wide));
#pragma unroll
  for (int c = 0; c < kLists; c++) {
    if (!((list_mask >> c) & 1u)) continue;  // lists another classify launch of this solve appends
    const unsigned long long m = __ballot(cls == c);
    if (m == 0ull) continue;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&cnt[1 + c], __popcll(m));
    base = __shfl(base, leader);
    if (cls == c) lists[(size_t)c * max_batch + base + __popcll(m & ((1ull << lane) - 1ull))] = i;
  }
}

// Launch form of the wide class holding n in [lo, hi] (cmpc_wide.h): one workgroup per list entry
// for the populous classes, persistent workgroups for the sparse ones. Populous: the class meets
// 6N +- 3 sqrt(N), the trot size (two feet in stance at every step) +- one standard deviation of n
// = 3 Bin(4N, 1/2) under random contact tables. Measured (profiles/r03_ab/r03_e): every class
// one-per-entry lost config 5 2 % to the drains of the sparse classes; every class persistent
// lost config 3 / 2 2-6 % to the spills of the 80-column persistent build. Below 16384 instances
// (the same threshold as class 1's split) the drains are short and every class is one-per-entry
// (config 2: 11.3 M -> 11.7 M QP/s).
// CMPC_WIDE_FORM (A/B): 1 every class one-per-entry, 2 every class persistent.
// (Round 4: only the class holding 6 N itself one-per-entry measured -0.3 % at config 3; the same
// with the 80 class kept one-per-entry at N <= 10, i.e. the 128 class persistent at N = 20 and
// the 120 class at N = 16, -1.0 % at config 5, +0.3 % at N = 16, profiles/r04_ab/r04_t*.)
// workgroups of the 80-column class's persistent launch over the tail class's hand-offs (an
// active set past 64 positions: none in any measured workload; one workgroup solves them in turn)
constexpr int kHandoffGrid = 1;
// workgroups of the looping launch behind a one-per-entry launch of a predicted grid (entries past
// the prediction; none when it held)
constexpr int kRestGrid = 32;

bool one_per_entry(int lo, int hi, int N, int batch) {
  static const int form = diag_knob("CMPC_WIDE_FORM", 0);
  if (form == 1 || batch < 16384) return true;
  if (form == 2) return false;
  // CMPC_POP_F_HI (A/B): the populous half-width in standard deviations from N = 11 (default 1)
  static const int pop_hi = diag_knob("CMPC_POP_F_HI", 100);
  const float f = (N > 10) ? 0.01f * (float)pop_hi : 1.f;
  const float mode = 6.f * (float)N, half = f * 3.f * sqrtf((float)N);
  return (float)hi >= mode - half && (float)lo <= mode + half;
}

}  // namespace

#ifndef CMPC_C1_WHOLE_BATCH  // A/B builds: class 1 over the whole batch at every horizon (round 3)
#define CMPC_C1_WHOLE_BATCH 0
#endif
#ifndef CMPC_HDR_MEMSET
#define CMPC_HDR_MEMSET 0
#endif

hipError_t launch_solve(const float* d_recs, int batch, const KParams& P, float* d_forces,
                        uint8_t* d_status, int32_t* d_iters, int* d_work, int max_batch,
                        hipStream_t stream, LaunchCtx& ctx, hipEvent_t* ev) {
  int* cnt = d_work + ctx.hdr * kHdr;             // zero: zeroed at create or by the last classify
  int* next_hdr = d_work + (ctx.hdr ^ 1) * kHdr;  // the next solve's, zeroed by this one's classify
  int* list[kLists];
  for (int j = 0; j < kLists; j++) list[j] = d_work + 2 * kHdr + (size_t)j * max_batch;
  hipError_t e = hipSuccess;
#if CMPC_HDR_MEMSET  // A/B builds: zero the header ahead of every solve instead (rounds 1-3)
  if ((e = hipMemsetAsync(cnt, 0, kHdr * sizeof(int), stream)) != hipSuccess) return e;
#endif
  if (batch <= 0) {  // keep the timing slots consistent (zero-length launches)
    if (ev)
      for (int i = 0; i < 3; i++) (void)hipEventRecord(ev[i], stream);
    return hipSuccess;
  }
  const int n_max = 12 * P.N;  // a class no instance of this horizon can reach is not launched
  // Class 1 as two builds — 60-wide rows over the whole batch (n <= 60) and 64-wide rows over the
  // classify list of 60 < n <= 64 — once the batch fills the GPU (config 3: 28.4 M -> 29.3 M
  // QP/s). Below that the step is latency-bound and the extra kernel lengthens a side-stream
  // chain (config 2, batch 4096: 11.2 M -> 9.9 M), so one 64-wide launch takes all n <= 64.
  // CMPC_SPLIT60_MIN (A/B): the smallest batch that gets the two builds
  static const int split_min = diag_knob("CMPC_SPLIT60_MIN", 16384);
  const bool split60 = (n_max <= 64) || (batch >= split_min);
  const int c1_nv = (n_max <= 60 || split60) ? 60 : 64;
  // from N = 11 the trot size 6N is above class 1's rows and few instances reach class 1: it runs
  // over a classify list (list 5) instead of the whole batch (config 5: 65536 record stagings and
  // exits per step, 84 MB)
  const bool c1_listed = 6 * P.N > 64 && !CMPC_C1_WHOLE_BATCH;
  // 64 < n <= 80 in the one-wave tail classes (N <= 10, no refinement; cmpc_tail.hip).
  // CMPC_TAIL=0 (diagnostic builds): the 80-column wide class as before (A/B)
  // The tail class (cmpc_tail.hip) takes 64 < n <= 72 at N <= 10 whatever the batch size (so a
  // record gets the same kernel, and the same forces, in any batch). Its placement depends on the
  // batch (measured on config-3 mixes, profiles/r05_j, r05_k; against the 80-column class for
  // every n <= 80: 4096 -0.7 %, 16384 -4 %, 32768 -1.5 %, 65536 +4.4 %, 262144 +7 %):
  //   1: on the handle's stream behind class 1, alone on the GPU once class 1 drains (from 131072
  //      instances: +7 % at 262144 where beside class 1 gave +3 %);
  //   2: first on its own side stream (side 2) beside class 1 (below 131072);
  //   0: first on side 0 ahead of the 80-column class; 3: ahead of class 1 on the handle's stream.
  // CMPC_TAIL=0 (diagnostic A/B builds): the 80-column wide class for every 64 < n <= 80.
  // CMPC_T8_POS forces a placement.
  static const int tail_env = diag_knob("CMPC_TAIL", 1);
  const bool tail = tail_env != 0 && tail_class(P, 65);
  const bool tail_on = tail && n_max > 64;
  // CMPC_WIDE_FIRST (A/B, N <= 10): the classify pass first on the handle's stream, the tail and
  // wide classes (hinted grids) launched on their side streams ahead of class 1, so their long
  // solves take SIMD slots before class 1's waves fill the GPU; 2: class 1 over its classify list
  static const int wf_env = diag_knob("CMPC_WIDE_FIRST", 0);
  const bool wide_first = wf_env > 0 && !c1_listed && n_max > 64;
  const bool c1_list_mode = c1_listed || (wide_first && wf_env == 2);
  static const int t8_env = diag_knob("CMPC_T8_POS", -1);
  // CMPC_TAIL_SELF=G (A/B, N <= 10): the tail class in its self-classifying form (no classify
  // list) on side 2 ahead of everything, G workgroups (1: one per chunk) over chunks of
  // CMPC_TAIL_SELF_CHUNK instances, so its long solves hold SIMD slots from the start instead of
  // waiting for class-1 waves to retire
  static const int tself_env = diag_knob("CMPC_TAIL_SELF", 0);
  static const int tself_chunk = diag_knob("CMPC_TAIL_SELF_CHUNK", 64);
  const bool tail_self = tself_env > 0 && tail_on && tself_chunk >= 1 && tself_chunk <= 64;
  const int t8_pos = tail_self ? -1 : (t8_env >= 0) ? t8_env : ((batch >= 131072 && !wide_first) ? 1 : 2);
  // side streams forked and joined by this solve (the third only for the tail class's own chain)
  const int nsides = (tail && (t8_pos == 2 || tail_self)) ? 3 : 2;
  // CMPC_C1_SIDE=1 (A/B, N <= 10 with the tail class on side 2): class 1 and the tail class swap
  // streams — class 1 (which ends first at small batches) on side 2, the tail class on the
  // handle's stream behind the classify pass — so the join waits on queues that are already idle
  static const int c1side_env = diag_knob("CMPC_C1_SIDE", 0);
  const bool c1_swap = c1side_env == 1 && tail_on && t8_pos == 2 && !c1_list_mode;
  hipStream_t c1_stream = c1_swap ? ctx.side[2] : stream;
  // the tail class's hand-offs, behind it on its stream: a one-workgroup persistent launch of the
  // 80-column class (it reads the final count once the tail class is done)
  static const int handoff_env = diag_knob("CMPC_HANDOFF", 1);  // 0: no hand-off launch (timing A/B only)
  auto launch_handoff = [&](hipStream_t s) -> hipError_t {
    if (!handoff_env) return hipSuccess;
    return launch_wide_w80(d_recs, P, d_forces, d_status, d_iters, list[10], &cnt[11], &cnt[kDeq + 10],
                           kHandoffGrid, s);
  };
  if (tail_self) {
    const int g = (tself_env == 1) ? (batch + tself_chunk - 1) / tself_chunk : tself_env;
    if ((e = hipEventRecord(ctx.fork, stream)) != hipSuccess ||
        (e = hipStreamWaitEvent(ctx.side[2], ctx.fork, 0)) != hipSuccess ||
        (e = launch_tail_self(d_recs, batch, P, d_forces, d_status, d_iters, list[10], &cnt[11], g, tself_chunk,
                              ctx.side[2])) != hipSuccess ||
        (e = launch_handoff(ctx.side[2])) != hipSuccess)
      return e;
  }
  bool cls_side_used = false;
  int tail_grid = batch;  // the tail class's grid (hinted below when the classify pass runs)
  int tail_rest = 0;      // workgroups of its looping launch over entries past that grid
  if (n_max > 64) {
    // From 16384 instances (and up to 4096) the classify pass runs on side 0 beside class 1 (which
    // needs no list up to N = 10: it skips the instances above its row width itself), side 1
    // waiting for the lists; in between, on the handle's stream ahead of everything. Round-3 batch
    // sweep (profiles/r03_ab/sweep2): beside class 1 +2 % at 16384 .. 131072 instances.
    // CMPC_CLASSIFY_SIDE=0/1 forces either placement (A/B).
    static const int cls_env = diag_knob("CMPC_CLASSIFY_SIDE", -1);
    // (Round 4 also measured the 80-column class launched ahead of class 1 as a persistent grid
    // resident before class 1 starts: config 3 -1 to -3 %, dropped.)
    // Round-4 sweep (profiles/r04_ab/r04_ks, beside vs ahead): 2048 +2.3 %, 4096 (config 2)
    // +3.2 %, 6144 0, 8192 -2 %, 12288 -1.5 %: beside at the smallest batches too, where class 1
    // starting without the classify pass's queue hop ahead of it pays most
    const bool cls_side = c1_swap ? true : wide_first ? false : (cls_env < 0) ? (batch >= 16384 || batch <= 4096) : (cls_env == 1);
    cls_side_used = cls_side;
    // CMPC_CLS_ON_TAIL=1 (A/B): the classify pass on the tail class's own stream (side 2), so the
    // tail class follows it in the same queue instead of after a cross-queue event (4096
    // instances: classify ends at 16 us, the tail class started at 39 us; profiles/r06_s2)
    static const int cls_tail_env = diag_knob("CMPC_CLS_ON_TAIL", 0);
    const int cls_s = (cls_side && cls_tail_env == 1 && tail && t8_pos == 2 && !c1_swap) ? 2 : 0;
    hipStream_t cs = cls_side ? ctx.side[cls_s] : stream;
    if (cls_side) {
      if ((e = hipEventRecord(ctx.fork, stream)) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(ctx.side[cls_s], ctx.fork, 0)) != hipSuccess) return e;
      if (c1_swap && (e = hipStreamWaitEvent(ctx.side[2], ctx.fork, 0)) != hipSuccess) return e;
    }
    // CMPC_CLS_PER_SIDE=1 (A/B, N <= 10, classify beside class 1, the tail class on side 2): every
    // side stream runs its own classify pass over the lists it consumes (side 0: 80 and the 120 class
    // when it is there; side 1: the 64-wide class-1 build, 96, 120; side 2: the tail class), so no
    // side stream waits on another queue's event (a cross-queue event wait cost 11-21 us at 4096
    // instances and the event between classify and the 80 class on one queue ~9 us, profiles/r06_s3)
    static const int cps_env = diag_knob("CMPC_CLS_PER_SIDE", 0);
    const int w120_side_c = 6 * P.N <= 80 ? 1 : 0;
    const bool per_side = cps_env == 1 && cls_side && cls_s == 0 && tail && t8_pos == 2 && !c1_swap && !tail_self &&
                          !c1_list_mode && n_max <= 120 && nsides == 3;
    const unsigned all_lists = (1u << kLists) - 1u;
    const unsigned m0 = (1u << 0) | (w120_side_c == 0 ? (1u << 8) : 0u);
    const unsigned m1 = (1u << 1) | (1u << 7) | (w120_side_c == 1 ? (1u << 8) : 0u);
    const unsigned m2 = (1u << 9);
    if (per_side)
      for (int s = 1; s < 3; s++)
        if ((e = hipStreamWaitEvent(ctx.side[s], ctx.fork, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(cmpc_classify_kernel, dim3((batch + 63) / 64), dim3(64), 0, cs,
                       d_recs, batch, P, cnt, d_work + 2 * kHdr, max_batch, c1_nv, next_hdr, c1_list_mode ? 1 : 0,
                       tail ? 1 : 0, ctx.d_hint, per_side ? m0 : all_lists, 1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (per_side)
      for (int s = 1; s < 3; s++) {
        hipLaunchKernelGGL(cmpc_classify_kernel, dim3((batch + 63) / 64), dim3(64), 0, ctx.side[s],
                           d_recs, batch, P, cnt, d_work + 2 * kHdr, max_batch, c1_nv, next_hdr, 0,
                           tail ? 1 : 0, nullptr, s == 1 ? m1 : m2, 0);
        if ((e = hipGetLastError()) != hipSuccess) return e;
      }
    ctx.last_hdr = ctx.hdr;
    if (!CMPC_HDR_MEMSET) ctx.hdr ^= 1;
    if (!per_side && (e = hipEventRecord(ctx.classified, cs)) != hipSuccess) return e;
    for (int s = 0; s < nsides && !per_side; s++)
      if (!(cls_side && s == cls_s) && !(c1_swap && s == 2) && !(tail_self && s == 2) && (e = hipStreamWaitEvent(ctx.side[s], ctx.classified, 0)) != hipSuccess) return e;
    if (c1_swap && (e = hipStreamWaitEvent(stream, ctx.classified, 0)) != hipSuccess) return e;
    // launch form per wide class (cmpc_wide.h): one workgroup per entry for the class that holds
    // the trot size n = 6N, persistent workgroups (dequeue counter) for the others
    auto dq = [&](int lst, int lo, int hi) -> int* {
      return one_per_entry(lo, hi, P.N, batch) ? nullptr : &cnt[kDeq + lst];
    };
    int grid_of[kLists];
    // Grids from the class counts of an earlier solve, from 16384 instances. The classify kernel
    // copies a finished solve's header to the host-mapped ctx.h_hint (no host wait); scaled to
    // this batch with a quarter and 64 workgroups of slack it sizes the wide classes' and the
    // tail class's grids. A class launched one workgroup per possible entry ends only when its
    // empty workgroups have drained, and at mid-size batches those wait for SIMD slots behind
    // class 1: at 32768 instances the tail class and the 96 class ended 0.12-0.18 ms after class 1
    // (profiles/r06_p). The persistent forms dequeue any count, so a hinted grid only bounds their
    // workgroups; a one-per-entry launch over the predicted entries is followed on its stream by a
    // small looping launch over any entries past them (kRestGrid workgroups of the class's
    // persistent build, or the tail class's looping kernel), which exit at once when the
    // prediction held. A class carrying the batch (N = 16's 96 class, N = 20's 120 class) predicts
    // more than the batch and keeps a batch-sized grid; config 5's 128 class no longer launches
    // 65536 workgroups for its few thousand instances. Below 16384 instances the drains are short and the grids stay batch-sized
    // (a hint there measured +-0.3 %, profiles/r06_hint2). CMPC_HINT=0 (A/B): no hints.
    static const int hint_env = diag_knob("CMPC_HINT", 1);
    static const int hint_min = diag_knob("CMPC_HINT_MIN", 16384);
    const volatile int* hint = (hint_env && ctx.h_hint && batch >= hint_min) ? ctx.h_hint : nullptr;
    const int hint_batch = hint ? hint[kHdrBatch] : 0;
    const bool hinting = hint_batch > 0;
    for (int j = 0; j < kLists; j++) {
      grid_of[j] = batch;
      if (!hinting) continue;
      const double g = (double)hint[1 + j] * (double)batch / (double)hint_batch * 1.25 + 64.0;
      if (g < (double)batch) grid_of[j] = (int)g;
    }
    grid_of[5] = grid_of[7] = batch;  // class-1 lists: their kernel takes one entry per workgroup
    // CMPC_EXACT_GRID=1 (diagnostic): read this solve's list lengths back first (a host round
    // trip per solve) and launch exact grids. Round 6 (profiles/r06_exact): 4096 instances -3 to
    // -9 %, 32768 -2 to -4 %, 65536 -4 %, N = 16 +1.4 % — the host wait holds class 1's launch back
    static const bool exact = diag_knob("CMPC_EXACT_GRID", 0) == 1;
    if (exact) {
      static int* h_cnt = nullptr;
      if (!h_cnt && (e = hipHostMalloc(reinterpret_cast<void**>(&h_cnt), kHdr * sizeof(int))) != hipSuccess)
        return e;
      if ((e = hipMemcpyAsync(h_cnt, cnt, kHdr * sizeof(int), hipMemcpyDeviceToHost, cs)) != hipSuccess ||
          (e = hipStreamSynchronize(cs)) != hipSuccess)
        return e;
      for (int j = 0; j < kLists; j++) grid_of[j] = h_cnt[1 + j];
    }
    const bool rest = hinting && !exact;  // entries past a predicted grid are possible
    tail_grid = grid_of[9];
    tail_rest = rest && tail_grid < batch ? kRestGrid : 0;
    // one wide class: persistent (hinted grid) or one-per-entry (+ the rest launch behind it)
    using WideFn = hipError_t (*)(const float*, const KParams&, float*, uint8_t*, int32_t*, const int*,
                                  const int*, int*, int, hipStream_t, int);
    auto wide = [&](WideFn fn, int lst, int lo, int hi, hipStream_t s) -> hipError_t {
      int* d = dq(lst, lo, hi);
      if (d) return fn(d_recs, P, d_forces, d_status, d_iters, list[lst], &cnt[1 + lst], d, grid_of[lst], s, 0);
      const int g = grid_of[lst];
      hipError_t r = fn(d_recs, P, d_forces, d_status, d_iters, list[lst], &cnt[1 + lst], nullptr, g, s, 0);
      if (r != hipSuccess || !rest || g >= batch) return r;
      return fn(d_recs, P, d_forces, d_status, d_iters, list[lst], &cnt[1 + lst], &cnt[kDeq + lst], kRestGrid, s,
                g);
    };
    // the tail class first on side 0 / side 2 (t8_pos above), its hand-offs (list 10) to the
    // 80-column class right behind it on the same stream
    hipStream_t t8_stream = c1_swap ? stream : ctx.side[(t8_pos == 0 || t8_pos == 2) ? t8_pos : 0];
    if (tail && (t8_pos == 0 || t8_pos == 2) &&
        ((e = launch_tail(d_recs, P, d_forces, d_status, d_iters, list[9], &cnt[10], list[10], &cnt[11],
                          grid_of[9], t8_stream, tail_rest)) != hipSuccess ||
         (e = launch_handoff(t8_stream)) != hipSuccess))
      return e;
    // CMPC_W96_FIRST (diagnostic A/B): the 96-column class ahead of the 64-wide class-1 build on
    // side 1 (its few long solves start at once instead of behind that build)
    static const int w96_first = diag_knob("CMPC_W96_FIRST", 0);
    auto launch_w96 = [&]() -> hipError_t {
      return n_max > 80 ? wide(launch_wide_w96, 1, 81, 96, ctx.side[1]) : hipSuccess;
    };
    // The 120-column build (97..120; at N <= 13 almost always empty: all-stance tables only) on
    // side 1 behind the 64-wide class-1 build and the 96 class. There its launch (a 14 us drain of
    // its empty persistent grid at 32768 instances) is the last kernel of the step
    // (profiles/r06_p), but ahead of them (CMPC_W120_FIRST=1, round 6) the drain waits for SIMD
    // slots while class 1 fills the GPU and holds the 64-wide build and the 96 class back:
    // 32768 instances -17 %, 65536 -14 %, 262144 -2 %, 4096 +0.3 % (profiles/r06_w120/ab.log).
    static const int w120_env = diag_knob("CMPC_W120_SIDE", -1);
    const int w120_side = (w120_env >= 0) ? (w120_env & 1) : (6 * P.N <= 80 ? 1 : 0);
    static const int w120_skip = diag_knob("CMPC_SKIP_W120", 0);  // timing A/B only (n 97-120 unsolved)
    static const int w120_first = diag_knob("CMPC_W120_FIRST", 0);
    const bool w120_early = w120_first && w120_side == 1;
    auto launch_w120 = [&]() -> hipError_t {
      return (n_max > 96 && !w120_skip)
                 ? wide(launch_wide_w120, 8, 97, 120, ctx.side[w120_side])
                 : hipSuccess;
    };
    if (w120_early && (e = launch_w120()) != hipSuccess) return e;
    if (w96_first && (e = launch_w96()) != hipSuccess) return e;
    // the 64-wide class-1 build over its list (60 < n <= 64), ahead of the wide classes on side 1
    // (side 0 carries the 80 class, the longest chain at N = 10)
    if (split60 && (e = launch_class1(64, d_recs, batch, P, d_forces, d_status, d_iters, list[7],
                                      &cnt[8], nullptr, nullptr, grid_of[7], ctx.side[1])) != hipSuccess)
      return e;
    // side 0: 80, 120, 144, 256; side 1: 96, 128, 192 (at N = 20 the 120-column class, which
    // carries the batch, runs beside the 128-column class)
    if ((e = wide(launch_wide_w80, 0, 65, 80, ctx.side[0])) != hipSuccess) return e;
    if (!w96_first && (e = launch_w96()) != hipSuccess) return e;
    // the 120-column build on side 0 from N = 14 (every trot instance at N = 17..20, beside the
    // 96-column trot class at N = 14..16); below, on side 1 behind the sparse 96 class: at N = 10
    // its launch (few or no instances) otherwise lengthens side 0's 80-class chain, the step's
    // critical path (config 3 timeline, profiles/r04_prof). CMPC_W120_SIDE=0/1 forces a side (A/B)
    if (!w120_early && (e = launch_w120()) != hipSuccess) return e;
    if (n_max > 120 && (e = wide(launch_wide_w128, 2, 121, 128, ctx.side[1])) != hipSuccess) return e;
    // The 144 class on side 0 behind the 120 class, the 192 class on side 1 behind the 128 class:
    // at N = 20 the two sparse classes then start as soon as either bulk class drains and run side
    // by side instead of back to back. Config 5 4.21 M -> 4.41 M QP/s against both on side 1
    // (profiles/r03_ab/sparse_side). CMPC_SPARSE_SIDE (A/B): the side streams of the 144 / 192
    // classes as two digits (11 = both on side 1)
    static const int sparse_side = diag_knob("CMPC_SPARSE_SIDE", 1);
    if (n_max > 128 &&
        (e = launch_wide_w144(d_recs, P, d_forces, d_status, d_iters, list[6], &cnt[7], &cnt[kDeq + 6], grid_of[6],
                              ctx.side[(sparse_side / 10) & 1])) != hipSuccess)
      return e;
    if (n_max > 144 && (e = launch_wide_w192(d_recs, P, d_forces, d_status, d_iters, list[3], &cnt[4], &cnt[kDeq + 3],
                                             grid_of[3], ctx.side[sparse_side % 10 & 1])) != hipSuccess)
      return e;
    if (n_max > 192 && (e = launch_wide_w256(d_recs, P, d_forces, d_status, d_iters, list[4], &cnt[5], &cnt[kDeq + 4],
                                             grid_of[4], ctx.side[0])) != hipSuccess)
      return e;
  }
  if (tail_on && t8_pos == 3) {  // the tail class ahead of class 1 on the handle's stream
    if (cls_side_used && (e = hipStreamWaitEvent(stream, ctx.classified, 0)) != hipSuccess) return e;
    if ((e = launch_tail(d_recs, P, d_forces, d_status, d_iters, list[9], &cnt[10], list[10], &cnt[11], tail_grid,
                         stream, tail_rest)) != hipSuccess ||
        (e = launch_handoff(stream)) != hipSuccess)
      return e;
  }
  if (ev) (void)hipEventRecord(ev[0], c1_stream);
  // class 1: up to N = 10 over the whole batch (it skips the instances above its row width
  // itself), from N = 11 over list 5
  if (c1_list_mode) {
    // class 1 over the classify list of n <= its row width (one workgroup per possible entry,
    // surplus ones exit after reading the count): behind the classify pass
    if (cls_side_used && (e = hipStreamWaitEvent(stream, ctx.classified, 0)) != hipSuccess) return e;
    e = launch_class1(c1_nv, d_recs, batch, P, d_forces, d_status, d_iters, list[5], &cnt[6], nullptr,
                      nullptr, batch, stream);
  } else {
    e = launch_class1(c1_nv, d_recs, batch, P, d_forces, d_status, d_iters, nullptr, nullptr, nullptr,
                      nullptr, batch, c1_stream);
  }
  if (e != hipSuccess) return e;
  if (tail_on && t8_pos == 1) {  // the tail class behind class 1 on the handle's stream
    if (cls_side_used && (e = hipStreamWaitEvent(stream, ctx.classified, 0)) != hipSuccess) return e;
    if ((e = launch_tail(d_recs, P, d_forces, d_status, d_iters, list[9], &cnt[10], list[10], &cnt[11], tail_grid,
                         stream, tail_rest)) != hipSuccess ||
        (e = launch_handoff(stream)) != hipSuccess)
      return e;
  }
  if (ev) (void)hipEventRecord(ev[1], c1_stream);
  if (n_max > 64) {
    for (int s = 0; s < nsides; s++) {
      if ((e = hipEventRecord(ctx.join[s], ctx.side[s])) != hipSuccess) return e;
      if ((e = hipStreamWaitEvent(stream, ctx.join[s], 0)) != hipSuccess) return e;
    }
  }
  if (ev) (void)hipEventRecord(ev[2], stream);
  return hipSuccess;
}

// One instance whose reduced size n the caller already knows (counted on the host from the
// record's gait table, the same test as the classify pass): exactly one kernel of the right
// class, no classify pass, no side-stream fork/join. d_one = {1, 0}: a one-entry instance list.
hipError_t launch_single(const float* d_rec, int n, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* d_one, hipStream_t stream,
                         bool allow_tail) {
  const int* cnt = d_one;
  const int* lst = d_one + 1;
  if (n <= 64)
    return launch_class1(n <= 60 ? 60 : 64, d_rec, 1, P, d_forces, d_status, d_iters, nullptr,
                         nullptr, nullptr, nullptr, 1, stream);
  static const int tail_env = diag_knob("CMPC_TAIL", 1);
  const bool in_tail = tail_env != 0 && tail_class(P, n);
  if (allow_tail && in_tail)
    return launch_tail(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, nullptr, 1, stream);
  if (!allow_tail && in_tail)  // a tail-class hand-off: the form the batched launch uses
    return launch_wide_w80_persist(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, stream);
  // the launch form the batched launch of this class would pick for a batch of one (one workgroup
  // per entry; the persistent form runs its loop once with deq == nullptr). Both forms round
  // alike (-ffp-contract=on, build.py): tests/test_gpu_parity.py::test_batch_size_invariance
  // solves the same records in a batch of 16384 (persistent sparse classes), in batches of 4096
  // and one at a time and requires bitwise-equal forces
#define CMPC_SINGLE_WIDE(W, LO, HI)                                                                 \
  if (n <= HI)                                                                                      \
    return one_per_entry(LO, HI, P.N, 1)                                                            \
               ? launch_wide_w##W(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, stream) \
               : launch_wide_w##W##_persist(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, \
                                            stream);
  CMPC_SINGLE_WIDE(80, 65, 80)
  CMPC_SINGLE_WIDE(96, 81, 96)
  CMPC_SINGLE_WIDE(120, 97, 120)
  CMPC_SINGLE_WIDE(128, 121, 128)
#undef CMPC_SINGLE_WIDE
  if (n <= 144) return launch_wide_w144(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, stream);
  if (n <= 192) return launch_wide_w192(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, stream);
  return launch_wide_w256(d_rec, P, d_forces, d_status, d_iters, lst, cnt, nullptr, 1, stream);
}

}  // namespace cmpc
