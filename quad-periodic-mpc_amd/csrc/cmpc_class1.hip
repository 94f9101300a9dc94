// cmpc_class1.hip — the hot path: fused condensation + friction-cone QP for instances with
// n <= 64 reduced force variables (every trot instance at N <= 10), one wavefront per instance.
//
// One wavefront computes one call of the reference's solve_mpc()
// (be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-982):
//   stance table + swing elimination (SolverMPC.cpp:859-894), model + closed-form c2qp
//   (cmpc_common.h), condensation of the reduced qH / qg (SolverMPC.cpp:806-814), the dense
//   QP (qpOASES QProblem::init in the reference, SolverMPC.cpp:955-969) solved exactly by a
//   Goldfarb-Idnani dual active-set method, scatter to q_soln (SolverMPC.cpp:970-982).
//
// MI355X mapping:
//   * lane v owns reduced variable v: row v of H, then of the Cholesky working matrix, then
//     row v of J = L^-T, held in 65 VGPRs (slot[0..63] + the gradient border slot[64]);
//   * LDS holds one packed 64x64 upper-row matrix (8.5 KB): H during assembly, then the raw
//     Cholesky columns. Because the trailing matrix of a right-looking Cholesky stays
//     symmetric, pivot column k is "register slot[k] of every lane": ONE ds_write_b32 per step
//     publishes it, and the broadcast reads are ds_read_b128;
//   * J = L^-T is solved left-looking inside the factorisation's pair steps: the stored columns
//     are -L's, lane v keeps x_j = J[v][j] in the registers of the finished H columns, and each
//     step adds the row sums over the finished columns (16-B broadcasts, four rows per read);
//   * the QP's triangular factor R is explicit, packed upper columns in the LDS region that held
//     L; its back substitution and re-triangularisation are readlane chains, and the J rows see
//     only straight-line Givens chains (identity rotations outside the active range);
//   * every loop over matrix columns is unrolled at compile time, so register indices are
//     constants; LDS traffic between lanes of the single wavefront needs no s_barrier.
// Everything is fp32 (the reference condenses in fp32: common_types.h:14).
#include <stdlib.h>

#include "cmpc_common.h"

#ifndef CMPC_W1_WAVES_60  // the 60-wide build's occupancy target (A/B builds; 5 measured config 3 -18 %, r04_q)
#define CMPC_W1_WAVES_60 4
#endif
#ifndef CMPC_W1_WAVES_PER_EU
#define CMPC_W1_WAVES_PER_EU 4
#endif
// Cholesky sweep chunks (of every 4) whose column broadcast goes through v_readlane instead of
// the LDS (see the Cholesky stage)
#ifndef CMPC_C1_RL
#define CMPC_C1_RL 0
#endif
// Active-set trips after which a wave raises its issue priority (0: never): the instances with
// many trips set the end of a batch that does not fill the GPU many times over
#ifndef CMPC_TRIP_PRIO_AT
#define CMPC_TRIP_PRIO_AT 0
#endif
#ifndef CMPC_C1_TRIP_PRIO
#define CMPC_C1_TRIP_PRIO 2
#endif
// chunks per group of the software-pipelined vector sweeps (piped_sweep)
#ifndef C1_PIPE_GRP
#define C1_PIPE_GRP 4
#endif
// Cholesky two pivots per step (rank-2 sweeps); 0: one pivot per step
#ifndef CMPC_C1_CHOL2
#define CMPC_C1_CHOL2 1
#endif
// J = L^-T left-looking inside the Cholesky's pair steps (no separate J pass; CMPC_C1_CHOL2 only):
// 2 four rows per 16-B read (config 3 +2 %, 32768 instances +2 %, 4096 +1.5 %, profiles/r06_s7),
// 1 two rows per 8-B read (-3 to -4 %), 0 the separate right-looking pass after the factorisation
#ifndef CMPC_C1_FUSEDJ
#define CMPC_C1_FUSEDJ 2
#endif
// (form 2) the J row sums' column loads software-pipelined one group ahead: config 3 +0.9 /
// +1.3 %, 4096 +0.6 / +0.8 %, 32768 -0.2 % (profiles/r06_s9/lib_ab.log); 0: one group at a time
#ifndef CMPC_C1_JPIPE
#define CMPC_C1_JPIPE 1
#endif
// the active set's row-long dot products (z = J2 d2, |d2|^2, J_v . w) as two interleaved FMA
// chains (dot4x2) instead of one (A/B)
#ifndef CMPC_C1_DOT2
#define CMPC_C1_DOT2 0
#endif
#if CMPC_C1_DOT2
#define C1_DOT dot4x2
#else
#define C1_DOT dot4
#endif
// (form 2) x = -J y accumulated inside the factorisation (two FMAs per pair step with the
// step's border values) instead of an LDS sweep after it: config 3 +0.8 / +1.8 %, 4096 +0.3 /
// +0.9 %, 32768 -0.4 / +1.4 % (profiles/r06_s12/lib_ab.log)
#ifndef CMPC_C1_XUNC
#define CMPC_C1_XUNC 1
#endif

// Phase profiler (diagnostic builds only, -DCMPC_PHASE_PROF): lane 0 of every solved instance
// adds the s_memtime cycles spent in each stage to g_c1_phase (scripts/phase_prof.py).
#ifdef CMPC_PHASE_PROF
__device__ unsigned long long g_c1_phase[16];
#define C1_MARK(i)                              \
  do {                                          \
    const unsigned long long _n = clock64();    \
    ph[i] += _n - t_last;                       \
    t_last = _n;                                \
  } while (0)
// active-set loop segments [8 + i], timed from the top of the trip
#define C1_SUB(i)                               \
  do {                                          \
    const unsigned long long _n = clock64();    \
    ph[8 + (i)] += _n - t_sub;                  \
    t_sub = _n;                                 \
  } while (0)
#else
#define C1_MARK(i) \
  do {             \
  } while (0)
#define C1_SUB(i) \
  do {            \
  } while (0)
#endif

// Placement profiler (diagnostic builds only, -DCMPC_PLACE_PROF): per instance the hardware
// wave id, the XCC id and the wall-clock (100 MHz) start / end of its wavefront
// (scripts/place_prof.py).
#ifdef CMPC_PLACE_PROF
constexpr int kPlaceMax = 65536;
__device__ unsigned int g_c1_place[4 * kPlaceMax];
#endif

namespace cmpc {
namespace {

constexpr int NL = 64;  // lanes of the wavefront (per-lane LDS arrays are sized by it)

// Row width NV (60 or 64: the 60-wide build takes every instance with n <= 60, i.e. all trot
// instances at N = 10, and saves the padding columns of the 64-wide sweeps); lanes v >= NV of a
// 60-wide build own no row.
template <int NV>
struct C1Geo {
  static constexpr int NG = NV / 4;
  static constexpr int PSZ = 4 * NG * NV - 8 * NG * (NG - 1);  // packed rows r: columns [r & ~3, NV)
  // offset of packed row r (16-B aligned)
  __host__ __device__ static constexpr int prow(int r) {
    return 4 * (r >> 2) * NV - 8 * (r >> 2) * ((r >> 2) - 1) + (r & 3) * (NV - 4 * (r >> 2));
  }
  // prow(r) - (r & ~3): element (r, c) lives at prow0(r) + c
  __host__ __device__ static constexpr int prow0(int r) { return prow(r) - (r & ~3); }
  // H's exchange between the condensation and the row loads: the plain packed upper triangle,
  // element (r, c >= r) at tri(r) + c. Lane v stores its row and loads the entries c >= v at
  // tri(v) + c: with these unaligned row starts the lanes of a half-wave hit distinct banks
  // (with the 16-B aligned rows of prow, which the Cholesky's ds_read_b128 broadcasts need, only
  // 16 bank groups: 650 -> 215 extra LDS cycles per instance at NV = 60 by a bank model)
  __host__ __device__ static constexpr int tri(int r) { return r * NV - ((r * (r + 1)) >> 1); }
  static_assert(NV * NV - ((NV * (NV + 1)) >> 1) <= 4 * NG * NV - 8 * NG * (NG - 1), "exchange fits P");
};
// R (upper triangular, q x q) packed by columns: R[i][j] at rcol(j) + i, i <= j
__device__ __forceinline__ int rcol(int j) { return (j * (j + 1)) >> 1; }
// largest q whose two packed triangles fit in `words`
constexpr int rinv_cols(int words) {
  int q = 0;
  while ((q + 1) * (q + 2) <= words) q++;
  return q;
}

// prep scratch inside P (P is not yet holding H while these are live)
constexpr int OFF_E = 0;
constexpr int OFF_ZE = OFF_E + 16 * MAXN;
constexpr int OFF_REC = OFF_ZE + 16 * MAXN;  // LDS copy of the instance record (16-B aligned)

// stance foot-steps a class-1 instance can have (n = 3 x stance <= 64); the stance scan stores
// only that many (an instance with more is handed on before they are read)
constexpr int C1_MAXFS = 24;

template <int NV>
struct SharedC1 {
  static_assert(NV % 4 == 0 && NV <= NL, "row width");
  static_assert(NV * (NV + 1) / 2 <= C1Geo<NV>::PSZ, "R must fit in P");
  static_assert(OFF_REC + CMPC_REC_WORDS(MAXN) <= C1Geo<NV>::PSZ, "prep scratch must fit in P");
  static_assert(3 * C1_MAXFS >= NV, "stance list");
  // the broadcast vector (y, then the masked d / Householder vector) lives in P's last NL words
  // once J is formed: the factor rows are dead, and R (at most NV (NV + 1) / 2 words) stays below
  // it. 256 B less: the 64-wide build fits 10 KB, i.e. 16 workgroups per CU (it had 15)
  static_assert(NV * (NV + 1) / 2 <= C1Geo<NV>::PSZ - NL, "vbuf in P's tail");
  __device__ __forceinline__ float* vbuf() { return &P[C1Geo<NV>::PSZ - NL]; }
  // R^-1 (active-set phase, while the active set has at most QI positions and nothing was
  // dropped): packed by columns like R, below vbuf; R's first QI columns stay below it
  static constexpr int QI = rinv_cols(C1Geo<NV>::PSZ - NL);
  static constexpr int RB = C1Geo<NV>::PSZ - NL - QI * (QI + 1) / 2;
  static_assert(QI * (QI + 1) / 2 <= RB, "R and R^-1 side by side");
  float P[C1Geo<NV>::PSZ];
  // arrays of different stages share one region: 10 KB of LDS per instance at NV = 60, so
  // sixteen one-wave workgroups (four waves per SIMD) fit a CU's 160 KB
  union {
    float BdtT[12][16];    // prep + condensation: Bdt transposed
    float ibuf[NL];        // Cholesky + J: 1 / sqrt(d_k) of pivot k
    struct {               // active set
      float bufA[NL], bufB[NL];  // published J rows ia (bufA) and iz (bufB + 16, running into cs)
      float cs[2 * NL];    // Givens (c, s) per column pair
    } gi;
  } u;
  float sub[C1_MAXFS];     // ub of each stance foot-step (gait * f_max)
  int sfs[C1_MAXFS];       // stance foot-step ids, in order
  int blkbase[MAXN + 2];   // first reduced variable of each horizon step
  unsigned char varblk[NL], varcol[NL];
  unsigned char cmask[NL];  // active flags of stance foot-step s's 6 constraints (bit t of byte s)
};

__device__ __forceinline__ void lsync() {
  // single-wavefront workgroup: LDS ops of one wave execute in issue order; this only stops
  // the compiler from moving LDS accesses across the point
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float fdiv(float a, float b) { return a * fast_rcp(b); }

// Register pin: forces every row element to be materialised at this point. Without it LLVM sinks
// the right-looking updates of slot[c] down to the step that first reads slot[c] (turning the
// factorisation left-looking in registers: O(n) multipliers and pivot values live per column,
// >1000 VGPR spills).
template <int M>
__device__ __forceinline__ void pin(float (&x)[M]) {
#pragma unroll
  for (int c = 0; c < M; c++) asm volatile("" : "+v"(x[c]));
}

// Scheduling fence inside long unrolled LDS->FMA sweeps: without it the scheduler issues every
// ds_read_b128 of a row up front (64 extra live VGPRs on top of the 65-slot row).
#ifndef CMPC_FENCE_COLS
#define CMPC_FENCE_COLS 16
#endif
#define CMPC_SWEEP_FENCE(c)                                                                  \
  do {                                                                                       \
    if (((c) & (CMPC_FENCE_COLS - 1)) == CMPC_FENCE_COLS - 4) __builtin_amdgcn_sched_barrier(0); \
  } while (0)

template <int NV>
__device__ __forceinline__ void solve_c1(const float* __restrict__ rec, const KParams& P,
                                         SharedC1<NV>& sh, float* __restrict__ fout,
                                         uint8_t* __restrict__ st_out, int32_t* __restrict__ it_out,
                                         int* __restrict__ ovf_list, int* __restrict__ ovf_count,
                                         int inst) {
  using G = C1Geo<NV>;
  const int v = threadIdx.x;
  const int N = P.N;
#ifdef CMPC_PHASE_PROF
  unsigned long long ph[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_sub = 0;
  unsigned long long t_last = clock64();
#endif
  // ---- stage the record in LDS: one 16-B load per lane, so the whole prep waits on a single
  // HBM round trip (record words are a multiple of 4, records 16-B aligned)
  {
    const float4* src = reinterpret_cast<const float4*>(rec);
    float4* dst = reinterpret_cast<float4*>(&sh.P[OFF_REC]);
    for (int t = v; t < (P.rec_words >> 2); t += 64) dst[t] = src[t];
  }
  lsync();
  const float* srec = &sh.P[OFF_REC];
  // ---- stance table + elimination: eliminated iff |gait * f_max| < 0.01 (SolverMPC.cpp:869-894)
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(srec + CMPC_REC_HDR + 12 * N);
  int nfs = 0;
  unsigned long long msk0 = 0ull, msk1 = 0ull;  // stance ballots of foot-steps 0..63, 64..127
  for (int c0 = 0; c0 < 4 * N; c0 += 64) {
    const int t = c0 + v;
    float ub = 0.f;
    bool f = false;
    if (t < 4 * N) {
      ub = (float)gait[t] * P.f_max;
      f = !(ub < 0.01f && ub > -0.01f);
    }
    const unsigned long long m = __ballot(f);
    if (c0 == 0) msk0 = m; else msk1 = m;
    const int pre = __popcll(m & ((1ull << v) - 1ull));
    if (f && nfs + pre < C1_MAXFS) {
      sh.sfs[nfs + pre] = t;
      sh.sub[nfs + pre] = ub;
    }
    nfs += __popcll(m);
  }
  const int n = 3 * nfs;
  if (n > NV) {  // hand the instance to the next size class
    if (v == 0 && ovf_list) ovf_list[atomicAdd(ovf_count, 1)] = inst;
    return;
  }
  lsync();
  {
    int kb = 0, kc = 0;
    if (v < n) {
      const int fs = sh.sfs[v / 3];
      kb = fs >> 2;
      kc = 3 * (fs & 3) + v % 3;
    }
    sh.varblk[v] = (unsigned char)kb;
    sh.varcol[v] = (unsigned char)kc;
    if (v <= N) {  // stance foot-steps before step v: popcounts of the ballots
      const int b0 = 4 * v, b1 = 4 * v - 64;
      const unsigned long long lo = (b0 >= 64) ? msk0 : (msk0 & ((1ull << b0) - 1ull));
      const unsigned long long hi = (b1 <= 0) ? 0ull : (msk1 & ((1ull << b1) - 1ull));
      sh.blkbase[v] = 3 * (__popcll(lo) + __popcll(hi));
    }
    for (int t = v; t < nfs; t += 64) sh.cmask[t] = 0;
  }
  Model md;
  make_model(srec, P.dt, md);
  make_bdt<64>(srec, md, v, sh.u.BdtT);
  lsync();
  if (v < N) {
    float e[13];
    state_error(srec, md, v, srec + CMPC_REC_HDR + 12 * v, e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.P[OFF_E + 16 * v + j] = e[j];
  }
  lsync();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  // gradient recursion ze_i = S e_i + Adt' ze_{i+1} (uniform: every lane computes it, lane j
  // stores component j)
  {
    float ze[13];
#pragma unroll
    for (int j = 0; j < 13; j++) ze[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      float e[13];
#pragma unroll
      for (int j = 0; j < 13; j++) e[j] = sh.P[OFF_E + 16 * i + j];
      recur(md, wts, e, ze);
      float mine = 0.f;
#pragma unroll
      for (int j = 0; j < 13; j++) mine = (v == j) ? ze[j] : mine;
      if (v < 13) sh.P[OFF_ZE + 16 * i + v] = mine;
    }
  }
  lsync();
  C1_MARK(0);

  // ---- condensation: lane v builds H[v][w] for w >= v into packed P, and its gradient g_v
  const bool real = v < n;
  float gv;
  {
    const int kv = real ? sh.varblk[v] : 0;
    const int cv = real ? sh.varcol[v] : 0;
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = real ? sh.u.BdtT[cv][j] : 0.f;
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.P[OFF_ZE + 16 * kv + j];
      gv = real ? 2.f * dot13(b, zk) : 0.f;  // qg = 2 B_qp' S (A_qp x0 + Q_qp f - X_d)
    }
    lsync();  // every ZE read is issued before P is overwritten
    const int myrow = G::tri(v);
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      // z_i = S Adt^{i-kv} b_v + Adt' z_{i+1}  (the S term only for i >= kv)
      const bool act = real && (i >= kv);
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = act ? fmaf(k2, u2[j], fmaf(k, u1[j], b[j])) : 0.f;
      recur(md, wts, gk, z);
      asm volatile("" ::: "memory");  // the Bdt column loads stay inside the step
      const int wb = __builtin_amdgcn_readfirstlane(sh.blkbase[i]);
      step_columns(sh.u.BdtT, step_mask(msk0, msk1, i), wb, z, [&](int w, float val) {
        if (w == v) val += P.alpha2;  // qH = 2 (B'SB + alpha I), SolverMPC.cpp:806
        if (act && w >= v) sh.P[myrow + w] = val;
      });
    }
  }
  lsync();
  C1_MARK(1);

  // ---- row v of H into registers (full symmetric; identity padding for v >= n) ----------
  float slot[NV + 1];
  {
    const int vv = (v < NV) ? v : 0;  // lanes without a row read row 0 (and keep a zero row)
    const int myrow = G::tri(vv);
    static_for<0, NV>([&](auto C) {
      constexpr int c = decltype(C)::value;
      const int addr = (c >= vv) ? myrow + c : G::tri(c) + vv;
      const float x = sh.P[addr];
      slot[c] = (real && c < n) ? x : ((c == v) ? 1.f : 0.f);
      if ((c & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
    slot[NV] = gv;
  }
  lsync();

  // ---- bordered Cholesky [H | g]: raw column k = slot[k] of every lane -> P row k ----------
  // Look-ahead: step k publishes column k+1 (and takes its pivot d_{k+1} and border g_{k+1})
  // as soon as the sweep chunk holding slot[k+1] is updated, so nothing of step k+1's setup
  // waits on the LDS. The broadcast of column k to every lane is split between two paths that
  // run concurrently: CMPC_C1_RL of every 4 sweep chunks take it by v_readlane into SGPRs (FMA
  // with an SGPR operand, VALU only), the others by ds_read_b128 broadcasts of the stored
  // column (the LDS delivers 4 B per lane per cycle; with every chunk on it the sweep is LDS
  // bound). The stored columns also feed J = L^-T below.
  int status = CMPC_OK;
  float my_inv = 1.f;
#if CMPC_C1_CHOL2
  // Two pivots per step (k even, k+1): one rank-2 sweep over the raw column k and column k+1
  // as it is after step k,
  //   slot[c] += a0 P_k[c] + a1 P_k+1[c]  (c >= k+2),  a0 = -H[v][k] / d_k,  a1 = -s1 / d_k+1,
  //   s1 = H[v][k+1] - beta H[v][k],  beta = H[k+1][k] / d_k,  d_k+1 = H[k+1][k+1] - beta H[k+1][k]
  // so the 60 serial steps (pivot, broadcast, LDS round trip) become 30 with the same FMA count.
  // Look-ahead: as soon as the sweep chunk holding columns k+2, k+3 is updated, the step takes
  // their pivot data by readlane, forms the next step's beta / d / 1/sqrt(d), and publishes
  // column k+2 and the corrected column k+3; so the next step starts on its sweep at once. The
  // stored columns (raw even, corrected odd) are what J = L^-T needs. Odd n: the last step's
  // second pivot is the identity padding row (H[n][n] = 1, no coupling).
  float i0n = 1.f, betan = 0.f, i1n = 1.f, g0n = 0.f, g1n = 0.f;
  // pivot data of the step at columns (j, j+1) from the current rows, and the publish of both
  // columns (lanes >= the columns' chunk start)
  auto look = [&](auto JJ) {
    constexpr int j = decltype(JJ)::value, j1 = j + 1;
    constexpr int cj = j & ~3, cj1 = j1 & ~3;
    if constexpr (j1 < NV) {  // (also instantiated, never called, past the last step)
    float d0 = rl(slot[j], j);
    const float h10 = rl(slot[j], j1);
    if (!(d0 > 0.f)) { status = CMPC_NOT_PD; d0 = 1e-30f; }
    i0n = __builtin_amdgcn_rsqf(d0);  // d is a normal positive pivot
    betan = h10 * (i0n * i0n);
    float d1 = fmaf(-h10, betan, rl(slot[j1], j1));
    if (!(d1 > 0.f)) { status = CMPC_NOT_PD; d1 = 1e-30f; }
    i1n = __builtin_amdgcn_rsqf(d1);
    g0n = rl(slot[NV], j);
    g1n = fmaf(-betan, g0n, rl(slot[NV], j1));  // border of row j+1 after step j
    const float s1 = fmaf(-slot[j], betan, slot[j1]);
#if CMPC_C1_FUSEDJ
    // the factor's columns themselves, negated: P'_j = -L[:, j] = -slot[j] / sqrt(d_j) (and the
    // corrected column j+1 likewise), so the sweep and the left-looking J both read them as they are
    g0n = -g0n * i0n;
    g1n = -g1n * i1n;
    if (v >= cj && v < NV) sh.P[G::prow(j) + v - cj] = (v >= j) ? -slot[j] * i0n : 0.f;
    if (v >= cj1 && v < NV) sh.P[G::prow(j1) + v - cj1] = (v >= j1) ? -s1 * i1n : 0.f;
#else
    if (v >= cj && v < NV) sh.P[G::prow(j) + v - cj] = (v >= j) ? slot[j] : 0.f;
    if (v >= cj1 && v < NV) sh.P[G::prow(j1) + v - cj1] = (v >= j1) ? s1 : 0.f;
#endif
    lsync();
    }
  };
  if (n > 0) look(std::integral_constant<int, 0>{});
  float jc2 = 0.f, jc3 = 0.f;  // (CMPC_C1_FUSEDJ 2) rows k+2, k+3 of J's sums, carried one pair step
  (void)jc2; (void)jc3;
  // (CMPC_C1_XUNC) x = -J y accumulated as J's entries are solved: y_k = -g0 of pair step k (the
  // border of row k after the pivots before it, scaled by -1/sqrt(d_k) in look)
  float xunc = 0.f;
  (void)xunc;
  static_for<0, NV / 2>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value;
    constexpr int k1 = k + 1, k2 = k + 2;
    constexpr int c0 = k & ~3, c1 = k1 & ~3, c2 = k2 & ~3;
    constexpr int rk = G::prow(k), rk1 = G::prow(k1);
    if (k < n) {
      const float i0 = i0n, beta = betan, i1 = i1n, g0 = g0n, g1 = g1n;
#if CMPC_C1_FUSEDJ
      if (v == k) my_inv = i0;
      if (v == k1) my_inv = i1;
      const float s0 = slot[k];
      const float s1 = fmaf(-s0, beta, slot[k1]);
      // row v of L in columns k, k+1 (the sweep adds l_vk P'_k + l_vk+1 P'_k+1, P' = -L)
      const float a0 = (v > k) ? s0 * i0 : 0.f;
      const float a1 = (v > k1) ? s1 * i1 : 0.f;
#else
      if (v == k) { my_inv = i0; sh.u.ibuf[k] = i0; }
      if (v == k1) { my_inv = i1; sh.u.ibuf[k1] = i1; }
      const float s0 = slot[k];
      const float s1 = fmaf(-s0, beta, slot[k1]);
      const float a0 = (v > k) ? -s0 * (i0 * i0) : 0.f;
      const float a1 = (v > k1) ? -s1 * (i1 * i1) : 0.f;
#endif
      slot[NV] = fmaf(a1, g1, fmaf(a0, g0, slot[NV]));
      static_for<c2 / 4, NV / 4>([&](auto JC) {
        constexpr int c = 4 * decltype(JC)::value;
        const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
        axpy4(a0, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        if constexpr (k2 < NV && c == c2) {
          if (k2 < n) look(std::integral_constant<int, k2>{});  // columns k+2, k+3 are final
        }
        CMPC_SWEEP_FENCE(c);
      });
#if CMPC_C1_FUSEDJ == 2
      // J = L^-T, left-looking, four rows per 16-B read: at k = 0 mod 4 the sums of rows k..k+3
      // over every finished column j < k (one ds_read_b128 broadcast of P'_j[k..k+3] per column,
      // four columns per group, the next group's loads issued before this group's FMAs, two
      // accumulators per row);
      // rows k, k+1 are finished here, rows k+2, k+3 carry to the next pair step, which adds the
      // terms of columns k, k+1 (two 8-B reads)
      if constexpr ((k & 3) == 0) {
        f2v t0 = {(v == k) ? 1.f : 0.f, 0.f}, t1 = {(v == k1) ? 1.f : 0.f, 0.f};
        f2v t2 = {(v == k + 2) ? 1.f : 0.f, 0.f}, t3 = {(v == k + 3) ? 1.f : 0.f, 0.f};
#if CMPC_C1_JPIPE
        // loads of the next column group issued before this group's FMAs (one group ahead)
        piped_sweep<0, k, 1>(
            [&](auto C) {
              constexpr int q = decltype(C)::value;  // columns q .. q+3 (4 | k)
              return F4x4{*reinterpret_cast<const float4*>(&sh.P[G::prow(q) + k - q]),
                          *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 1) + k - q]),
                          *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 2) + k - q]),
                          *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 3) + k - q])};
            },
            [&](auto C, F4x4 l) {
              constexpr int q = decltype(C)::value;
              const float4 la = l.a, lb = l.b, lc = l.c, ld = l.d;
#else
        static_for<0, k / 4>([&](auto QC) {
          constexpr int q = 4 * decltype(QC)::value;  // columns q .. q+3 (4 | k)
          const float4 la = *reinterpret_cast<const float4*>(&sh.P[G::prow(q) + k - q]);
          const float4 lb = *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 1) + k - q]);
          const float4 lc = *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 2) + k - q]);
          const float4 ld = *reinterpret_cast<const float4*>(&sh.P[G::prow(q + 3) + k - q]);
#endif
          t0.x = fmaf(slot[q], la.x, t0.x); t1.x = fmaf(slot[q], la.y, t1.x);
          t2.x = fmaf(slot[q], la.z, t2.x); t3.x = fmaf(slot[q], la.w, t3.x);
          t0.y = fmaf(slot[q + 1], lb.x, t0.y); t1.y = fmaf(slot[q + 1], lb.y, t1.y);
          t2.y = fmaf(slot[q + 1], lb.z, t2.y); t3.y = fmaf(slot[q + 1], lb.w, t3.y);
          t0.x = fmaf(slot[q + 2], lc.x, t0.x); t1.x = fmaf(slot[q + 2], lc.y, t1.x);
          t2.x = fmaf(slot[q + 2], lc.z, t2.x); t3.x = fmaf(slot[q + 2], lc.w, t3.x);
          t0.y = fmaf(slot[q + 3], ld.x, t0.y); t1.y = fmaf(slot[q + 3], ld.y, t1.y);
          t2.y = fmaf(slot[q + 3], ld.z, t2.y); t3.y = fmaf(slot[q + 3], ld.w, t3.y);
#if CMPC_C1_JPIPE
            });
#else
          __builtin_amdgcn_sched_barrier(0);
        });
#endif
        const float hk = sh.P[G::prow(k) + k1 - (k & ~3)];  // -L[k+1][k]
        const float xk = (t0.x + t0.y) * i0;
        slot[k] = xk;
        slot[k1] = fmaf(xk, hk, t1.x + t1.y) * i1;
#if CMPC_C1_XUNC
        xunc = fmaf(slot[k1], g1, fmaf(xk, g0, xunc));
#endif
        jc2 = t2.x + t2.y;
        jc3 = t3.x + t3.y;
        asm volatile("" : "+v"(jc2), "+v"(jc3));
      } else {
        constexpr int km = k - 2;  // the columns of the pair step before (k - 2 = 0 mod 4)
        const float2 l0 = *reinterpret_cast<const float2*>(&sh.P[G::prow(km) + k - (km & ~3)]);
        const float2 l1 = *reinterpret_cast<const float2*>(&sh.P[G::prow(km + 1) + k - (km & ~3)]);
        const float hk = sh.P[G::prow(k) + k1 - (k & ~3)];
        const float e0 = fmaf(slot[km + 1], l1.x, fmaf(slot[km], l0.x, jc2));
        const float e1 = fmaf(slot[km + 1], l1.y, fmaf(slot[km], l0.y, jc3));
        const float xk = e0 * i0;
        slot[k] = xk;
        slot[k1] = fmaf(xk, hk, e1) * i1;
#if CMPC_C1_XUNC
        xunc = fmaf(slot[k1], g1, fmaf(xk, g0, xunc));
#endif
      }
#elif CMPC_C1_FUSEDJ
      // J = L^-T, left-looking: lane v solves L x = e_v, x_k = (d_vk - sum_{j<k} L[k][j] x_j) / L[k][k];
      // x_j (j < k) sit in the registers of the factor's finished columns, L[k][j], L[k+1][j] are
      // one 8-B broadcast of the stored column j (k even, rows start 16-B aligned), two interleaved
      // accumulators per row keep the FMA chains short. Every column of the factor is thus read
      // once more here instead of in a separate pass of 30 serial steps after the factorisation.
      {
        float e0 = (v == k) ? 1.f : 0.f, e1 = (v == k1) ? 1.f : 0.f, o0 = 0.f, o1 = 0.f;
        static_for<0, k>([&](auto JJ) {
          constexpr int j = decltype(JJ)::value;
          const float2 lj = *reinterpret_cast<const float2*>(&sh.P[G::prow(j) + k - (j & ~3)]);
          if constexpr ((j & 1) == 0) {
            e0 = fmaf(slot[j], lj.x, e0);
            e1 = fmaf(slot[j], lj.y, e1);
          } else {
            o0 = fmaf(slot[j], lj.x, o0);
            o1 = fmaf(slot[j], lj.y, o1);
          }
          if constexpr ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
        const float hk = sh.P[G::prow(k) + k1 - (k & ~3)];  // -L[k+1][k]
        const float xk = (e0 + o0) * i0;
        slot[k] = xk;
        slot[k1] = fmaf(xk, hk, e1 + o1) * i1;
      }
#endif
      pin(slot);
    }
  });
#else
  float dnext = 1.f, gnext = 0.f;
  if (n > 0) {
    if (v < NV) sh.P[G::prow(0) + v] = slot[0];
    dnext = rl(slot[0], 0);
    gnext = rl(slot[NV], 0);
    lsync();
  }
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int c0 = k & ~3;
    constexpr int rk = G::prow(k);
    constexpr int k1 = k + 1;
    constexpr int c1 = k1 & ~3;
    if (k < n) {
      float d = dnext;
      const float gk = gnext;
      if (!(d > 0.f)) { status = CMPC_NOT_PD; d = 1e-30f; }
      const float inv = __builtin_amdgcn_rsqf(d);  // d is a normal positive pivot
      if (v == k) { my_inv = inv; sh.u.ibuf[k] = inv; }
      const float colk = slot[k];  // lane c holds the raw column entry of row c
      const float a = (v > k) ? -colk * (inv * inv) : 0.f;
      slot[NV] = fmaf(a, gk, slot[NV]);
      static_for<c0 / 4, NV / 4>([&](auto JC) {
        constexpr int c = 4 * decltype(JC)::value;
        if constexpr (((c / 4) & 3) < CMPC_C1_RL) {
          // four readlanes into distinct SGPRs ahead of the four FMAs: a readlane's SGPR
          // result needs two wait states before a VALU may read it
          float s4[4];
          static_for<0, 4>([&](auto EC) {
            constexpr int cc = c + decltype(EC)::value;
            s4[EC] = (cc >= k) ? rl(colk, cc) : 0.f;
          });
          asm volatile("" : "+s"(s4[0]), "+s"(s4[1]), "+s"(s4[2]), "+s"(s4[3]));
          static_for<0, 4>([&](auto EC) {
            constexpr int cc = c + decltype(EC)::value;
            if constexpr (cc >= k) slot[cc] = fmaf(a, s4[EC], slot[cc]);
          });
        } else {
          const float4 r4 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
          axpy4(a, r4, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        }
        if constexpr (k1 < NV && c == c1) {
          if (k1 < n) {  // publish column k+1 (final after this chunk)
            constexpr int rk1 = G::prow(k1);
            if (v >= c1 && v < NV) sh.P[rk1 + v - c1] = (v >= k1) ? slot[k1] : 0.f;
            dnext = rl(slot[k1], k1);
            gnext = rl(slot[NV], k1);
            lsync();
          }
        }
        CMPC_SWEEP_FENCE(c);
      });
      pin(slot);
    }
  });
#endif
  const float yv = (v < n) ? slot[NV] * my_inv : 0.f;  // L y = g
  lsync();
  C1_MARK(2);

  // ---- J = L^-T: lane v solves L x = e_v (column v of L^-1 = row v of J) -----------------
#if CMPC_C1_CHOL2 && CMPC_C1_FUSEDJ
  // done inside the factorisation above; the columns past n are the identity rows' e_v already
#else
  static_for<0, NV>([&](auto C) {
    constexpr int c = decltype(C)::value;
    slot[c] = (c == v) ? 1.f : 0.f;
  });
#endif
#if CMPC_C1_CHOL2 && CMPC_C1_FUSEDJ
#elif CMPC_C1_CHOL2
  // two columns per step, as the factorisation: x_k, then x_k+1 after column k's term, then one
  // rank-2 sweep over the stored columns k, k+1 (the odd-n padding column is the identity)
  static_for<0, NV / 2>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value;
    constexpr int k1 = k + 1, c2 = (k + 2) & ~3;
    constexpr int c0 = k & ~3, c1 = k1 & ~3;
    constexpr int rk = G::prow(k), rk1 = G::prow(k1);
    if (k < n) {  // P and ibuf are read-only here: no per-step LDS ordering needed
      const float i0 = sh.u.ibuf[k], i1 = sh.u.ibuf[k1];
      const float h = sh.P[rk + k1 - c0];  // L[k+1][k] sqrt(d_k)
      const float x0 = slot[k] * i0;
      const float x1 = fmaf(-h * i0, x0, slot[k1]) * i1;
      const float a0 = -x0 * i0, a1 = -x1 * i1;
#pragma unroll
      for (int c = c2; c < NV; c += 4) {
        const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
        axpy4(a0, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        CMPC_SWEEP_FENCE(c);
      }
      slot[k] = x0;
      slot[k1] = x1;
      pin(slot);
    }
  });
#else
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int c0 = k & ~3;
    constexpr int rk = G::prow(k);
    if (k < n) {  // P and ibuf are read-only here: no per-step LDS ordering needed
      const float inv = sh.u.ibuf[k];
      const float xk = slot[k] * inv;
      const float a = -xk * inv;
#pragma unroll
      for (int c = c0; c < NV; c += 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        axpy4(a, r4, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        CMPC_SWEEP_FENCE(c);
      }
      slot[k] = xk;
      pin(slot);
    }
  });
#endif

  C1_MARK(3);
  // ---- unconstrained minimiser x = -J y ----------------------------------------------------
#if CMPC_C1_FUSEDJ == 2 && CMPC_C1_XUNC
  (void)yv;
  float xv = (v < n) ? xunc : 0.f;  // accumulated in the factorisation's steps
#else
  sh.vbuf()[v] = yv;
  lsync();
  f2v xacc = {0.f, 0.f};
  piped_sweep<0, NV, C1_PIPE_GRP>(
      [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
      [&](auto C, float4 y4) {
        constexpr int c = decltype(C)::value;
        dot4(xacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], y4);
      });
  float xv = (v < n) ? -(xacc.x + xacc.y) : 0.f;
  lsync();
#endif

  // ---- Goldfarb-Idnani dual active set on the friction pyramids -----------------------------
  // One flat loop, one active-set step per trip. The QP's triangular factor R (q x q) is kept
  // explicitly, packed by columns in P (the L rows are dead once J is formed): back substitution
  // and the re-triangularisation after a drop are readlane chains over LDS. The J rows in
  // registers see the same straight-line code on every trip — a Householder reflection (the
  // add step; beta = 0 on a drop) and an ascending Givens chain (the drop step; identity
  // rotations otherwise) — so their registers carry through the loop without copies.
  const float mui = P.mu_inv;
  const float fnorm = rsqrtf(mui * mui + 1.f);
  int q = 0;
  int iters = 0;
  float u_reg = 0.f;   // lane j < q: dual of active constraint j
  int act_reg = 0;     // lane j < q: id of active constraint j
  int p = -1;          // constraint being added (-1: pick the most violated one)
  Cons cp{};
  float up = 0.f;
  bool rinv_ok = true;  // R^-1 kept beside R (wave-uniform)
  lsync();
  if (status == CMPC_OK) {
    for (;;) {
      pin(slot);
      const int v = tid_opq();  // re-materialised: keeps per-lane addresses out of the preheader
#ifdef CMPC_PHASE_PROF
      t_sub = clock64();
#endif
      if (p < 0) {
        // foot-step v's forces from lanes 3v .. 3v+2 by ds_bpermute (no LDS store + reload)
        const float fx = __shfl(xv, 3 * v), fy = __shfl(xv, 3 * v + 1), fz = __shfl(xv, 3 * v + 2);
        float best = 0.f;
        int bid = 0x7fffffff;
        if (v < nfs) {
          const unsigned fm = sh.cmask[v];
          float sl[6];
          sl[0] = (mui * fx + fz) * fnorm;
          sl[1] = (-mui * fx + fz) * fnorm;
          sl[2] = (mui * fy + fz) * fnorm;
          sl[3] = (-mui * fy + fz) * fnorm;
          sl[4] = fz;
          sl[5] = sh.sub[v] - fz;
#pragma unroll
          for (int t = 0; t < 6; t++)
            if (!((fm >> t) & 1u) && sl[t] < best) { best = sl[t]; bid = 6 * v + t; }
        }
        const float xmax = wave_max(fabsf(xv));
        wave_argmin(best, bid);
        const float tol = 1e-5f * fmaxf(1.f, xmax);
        if (bid == 0x7fffffff || best >= -tol) break;
        p = __builtin_amdgcn_readfirstlane(bid);
        cp = decode_cons(p, mui, sh.sub[p / 6]);
        up = 0.f;
      }
      C1_SUB(0);
      if (++iters > P.max_iter + 2 * n) { status = CMPC_MAX_ITER; break; }
#if CMPC_TRIP_PRIO_AT > 0
      // a long solve: issue ahead of the other waves on this SIMD (shorter makespan tail)
      if (iters == CMPC_TRIP_PRIO_AT) __builtin_amdgcn_s_setprio(CMPC_C1_TRIP_PRIO);
#endif
      // d = J' n+ : rows ia, iz of J through LDS (dword stores: wide stores would tie the row
      // registers into tuples)
      if (v == cp.ia || v == cp.iz) {  // both rows in one pass (two lanes per store)
        // lane iz's row 16 words past bufB's start (into cs, written only later in a drop trip):
        // lanes ia and iz, neighbours in one half-wave, then store to different banks
        const int boff = (v == cp.iz) ? NL + 16 : 0;
#pragma unroll
        for (int c = 0; c < NV; c++) {
          sh.u.gi.bufA[boff + c] = slot[c];
          if ((c & 15) == 15) __builtin_amdgcn_sched_barrier(0);
        }
      }
      lsync();
      const float dv = (cp.ia != cp.iz) ? fmaf(cp.ca, sh.u.gi.bufA[v], cp.cb * sh.u.gi.bufB[16 + v])
                                        : cp.cb * sh.u.gi.bufB[16 + v];
      const float dm = (v >= q && v < n) ? dv : 0.f;
      sh.vbuf()[v] = dm;
      lsync();
      // z = J2 d2 (primal step direction), zn = |d2|^2 = z' n+, dn = |d|^2
      f2v zacc = {0.f, 0.f}, nacc = {0.f, 0.f};
      piped_sweep<0, NV, C1_PIPE_GRP>(
          [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
          [&](auto C, float4 m4) {
            constexpr int c = decltype(C)::value;
            C1_DOT(zacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], m4);
            C1_DOT(nacc, m4.x, m4.y, m4.z, m4.w, m4);
          });
      float zv = zacc.x + zacc.y, zn = nacc.x + nacc.y;
      // materialise both sums here: otherwise the FMAs sink below the back substitution loop
      // and the NV loaded values of vbuf stay live across it (158 VGPRs, three waves per SIMD)
      asm volatile("" : "+v"(zv), "+v"(zn));
      const float dn = wave_sum((v < n) ? dv * dv : 0.f);
      C1_SUB(1);
      // r = R^-1 d1 (lane i ends with r_i). While R^-1 is kept (every step so far an add, q <=
      // QI) it is a matvec over its packed columns: no dependent chain, four columns per trip.
      // Otherwise a back substitution over the packed columns of R, software-pipelined (the LDS
      // reads of step i - 1 are issued before step i's readlane / divide / FMA chain).
      float acc = dv, r_reg = 0.f;
      if (rinv_ok) {
        using S = SharedC1<NV>;
        float a0 = 0.f, a1 = 0.f;
        int j = 0;
        for (; j + 4 <= q; j += 4) {
          const float x0 = sh.P[S::RB + rcol(j) + v], x1 = sh.P[S::RB + rcol(j + 1) + v];
          const float x2 = sh.P[S::RB + rcol(j + 2) + v], x3 = sh.P[S::RB + rcol(j + 3) + v];
          a0 = fmaf((v <= j) ? x0 : 0.f, rl(dv, j), a0);
          a1 = fmaf((v <= j + 1) ? x1 : 0.f, rl(dv, j + 1), a1);
          a0 = fmaf((v <= j + 2) ? x2 : 0.f, rl(dv, j + 2), a0);
          a1 = fmaf((v <= j + 3) ? x3 : 0.f, rl(dv, j + 3), a1);
        }
        for (; j < q; j++) {
          const float x0 = sh.P[S::RB + rcol(j) + v];
          a0 = fmaf((v <= j) ? x0 : 0.f, rl(dv, j), a0);
        }
        r_reg = (v < q) ? a0 + a1 : 0.f;
      } else {
        float pd = 1.f, pv = 0.f;
        if (q > 0) {
          pd = sh.P[rcol(q - 1) + q - 1];
          pv = sh.P[rcol(q - 1) + v];
        }
        for (int i = q - 1; i >= 0; i--) {
          float pd_n = 1.f, pv_n = 0.f;
          if (i > 0) {
            pd_n = sh.P[rcol(i - 1) + i - 1];
            pv_n = sh.P[rcol(i - 1) + v];
          }
          const float ri = fdiv(rl(acc, i), pd);
          if (v < i) acc = fmaf(-pv, ri, acc);
          r_reg = (v == i) ? ri : r_reg;
          pd = pd_n;
          pv = pv_n;
        }
      }
      // partial (dual) step t1, full (primal) step t2
      float t1 = kBigF;
      int kk = 0x7fffffff;
      if (v < q && r_reg > 0.f) { t1 = fmaxf(fdiv(u_reg, r_reg), 0.f); kk = v; }
      wave_argmin(t1, kk);
      const float spv = fmaf(cp.ca, rl(xv, cp.ia), fmaf(cp.cb, rl(xv, cp.iz), -cp.bp));
      const bool zero_step = !(zn > 1e-9f * dn);
      const float t2 = zero_step ? kBigF : -fdiv(spv, zn);
      const float t = fminf(t1, t2);
      if (t >= kBigF) { status = CMPC_INFEASIBLE; break; }
      if (v < q) u_reg = fmaf(-t, r_reg, u_reg);
      up += t;
      if (!zero_step) xv = fmaf(t, zv, xv);
      C1_SUB(2);
      const bool add = !zero_step && t2 <= t1;
      const bool add_u = __builtin_amdgcn_readfirstlane((int)add) != 0;
      float beta = 0.f;
      if (add) {
        // ---- add p: the Householder reflection I - beta w w' on columns q..n-1 maps
        // d[q..n-1] to -sgn(d_q) |d[q..n-1]| e_q; R gains the column (d[0..q-1], -sgn ts)
        const float ts = sqrtf(zn);
        const float dq = rl(dv, q);
        const float sgn = (dq >= 0.f) ? 1.f : -1.f;
        beta = fast_rcp(ts * (ts + fabsf(dq)));  // 2 / (w'w)
        sh.vbuf()[v] = (v == q) ? dq + sgn * ts : dm;
        const int offq = rcol(q);
        if (v < q) sh.P[offq + v] = dv;
        if (v == q) {
          sh.P[offq + q] = -sgn * ts;
          u_reg = up;
          act_reg = p;
        }
        // R^-1 gains the column (-r / rho, 1 / rho), rho = R's new diagonal: [R d1; 0 rho]^-1
        if (rinv_ok) {
          if (q < SharedC1<NV>::QI) {
            const float irho = 1.f / (-sgn * ts);
            const int offi = SharedC1<NV>::RB + rcol(q);
            if (v < q) sh.P[offi + v] = -r_reg * irho;
            if (v == q) sh.P[offi + q] = irho;
          } else {
            rinv_ok = false;
          }
        }
        if (v == 0) sh.cmask[p / 6] |= (unsigned char)(1u << (p % 6));
      } else {
        // ---- drop active constraint kk: shift positions kk+1..q-1 down, remove column kk of
        // R and re-triangularise rows kk..q-1 (lane c rebuilds column c of R in place: every
        // read of an old entry precedes, in this wavefront's LDS order, the write reusing it)
        sh.vbuf()[v] = 0.f;
        const int k = __builtin_amdgcn_readfirstlane(kk);
        const int ak = rli(act_reg, k);
        if (v == 0) sh.cmask[ak / 6] &= (unsigned char)~(1u << (ak % 6));
        const int a_nx = lane_next_i(act_reg, act_reg);
        const float u_nx = lane_next(u_reg, u_reg);
        if (v >= k && v < q - 1) { act_reg = a_nx; u_reg = u_nx; }
        if (v < k || v > q - 2) *reinterpret_cast<float2*>(&sh.u.gi.cs[2 * v]) = make_float2(1.f, 0.f);
        const bool in_c = v >= k && v <= q - 2;
        float top = in_c ? sh.P[rcol(v + 1) + k] : 0.f;
        lsync();
        for (int r = 0; r < k; r++) {
          const float x = in_c ? sh.P[rcol(v + 1) + r] : 0.f;
          lsync();
          if (in_c) sh.P[rcol(v) + r] = x;
          lsync();
        }
        for (int j = k; j <= q - 2; j++) {
          const bool on = in_c && v >= j;
          const float bot = on ? sh.P[rcol(v + 1) + j + 1] : 0.f;
          lsync();
          const float a0 = rl(top, j), b0 = rl(bot, j);
          const float h = sqrtf(a0 * a0 + b0 * b0);
          float cc = 1.f, sn = 0.f;
          if (h > 0.f) { const float ih = fast_rcp(h); cc = a0 * ih; sn = b0 * ih; }
          if (on) {
            sh.P[rcol(v) + j] = fmaf(cc, top, sn * bot);
            top = fmaf(-sn, top, cc * bot);
          }
          if (v == 0) *reinterpret_cast<float2*>(&sh.u.gi.cs[2 * j]) = make_float2(cc, sn);
          lsync();
        }
        // R^-1 through the drop. With H = R E (column k removed) and R' = G' H restricted to its
        // first q - 1 rows (the Givens chain above), E' R^-1 is a left inverse of H, so
        //   R'^-1 = E' R^-1 G[:, 0:q-1]:
        // R^-1 without row k, the same rotations on its columns as on J's (j = k .. q-2), the
        // last column dropped. Lane i streams its row through the chain with one carried value
        // (rows i > k move up one; their entries left of column i - 1 are zero and stay so).
        if (rinv_ok) {
          using S = SharedC1<NV>;
          const int i = v;
          const bool live = i < q && i != k;
          const int i2 = (i > k) ? i - 1 : i;
          int j = (i > k) ? i - 1 : k;  // first rotation that touches row i
          float carry = (live && j >= i) ? sh.P[S::RB + rcol(j) + i] : 0.f;
          for (int jj = k; jj <= q - 2; jj++) {
            const float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * jj]);
            const float b = (live && jj >= j && jj + 1 >= i) ? sh.P[S::RB + rcol(jj + 1) + i] : 0.f;
            lsync();
            if (live && jj >= j) {
              sh.P[S::RB + rcol(jj) + i2] = fmaf(cs2.x, carry, cs2.y * b);
              carry = fmaf(-cs2.y, carry, cs2.x * b);
            }
          }
        }
      }
      lsync();
      C1_SUB(3);
      // The reflection runs on every trip (beta = 0 on a drop: a uniform branch around it costs 27
      // spilled VGPRs); the Givens chain only on a drop (add_u is wave-uniform; the branch leaves
      // the register allocation unchanged, same instruction count).
      {
        // J <- J (I - beta w w'): tw = J_v . w, J_v -= beta tw w  (no-op on a drop: beta = 0)
        f2v tacc = {0.f, 0.f};
        piped_sweep<0, NV, C1_PIPE_GRP>(
            [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
            [&](auto C, float4 w4) {
              constexpr int c = decltype(C)::value;
              C1_DOT(tacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], w4);
            });
        const float bt = -beta * (tacc.x + tacc.y);
        // re-read w from LDS: without this point the compiler keeps all NV values of the first
        // sweep's loads live for the second (a whole row of extra VGPRs)
        asm volatile("" ::: "memory");
        piped_sweep<0, NV, C1_PIPE_GRP>(
            [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
            [&](auto C, float4 w4) {
              constexpr int c = decltype(C)::value;
              axpy4(bt, w4, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
            });
      }
      C1_SUB(4);
      if (!add_u) {
        // J columns (j, j+1) <- Givens chain j = 0 .. NV-2 (drops only)
        static_for<0, NV - 1>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          const float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * j]);
          const float x0 = slot[j], x1 = slot[j + 1];
          slot[j] = fmaf(cs2.x, x0, cs2.y * x1);
          slot[j + 1] = fmaf(-cs2.y, x0, cs2.x * x1);
          if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
      }
      C1_SUB(5);
#ifdef CMPC_PHASE_PROF
      ph[14] += add ? 0ull : 1ull;
#endif
      if (add) {
        q++;
        p = -1;
      } else {
        q--;
      }
      lsync();
    }
  }

  C1_MARK(4);
  // ---- scatter (q_soln layout 12 k + 3 leg + axis, swing -> 0) staged in LDS, coalesced out
  const bool ok = (status == CMPC_OK);
  for (int t = v; t < 12 * N; t += 64) sh.P[t] = 0.f;
  lsync();
  if (ok && v < n) sh.P[12 * sh.varblk[v] + sh.varcol[v]] = xv;
  lsync();
  for (int t = 4 * v; t < P.out_cols; t += 256)  // (the leading steps kept, 12 N by default)
    *reinterpret_cast<float4*>(&fout[t]) = *reinterpret_cast<const float4*>(&sh.P[t]);
  if (v == 0) {
    st_out[0] = (uint8_t)status;
    if (it_out) it_out[0] = iters;
  }
#ifdef CMPC_PHASE_PROF
  C1_MARK(5);
  if (v == 0) {
    ph[6] = 1;
    ph[7] = (unsigned long long)iters;
#pragma unroll
    for (int i = 0; i < 16; i++) atomicAdd(&g_c1_phase[i], ph[i]);
  }
#endif
}

}  // namespace

template <int NV>
__global__ __launch_bounds__(64, NV == 60 ? CMPC_W1_WAVES_60 : CMPC_W1_WAVES_PER_EU) void cmpc_solve_c1_kernel(
    const float* __restrict__ recs, int batch, KParams P, float* __restrict__ forces,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, const int* __restrict__ in_list,
    const int* __restrict__ in_count, int* __restrict__ ovf_list, int* __restrict__ ovf_count) {
  // one instance per workgroup, no grid-stride loop: a loop around the solve would let LICM
  // hoist hundreds of lane-invariant addresses / masks out of it and spill them
  __shared__ SharedC1<NV> sh;
  int t = blockIdx.x;
  if (in_list) {  // list mode: workgroup i takes list entry i (surplus workgroups exit)
    if (t >= *in_count) return;
    t = in_list[t];
  } else if (t >= batch) {
    return;
  }
#ifdef CMPC_PLACE_PROF
  const unsigned long long t_start = wall_clock64();
  const unsigned hw_id = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const unsigned xcc_id = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
#endif
  solve_c1<NV>(recs + (size_t)t * P.rec_words, P, sh, forces + (size_t)t * P.out_cols, status + t,
               iters ? iters + t : nullptr, ovf_list, ovf_count, t);
#ifdef CMPC_PLACE_PROF
  const unsigned long long t_end = wall_clock64();
  if (threadIdx.x == 0 && t < kPlaceMax) {
    g_c1_place[4 * t + 0] = hw_id;
    g_c1_place[4 * t + 1] = xcc_id;
    g_c1_place[4 * t + 2] = (unsigned)t_start;
    g_c1_place[4 * t + 3] = (unsigned)t_end;
  }
#endif
}

hipError_t launch_class1(int nv, const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         int* ovf_list, int* ovf_count, int grid, hipStream_t stream) {
  if (grid <= 0) return hipSuccess;
  // CMPC_C1_DYN_LDS=<bytes> (diagnostic build only): extra dynamic LDS per workgroup, i.e. fewer class-1
  // workgroups per CU (placement / occupancy experiments)
  static const unsigned dyn = (unsigned)diag_knob("CMPC_C1_DYN_LDS", 0);
  if (nv == 60)
    hipLaunchKernelGGL(cmpc_solve_c1_kernel<60>, dim3(grid), dim3(64), dyn, stream, d_recs, batch, P,
                       d_forces, d_status, d_iters, in_list, in_count, ovf_list, ovf_count);
  else
    hipLaunchKernelGGL(cmpc_solve_c1_kernel<64>, dim3(grid), dim3(64), dyn, stream, d_recs, batch, P,
                       d_forces, d_status, d_iters, in_list, in_count, ovf_list, ovf_count);
  return hipGetLastError();
}

}  // namespace cmpc

#ifdef CMPC_PHASE_PROF
// cycles per stage summed over solved class-1 instances: prep, condensation, Cholesky, J,
// active set (incl. x = -J y), scatter; [6] instances, [7] active-set iterations. Resets.
extern "C" int cmpc_debug_phase_read(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c1_phase), sizeof(unsigned long long) * 16) != hipSuccess)
    return -1;
  unsigned long long z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_c1_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef CMPC_PLACE_PROF
// per instance [hw_id, xcc_id, start, end] of the last class-1 launches (instances < 65536)
extern "C" int cmpc_debug_place_read(unsigned int* out, int n) {
  if (n > kPlaceMax) n = kPlaceMax;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_c1_place), sizeof(unsigned int) * 4 * n) == hipSuccess ? 0 : -1;
}
#endif
