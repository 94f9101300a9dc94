// cmpc_tail.hip — one wavefront per instance for 64 < n <= 64 + T reduced force variables: the
// "tail class", built with T = 8 (n 66..72: four fifths of the random-contact instances above
// class 1 at N <= 10). The template also builds T = 16 (n <= 80), which measured no faster than the
// 80-column wide class it would replace (69 vs 68-70 ns per instance, 132 spilled VGPRs;
// profiles/r05_c) and is not instantiated.
//
// Same computation as cmpc_class1.hip — one call of the reference's solve_mpc()
// (be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-982): stance table + swing
// elimination (:859-894), model + closed-form c2qp, structured condensation of the reduced qH / qg
// (:806-814), bordered Cholesky, J = L^-T, the Goldfarb-Idnani dual active set in place of
// qpOASES QProblem::init (:955-969), scatter to q_soln (:970-982).
//
// MI355X mapping ("tail class"): class 1's one-wavefront layout, lane v owning row
// v of every working matrix in NV = 64 + T registers, plus T "tail" rows 64..NV-1 that have no
// lane of their own:
//   * the tail rows of H / L are the transposes of the lanes' registers 64..NV-1 (symmetry), so
//     the Cholesky's 64 main pivots sweep full NV-wide rows exactly as class 1 does; the tail
//     block H22 (T x T) rides along in T / (64/T) registers per lane (row 64 + lane / (64/T));
//   * the last T pivots factor the T x T Schur complement in lanes 0..T-1 (short rows);
//   * J's tail rows (T x NV) live in NV T / 64 registers per lane: lane l holds columns
//     [SW s, SW s + SW) of tail row l / (64/T), s = l % (64/T); their reductions stay inside a
//     quad / half-row of lanes (DPP), their Givens chains cross the segments at seams (DPP shifts);
//   * no s_barrier anywhere (one wave): the wide classes' 3-wave workgroups spent one per pivot
//     pair. Active-set positions stay in lanes (q <= 64); an instance whose active set would grow
//     past 64 positions is handed to the 80-column wide class (ovf list), which solves it afresh.
// Everything is fp32 (the reference condenses in fp32: common_types.h:14).
#include "cmpc_common.h"

#ifndef CMPC_TAIL_WAVES_PER_EU
#define CMPC_TAIL_WAVES_PER_EU 3
#endif
#ifndef CMPC_TRIP_PRIO_AT  // active-set trips after which a wave raises its priority (0: never)
#define CMPC_TRIP_PRIO_AT 0
#endif
#ifndef CMPC_TAIL_TRIP_PRIO
#define CMPC_TAIL_TRIP_PRIO 3
#endif
// the active set's row-long dot products as two interleaved FMA chains (A/B)
#ifndef CMPC_TAIL_DOT2
#define CMPC_TAIL_DOT2 0
#endif
#if CMPC_TAIL_DOT2
#define T_DOT dot4x2
#else
#define T_DOT dot4
#endif
#ifndef CMPC_TAIL_PRIO  // s_setprio of the tail classes' waves: issue ahead of the class-1 waves on their SIMDs
#define CMPC_TAIL_PRIO 1
#endif
#ifndef TAIL_PIPE_GRP
#define TAIL_PIPE_GRP 4
#endif

// Phase profiler (diagnostic builds only, -DCMPC_PHASE_PROF): lane 0 of every solved instance
// adds the s_memtime cycles of each stage to g_t_phase (scripts/phase_prof.py --tail)
#ifdef CMPC_PHASE_PROF
__device__ unsigned long long g_t_phase[16];
#define T_MARK(i)                               \
  do {                                          \
    const unsigned long long _n = clock64();    \
    ph[i] += _n - t_last;                       \
    t_last = _n;                                \
  } while (0)
#else
#define T_MARK(i) \
  do {            \
  } while (0)
#endif

namespace cmpc {
namespace {

constexpr int kTailRows = 8;  // T of the built kernel (NV = 72)

template <int T>
struct TGeo {
  static_assert(T == 8 || T == 16, "tail rows");
  static constexpr int NV = 64 + T;         // row width
  static constexpr int NG = NV / 4;
  static constexpr int PSZ = 4 * NG * NV - 8 * NG * (NG - 1);  // packed rows r: columns [r & ~3, NV)
  __host__ __device__ static constexpr int prow(int r) {
    return 4 * (r >> 2) * NV - 8 * (r >> 2) * ((r >> 2) - 1) + (r & 3) * (NV - 4 * (r >> 2));
  }
  // H's exchange after the condensation: plain packed upper triangle, (r, c >= r) at tri(r) + c
  __host__ __device__ static constexpr int tri(int r) { return r * NV - ((r * (r + 1)) >> 1); }
  static constexpr int LPR = 64 / T;        // lanes per tail row
  static constexpr int TQ = T / LPR;        // H22 columns per lane during the main pivots
  static constexpr int SW = NV / LPR;       // J tail-row columns per lane (a segment)
  static constexpr int MAXFS = (NV + 2) / 3;  // stance foot-steps
  static_assert(NV * (NV + 1) / 2 <= PSZ, "exchange fits P");
  static_assert(64 * 65 / 2 <= PSZ - NV, "R (q <= 64) below vbuf");
};

constexpr int T_OFF_E = 0;
constexpr int T_OFF_ZE = T_OFF_E + 16 * MAXN;
constexpr int T_OFF_REC = T_OFF_ZE + 16 * MAXN;

// R (upper triangular, q x q) packed by columns: R[i][j] at rcol(j) + i, i <= j
__device__ __forceinline__ int rcol(int j) { return (j * (j + 1)) >> 1; }

constexpr int tail_rinv_cols(int words) {
  int q = 0;
  while ((q + 1) * (q + 2) <= words) q++;
  return q;
}

template <int T>
struct SharedT {
  using G = TGeo<T>;
  static_assert(T_OFF_REC + CMPC_REC_WORDS(MAXN) <= G::PSZ, "prep scratch must fit in P");
  // vbuf (the broadcast vector: y, then the masked d / Householder vector) in P's last NV words
  __device__ __forceinline__ float* vbuf() { return &P[G::PSZ - G::NV]; }
  // R^-1 beside R (q <= QI, adds only), below vbuf; R's first QI columns stay below it
  static constexpr int QI = tail_rinv_cols(G::PSZ - G::NV);
  static constexpr int RB = G::PSZ - G::NV - QI * (QI + 1) / 2;
  static_assert(QI * (QI + 1) / 2 <= RB, "R and R^-1 side by side");
  float P[G::PSZ];
  union {
    float BdtT[12][16];        // prep + condensation
    struct {                   // Cholesky + J
      float ibuf[G::NV];       // 1 / sqrt(d_k)
      float bpair[G::NV / 2];  // beta of the pivot pair (k, k+1) (0 for the tail pivots)
      float h22[T * T];        // tail block exchange (row-major), then J22
      float gt[T];             // tail borders
    } ch;
    struct {                   // active set
      float bufA[G::NV], bufB[G::NV];  // published J rows ia, iz (bufA[NV + c] = bufB[c])
      float cs[2 * 64];        // Givens (c, s) per column pair (j <= 62: q <= 64)
      float xs[G::NV];         // x by reduced variable
    } gi;
  } u;
  float gtail[T];              // tail rows' gradient (condensation)
  float sub[G::MAXFS];
  int sfs[G::MAXFS];
  int blkbase[MAXN + 2];
  unsigned char varblk[G::NV], varcol[G::NV];
  unsigned char cmask[G::MAXFS];
};

__device__ __forceinline__ void tsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

template <int M>
__device__ __forceinline__ void tpin(float (&x)[M]) {
#pragma unroll
  for (int c = 0; c < M; c++) asm volatile("" : "+v"(x[c]));
}

#define CMPC_TSWEEP_FENCE(c)                                       \
  do {                                                             \
    if (((c) & 15) == 12) __builtin_amdgcn_sched_barrier(0);       \
  } while (0)

// sum over the LPR lanes of a tail row's group (uniform within the group)
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
  v += dppf<kDppQuadSwap1>(0.f, v);
  v += dppf<kDppQuadSwap2>(0.f, v);
  if constexpr (LPR == 8) v += dppf<kDppRowHalfMirror>(0.f, v);
  return v;
}

template <int T>
__device__ __forceinline__ void solve_t(const float* __restrict__ rec, const KParams& P,
                                        SharedT<T>& sh, float* __restrict__ fout,
                                        uint8_t* __restrict__ st_out, int32_t* __restrict__ it_out,
                                        int* __restrict__ ovf_list, int* __restrict__ ovf_count,
                                        int inst) {
  using G = TGeo<T>;
  constexpr int NV = G::NV, LPR = G::LPR, TQ = G::TQ, SW = G::SW;
  // opaque lane id / horizon: in the persistent form nothing derived from them is hoisted out of
  // the dequeue loop (and kept live, or spilled, across the whole solve)
  const int v = tid_opq();
  const int ti = v / LPR, ts = v % LPR;  // tail row / segment of this lane
  const int N = opaque(P.N);
#ifdef CMPC_PHASE_PROF
  unsigned long long ph[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_last = clock64();
#endif
  // ---- stage the record in LDS (one 16-B load per lane)
  {
    const float4* src = reinterpret_cast<const float4*>(rec);
    float4* dst = reinterpret_cast<float4*>(&sh.P[T_OFF_REC]);
    for (int t = v; t < (P.rec_words >> 2); t += 64) dst[t] = src[t];
  }
  tsync();
  const float* srec = &sh.P[T_OFF_REC];
  // ---- stance table + elimination (SolverMPC.cpp:869-894)
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(srec + CMPC_REC_HDR + 12 * N);
  int nfs = 0;
  unsigned long long msk0 = 0ull, msk1 = 0ull;
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
    if (f && nfs + pre < G::MAXFS) {
      sh.sfs[nfs + pre] = t;
      sh.sub[nfs + pre] = ub;
    }
    nfs += __popcll(m);
  }
  const int n = 3 * nfs;
  if (n > NV || n <= 64) {  // not this class's instance (classify routes exactly)
    if (v == 0) { st_out[0] = CMPC_BAD_INPUT; if (it_out) it_out[0] = 0; }
    return;
  }
  tsync();
  for (int t = v; t < NV; t += 64) {
    int kb = 0, kc = 0;
    if (t < n) {
      const int fs = sh.sfs[t / 3];
      kb = fs >> 2;
      kc = 3 * (fs & 3) + t % 3;
    }
    sh.varblk[t] = (unsigned char)kb;
    sh.varcol[t] = (unsigned char)kc;
  }
  if (v <= N) {
    const int b0 = 4 * v, b1 = 4 * v - 64;
    const unsigned long long lo = (b0 >= 64) ? msk0 : (msk0 & ((1ull << b0) - 1ull));
    const unsigned long long hi = (b1 <= 0) ? 0ull : (msk1 & ((1ull << b1) - 1ull));
    sh.blkbase[v] = 3 * (__popcll(lo) + __popcll(hi));
  }
  if (v < nfs) sh.cmask[v] = 0;
  Model md;
  make_model(srec, P.dt, md);
  make_bdt<64>(srec, md, v, sh.u.BdtT);
  tsync();
  if (v < N) {
    float e[13];
    state_error(srec, md, v, srec + CMPC_REC_HDR + 12 * v, e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.P[T_OFF_E + 16 * v + j] = e[j];
  }
  tsync();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  {
    float ze[13];
#pragma unroll
    for (int j = 0; j < 13; j++) ze[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      float e[13];
#pragma unroll
      for (int j = 0; j < 13; j++) e[j] = sh.P[T_OFF_E + 16 * i + j];
      recur(md, wts, e, ze);
      float mine = 0.f;
#pragma unroll
      for (int j = 0; j < 13; j++) mine = (v == j) ? ze[j] : mine;
      if (v < 13) sh.P[T_OFF_ZE + 16 * i + v] = mine;
    }
  }
  tsync();

  // ---- condensation: lane v builds H[v][w], w >= v, into the packed triangle (class 1's
  // recursion); lanes v < T then build the tail rows 64 + v over the last steps
  float gv;
  {
    const int kv = sh.varblk[v];
    const int cv = sh.varcol[v];
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = sh.u.BdtT[cv][j];
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.P[T_OFF_ZE + 16 * kv + j];
      gv = 2.f * dot13(b, zk);  // qg = 2 B_qp' S (A_qp x0 + Q_qp f - X_d)
      // the tail row 64 + v's gradient
      const bool tr = v < T && 64 + v < n;
      const int kt = tr ? sh.varblk[64 + v] : 0, ct = tr ? sh.varcol[64 + v] : 0;
      float bt[13], zt[13];
#pragma unroll
      for (int j = 0; j < 13; j++) {
        bt[j] = sh.u.BdtT[ct][j];
        zt[j] = sh.P[T_OFF_ZE + 16 * kt + j];
      }
      const float gtl = tr ? 2.f * dot13(bt, zt) : 0.f;
      if (v < T) sh.gtail[v] = gtl;
    }
    tsync();  // every ZE read is issued before P is overwritten
    const int myrow = G::tri(v);
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      const bool act = i >= kv;
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = act ? fmaf(k2, u2[j], fmaf(k, u1[j], b[j])) : 0.f;
      recur(md, wts, gk, z);
      asm volatile("" ::: "memory");
      const int wb = __builtin_amdgcn_readfirstlane(sh.blkbase[i]);
      step_columns(sh.u.BdtT, step_mask(msk0, msk1, i), wb, z, [&](int w, float val) {
        if (w == v) val += P.alpha2;  // qH = 2 (B'SB + alpha I), SolverMPC.cpp:806
        if (act && w >= v) sh.P[myrow + w] = val;
      });
    }
  }
  {
    // tail rows r = 64 + v (v < T): the same recursion over the steps that hold tail columns
    const int r = 64 + v;
    const bool real = v < T && r < n;
    const int kv = real ? sh.varblk[r] : 0;
    const int cv = real ? sh.varcol[r] : 0;
    const int k64 = __builtin_amdgcn_readfirstlane((int)sh.varblk[64]);
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = sh.u.BdtT[cv][j];
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    const int myrow = G::tri(real ? r : 64);
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    for (int i = N - 1; i >= k64; i--) {
      const bool act = real && i >= kv;
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = act ? fmaf(k2, u2[j], fmaf(k, u1[j], b[j])) : 0.f;
      recur(md, wts, gk, z);
      asm volatile("" ::: "memory");
      const int wb = __builtin_amdgcn_readfirstlane(sh.blkbase[i]);
      step_columns(sh.u.BdtT, step_mask(msk0, msk1, i), wb, z, [&](int w, float val) {
        if (w == r) val += P.alpha2;
        if (act && w >= r) sh.P[myrow + w] = val;
      });
    }
  }
  tsync();

  T_MARK(0);
  // ---- row v of H into registers; the tail block H22 into the T layout (lane: row 64 + ti,
  // columns TQ ts .. TQ ts + TQ - 1 of the block); identity padding past n
  float slot[NV + 1];
  {
    const int myrow = G::tri(v);
    static_for<0, NV>([&](auto C) {
      constexpr int c = decltype(C)::value;
      const int addr = (c >= v) ? myrow + c : G::tri(c) + v;
      const float x = sh.P[addr];
      if constexpr (c < 64) {
        slot[c] = x;  // n > 64: every main column is real
      } else {
        slot[c] = (c < opaque(n)) ? x : 0.f;  // (opaque: the n tests are not kept live as masks)
      }
      if ((c & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
    slot[NV] = gv;
  }
  float tq[TQ];
  float gt;  // border of tail row 64 + ti (replicated over its LPR lanes)
  {
    const int r = 64 + ti;
#pragma unroll
    for (int m = 0; m < TQ; m++) {
      const int c = 64 + TQ * ts + m;
      const int addr = (c >= r) ? G::tri(r) + c : G::tri(c) + r;
      const float x = sh.P[addr];
      tq[m] = (r < n && c < n) ? x : ((r == c) ? 1.f : 0.f);
    }
    gt = (r < n) ? sh.gtail[ti] : 0.f;
  }
  tsync();

  T_MARK(1);
  // ---- bordered Cholesky [H | g], main pivots 0..63, two per step (class 1's look-ahead form:
  // raw column k and column k+1 corrected by beta into P's packed rows, from the lanes' register
  // k / k+1). The tail parts (rows 64..NV-1) of a pivot pair's columns are the registers 64..NV-1
  // of lanes k and k+1, stored raw by those lanes once the previous step's sweep has updated them
  // (the tail chunks are the last of every sweep); the tail chunks and the tail block apply them
  // with the raw-column coefficients (a0 - beta a1, a1).
  int status = CMPC_OK;
  float my_inv = 1.f;
  float i0n = 1.f, betan = 0.f, i1n = 1.f, g0n = 0.f, g1n = 0.f;
  auto look = [&](auto JJ) {
    constexpr int j = decltype(JJ)::value, j1 = j + 1;
    constexpr int cj = j & ~3, cj1 = j1 & ~3;
    if constexpr (j1 < 64) {
      float d0 = rl(slot[j], j);
      const float h10 = rl(slot[j], j1);
      if (!(d0 > 0.f)) { status = CMPC_NOT_PD; d0 = 1e-30f; }
      i0n = __builtin_amdgcn_rsqf(d0);
      betan = h10 * (i0n * i0n);
      float d1 = fmaf(-h10, betan, rl(slot[j1], j1));
      if (!(d1 > 0.f)) { status = CMPC_NOT_PD; d1 = 1e-30f; }
      i1n = __builtin_amdgcn_rsqf(d1);
      g0n = rl(slot[NV], j);
      g1n = fmaf(-betan, g0n, rl(slot[NV], j1));
      const float s1 = fmaf(-slot[j], betan, slot[j1]);
      if (v >= cj) sh.P[G::prow(j) + v - cj] = (v >= j) ? slot[j] : 0.f;
      if (v >= cj1) sh.P[G::prow(j1) + v - cj1] = (v >= j1) ? s1 : 0.f;
      tsync();
    }
  };
  // tail parts of the pair (j, j+1): lanes j and j+1 store their registers 64..NV-1 (raw)
  auto pub_tail = [&](auto JJ) {
    constexpr int j = decltype(JJ)::value, j1 = j + 1;
    constexpr int bj = G::prow(j) + 64 - (j & ~3), bj1 = G::prow(j1) + 64 - (j1 & ~3);
    {
      // readlane form: lane i < T stores row 64 + i of column j, lane T + i of column j1 (one
      // predicated store, no per-lane branch around the row registers)
      float x = 0.f;
      static_for<0, T>([&](auto M) {
        constexpr int m = decltype(M)::value;
        const float a = rl(slot[64 + m], j), b = rl(slot[64 + m], j1);
        x = (v == m) ? a : x;
        x = (v == T + m) ? b : x;
      });
      if (v < 2 * T) sh.P[(v < T) ? bj + v : bj1 + v - T] = x;
    }
  };
  look(std::integral_constant<int, 0>{});
  pub_tail(std::integral_constant<int, 0>{});
  tsync();
  static_for<0, 32>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value;
    constexpr int k1 = k + 1, k2 = k + 2;
    constexpr int c0 = k & ~3, c1 = k1 & ~3, c2 = k2 & ~3;
    constexpr int rk = G::prow(k), rk1 = G::prow(k1);
    const float i0 = i0n, beta = betan, i1 = i1n, g0 = g0n, g1 = g1n;
    if (v == k) { my_inv = i0; sh.u.ch.ibuf[k] = i0; }
    if (v == k1) { my_inv = i1; sh.u.ch.ibuf[k1] = i1; }
    if (v == 0) sh.u.ch.bpair[k / 2] = beta;
    const float s0 = slot[k];
    const float s1 = fmaf(-s0, beta, slot[k1]);
    const float a0 = (v > k) ? -s0 * (i0 * i0) : 0.f;
    const float a1 = (v > k1) ? -s1 * (i1 * i1) : 0.f;
    slot[NV] = fmaf(a1, g1, fmaf(a0, g0, slot[NV]));
    static_for<c2 / 4, 16>([&](auto JC) {
      constexpr int c = 4 * decltype(JC)::value;
      const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
      const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
      axpy4(a0, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
      axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
      if constexpr (k2 < 64 && c == c2) look(std::integral_constant<int, k2>{});
      CMPC_TSWEEP_FENCE(c);
    });
    // materialise the main columns here: otherwise the FMAs sink below the divergent stores that
    // follow (IR-level sinking toward the step's pin) and every loaded chunk stays live (800 spills)
    tpin(slot);
    {
      // tail chunks (raw columns)
      const float a0t = fmaf(-beta, a1, a0);
      static_for<16, NV / 4>([&](auto JC) {
        constexpr int c = 4 * decltype(JC)::value;
        const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
        axpy4(a0t, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
      });
      tpin(slot);
      // the tail block and borders: row 64 + ti's coefficients from its raw entries
      const float h0 = sh.P[rk + 64 + ti - c0], h1 = sh.P[rk1 + 64 + ti - c1];
      const float s1t = fmaf(-h0, beta, h1);
      const float a1r = -s1t * (i1 * i1);
      const float a0c = -h0 * (i0 * i0);
      const float a0r = fmaf(-beta, a1r, a0c);
#pragma unroll
      for (int m = 0; m < TQ; m++) {
        const float p0 = sh.P[rk + 64 + TQ * ts + m - c0], p1 = sh.P[rk1 + 64 + TQ * ts + m - c1];
        tq[m] = fmaf(a1r, p1, fmaf(a0r, p0, tq[m]));
      }
      gt = fmaf(a1r, g1, fmaf(a0c, g0, gt));
    }
    if constexpr (k2 < 64) pub_tail(std::integral_constant<int, k2>{});
    tsync();
    tpin(slot);
    tpin(tq);
    asm volatile("" : "+v"(gt));
  });

  T_MARK(2);
  // ---- the tail pivots 64..NV-1: the T x T Schur complement, row 64 + i in lane i < T (T
  // registers), one pivot per step; padding rows (>= n) are identity rows. Columns go to P's packed
  // rows (J below reads them like the main columns; their pair beta is 0)
  float yt = 0.f;  // lane i < T: y of tail row 64 + i
  {
#pragma unroll
    for (int m = 0; m < TQ; m++) sh.u.ch.h22[ti * T + TQ * ts + m] = tq[m];
    if (ts == 0) sh.u.ch.gt[ti] = gt;
    tsync();
    float trow[T];
    const int li = (v < T) ? v : 0;
    static_for<0, T>([&](auto C) {
      constexpr int c = decltype(C)::value;
      trow[c] = (v < T) ? sh.u.ch.h22[li * T + c] : 0.f;
    });
    float gti = (v < T) ? sh.u.ch.gt[li] : 0.f;
    float tinv = 1.f;
    tsync();
    static_for<0, T>([&](auto TT) {
      constexpr int t = decltype(TT)::value;
      constexpr int k = 64 + t, ck = k & ~3, rk = G::prow(k);
      if (v < T && v >= ck - 64) sh.P[rk + 64 + v - ck] = (v >= t) ? trow[t] : 0.f;
      tsync();
      float d = rl(trow[t], t);
      if (!(d > 0.f)) { status = CMPC_NOT_PD; d = 1e-30f; }
      const float inv = __builtin_amdgcn_rsqf(d);
      if (v == t) tinv = inv;
      if (v == 0) {
        sh.u.ch.ibuf[k] = inv;
        if ((t & 1) == 0) sh.u.ch.bpair[k / 2] = 0.f;
      }
      const float gk = rl(gti, t);
      const float a = (v < T && v > t) ? -trow[t] * (inv * inv) : 0.f;
      static_for<t + 1, T>([&](auto C) {
        constexpr int c = decltype(C)::value;
        trow[c] = fmaf(a, sh.P[rk + 64 + c - ck], trow[c]);
      });
      gti = fmaf(a, gk, gti);
      tpin(trow);
      asm volatile("" : "+v"(gti));
    });
    yt = (v < T && 64 + v < n) ? gti * tinv : 0.f;
  }
  const float yv = slot[NV] * my_inv;  // L y = g (main rows)
  tsync();

  T_MARK(3);
  // ---- J = L^-T: lane v solves L x = e_v over the stored columns (class 1's two-column steps);
  // the tail chunks apply the raw tail parts of the main pairs with (a0 - beta a1, a1)
  static_for<0, NV>([&](auto C) {
    constexpr int c = decltype(C)::value;
    slot[c] = (c == v) ? 1.f : 0.f;
  });
  static_for<0, NV / 2>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value;
    constexpr int k1 = k + 1, c2 = (k + 2) & ~3;
    constexpr int c0 = k & ~3, c1 = k1 & ~3;
    constexpr int rk = G::prow(k), rk1 = G::prow(k1);
    if (k < 64 || k < opaque(n)) {
      const float i0 = sh.u.ch.ibuf[k], i1 = sh.u.ch.ibuf[k1];
      const float h = sh.P[rk + k1 - c0];  // L[k+1][k] sqrt(d_k)
      const float x0 = slot[k] * i0;
      const float x1 = fmaf(-h * i0, x0, slot[k1]) * i1;
      const float a0 = -x0 * i0, a1 = -x1 * i1;
      if constexpr (c2 < 64) {
#pragma unroll
        for (int c = c2; c < 64; c += 4) {
          const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
          const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
          axpy4(a0, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
          axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
          CMPC_TSWEEP_FENCE(c);
        }
      }
      const float a0t = (k < 64) ? fmaf(-sh.u.ch.bpair[k / 2], a1, a0) : a0;
#pragma unroll
      for (int c = (c2 > 64 ? c2 : 64); c < NV; c += 4) {
        const float4 r0 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        const float4 r1 = *reinterpret_cast<const float4*>(&sh.P[rk1 + c - c1]);
        axpy4(a0t, r0, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
        axpy4(a1, r1, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
      }
      slot[k] = x0;
      slot[k1] = x1;
      tpin(slot);
    }
  });
  // J's tail rows: J22 = L22^-T (lane i < T solves over the tail columns), then into the segment
  // layout (lane: tail row ti, columns [SW ts, SW ts + SW))
  float jt[SW];
  {
    float xr[T];
    static_for<0, T>([&](auto C) {
      constexpr int c = decltype(C)::value;
      xr[c] = (c == v) ? 1.f : 0.f;
    });
    static_for<0, T / 2>([&](auto KB) {
      constexpr int t = 2 * decltype(KB)::value, t1 = t + 1;
      constexpr int k = 64 + t, k1 = k + 1, ck = k & ~3, ck1 = k1 & ~3;
      constexpr int rk = G::prow(k), rk1 = G::prow(k1);
      if (k < n) {
        const float i0 = sh.u.ch.ibuf[k], i1 = sh.u.ch.ibuf[k1];
        const float h = sh.P[rk + k1 - ck];
        const float x0 = xr[t] * i0;
        const float x1 = fmaf(-h * i0, x0, xr[t1]) * i1;
        const float a0 = -x0 * i0, a1 = -x1 * i1;
        static_for<t + 2, T>([&](auto C) {
          constexpr int c = decltype(C)::value;
          xr[c] = fmaf(a1, sh.P[rk1 + 64 + c - ck1], fmaf(a0, sh.P[rk + 64 + c - ck], xr[c]));
        });
        xr[t] = x0;
        xr[t1] = x1;
        tpin(xr);
      }
    });
    tsync();  // the tail block exchange area is free (h22 read above, before the pivots)
    if (v < T) {
      static_for<0, T>([&](auto C) {
        constexpr int c = decltype(C)::value;
        sh.u.ch.h22[v * T + c] = xr[c];
      });
    }
    tsync();
#pragma unroll
    for (int m = 0; m < SW; m++) {
      const int c = SW * ts + m;
      jt[m] = (c >= 64) ? sh.u.ch.h22[ti * T + (c >= 64 ? c - 64 : 0)] : 0.f;
    }
  }
  tsync();

  T_MARK(4);
  // ---- unconstrained minimiser x = -J y (main rows: lanes; tail rows: segment dots)
  sh.vbuf()[v] = yv;
  if (v < T) sh.vbuf()[64 + v] = yt;
  tsync();
  f2v xacc = {0.f, 0.f};
  piped_sweep<0, NV, TAIL_PIPE_GRP>(
      [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
      [&](auto C, float4 y4) {
        constexpr int c = decltype(C)::value;
        dot4(xacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], y4);
      });
  float xv = -(xacc.x + xacc.y);
  float xt;
  {
    float a = 0.f;
#pragma unroll
    for (int m = 0; m < SW; m++) a = fmaf(jt[m], sh.vbuf()[SW * ts + m], a);
    xt = (64 + ti < n) ? -group_sum<LPR>(a) : 0.f;
  }
  tsync();

  T_MARK(5);
  // ---- Goldfarb-Idnani dual active set on the friction pyramids (class 1's loop; the tail
  // rows' parts beside every row operation)
  const float mui = P.mu_inv;
  const float fnorm = rsqrtf(mui * mui + 1.f);
  int q = 0;
  int iters = 0;
  float u_reg = 0.f;
  int act_reg = 0;
  int p = -1;
  Cons cp{};
  float up = 0.f;
  bool rinv_ok = true;
  bool handoff = false;
  using S = SharedT<T>;
  if (status == CMPC_OK) {
    for (;;) {
      tpin(slot);
      tpin(jt);
      const int v = tid_opq();
      const int ti = v / LPR, ts = v % LPR;
      sh.u.gi.xs[v] = xv;
      if (ts == 0 && ti < T) sh.u.gi.xs[64 + ti] = xt;
      tsync();
      if (p < 0) {
        float best = 0.f, xm = 0.f;
        int bid = 0x7fffffff;
        if (v < nfs) {
          const float fx = sh.u.gi.xs[3 * v], fy = sh.u.gi.xs[3 * v + 1], fz = sh.u.gi.xs[3 * v + 2];
          xm = fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz)));
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
        const float xmax = wave_max(xm);
        wave_argmin(best, bid);
        const float tol = 1e-5f * fmaxf(1.f, xmax);
        if (bid == 0x7fffffff || best >= -tol) break;
        p = __builtin_amdgcn_readfirstlane(bid);
        cp = decode_cons(p, mui, sh.sub[p / 6]);
        up = 0.f;
      }
      if (++iters > P.max_iter + 2 * n) { status = CMPC_MAX_ITER; break; }
#if CMPC_TRIP_PRIO_AT > 0
      if (iters == CMPC_TRIP_PRIO_AT) __builtin_amdgcn_s_setprio(CMPC_TAIL_TRIP_PRIO);
#endif
      // d = J' n+: rows ia, iz of J through LDS (main rows from their lanes, tail rows from their
      // segments)
      if (v == cp.ia || v == cp.iz) {
        const int boff = (v == cp.iz) ? NV : 0;
#pragma unroll
        for (int c = 0; c < NV; c++) {
          sh.u.gi.bufA[boff + c] = slot[c];
          if ((c & 15) == 15) __builtin_amdgcn_sched_barrier(0);
        }
      }
      if (cp.iz >= 64) {  // uniform: a tail row is exported (iz >= ia; fz is the last of a foot-step)
        const int r = 64 + ti;
        if (r == cp.ia || r == cp.iz) {
          const int boff = (r == cp.iz) ? NV : 0;
#pragma unroll
          for (int m = 0; m < SW; m++) sh.u.gi.bufA[boff + SW * ts + m] = jt[m];
        }
      }
      tsync();
      const float dv = (cp.ia != cp.iz) ? fmaf(cp.ca, sh.u.gi.bufA[v], cp.cb * sh.u.gi.bufB[v]) : cp.cb * sh.u.gi.bufB[v];
      float dvt = 0.f;  // column 64 + v (v < T)
      if (v < T)
        dvt = (cp.ia != cp.iz) ? fmaf(cp.ca, sh.u.gi.bufA[64 + v], cp.cb * sh.u.gi.bufB[64 + v])
                               : cp.cb * sh.u.gi.bufB[64 + v];
      const float dm = (v >= q) ? dv : 0.f;
      sh.vbuf()[v] = dm;
      if (v < T) sh.vbuf()[64 + v] = dvt;
      tsync();
      // z = J2 d2, zn = |d2|^2, dn = |d|^2
      f2v zacc = {0.f, 0.f}, nacc = {0.f, 0.f};
      piped_sweep<0, NV, TAIL_PIPE_GRP>(
          [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
          [&](auto C, float4 m4) {
            constexpr int c = decltype(C)::value;
            T_DOT(zacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], m4);
            T_DOT(nacc, m4.x, m4.y, m4.z, m4.w, m4);
          });
      float zv = zacc.x + zacc.y, zn = nacc.x + nacc.y;
      float zt;
      {
        float a = 0.f;
#pragma unroll
        for (int m = 0; m < SW; m++) a = fmaf(jt[m], sh.vbuf()[SW * ts + m], a);
        zt = group_sum<LPR>(a);
      }
      asm volatile("" : "+v"(zv), "+v"(zn), "+v"(zt));
      const float dn = wave_sum(fmaf(dv, dv, dvt * dvt));
      // r = R^-1 d1 (class 1)
      float acc = dv, r_reg = 0.f;
      if (rinv_ok) {
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
          const float ri = rl(acc, i) * fast_rcp(pd);
          if (v < i) acc = fmaf(-pv, ri, acc);
          r_reg = (v == i) ? ri : r_reg;
          pd = pd_n;
          pv = pv_n;
        }
      }
      float t1 = kBigF;
      int kk = 0x7fffffff;
      if (v < q && r_reg > 0.f) { t1 = fmaxf(u_reg * fast_rcp(r_reg), 0.f); kk = v; }
      wave_argmin(t1, kk);
      const float xa = (cp.ia < 64) ? rl(xv, cp.ia & 63) : rl(xt, LPR * ((cp.ia - 64) & (T - 1)));
      const float xz = (cp.iz < 64) ? rl(xv, cp.iz & 63) : rl(xt, LPR * ((cp.iz - 64) & (T - 1)));
      const float spv = fmaf(cp.ca, xa, fmaf(cp.cb, xz, -cp.bp));
      const bool zero_step = !(zn > 1e-9f * dn);
      const float t2 = zero_step ? kBigF : -(spv * fast_rcp(zn));
      const float t = fminf(t1, t2);
      if (t >= kBigF) { status = CMPC_INFEASIBLE; break; }
      const bool add = !zero_step && t2 <= t1;
      const bool add_u = __builtin_amdgcn_readfirstlane((int)add) != 0;
      if (add_u && q >= 64) { handoff = true; break; }  // a 65th active position: the wide class
      if (v < q) u_reg = fmaf(-t, r_reg, u_reg);
      up += t;
      if (!zero_step) {
        xv = fmaf(t, zv, xv);
        xt = fmaf(t, zt, xt);
      }
      float beta = 0.f;
      if (add) {
        const float tsq = sqrtf(zn);
        const float dq = rl(dv, q);
        const float sgn = (dq >= 0.f) ? 1.f : -1.f;
        beta = fast_rcp(tsq * (tsq + fabsf(dq)));
        sh.vbuf()[v] = (v == q) ? dq + sgn * tsq : dm;
        const int offq = rcol(q);
        if (v < q) sh.P[offq + v] = dv;
        if (v == q) {
          sh.P[offq + q] = -sgn * tsq;
          u_reg = up;
          act_reg = p;
        }
        if (rinv_ok) {
          if (q < S::QI) {
            const float irho = 1.f / (-sgn * tsq);
            const int offi = S::RB + rcol(q);
            if (v < q) sh.P[offi + v] = -r_reg * irho;
            if (v == q) sh.P[offi + q] = irho;
          } else {
            rinv_ok = false;
          }
        }
        if (v == 0) sh.cmask[p / 6] |= (unsigned char)(1u << (p % 6));
      } else {
        // drop active constraint kk (class 1)
        sh.vbuf()[v] = 0.f;
        if (v < T) sh.vbuf()[64 + v] = 0.f;
        const int k = __builtin_amdgcn_readfirstlane(kk);
        const int ak = rli(act_reg, k);
        if (v == 0) sh.cmask[ak / 6] &= (unsigned char)~(1u << (ak % 6));
        const int a_nx = lane_next_i(act_reg, act_reg);
        const float u_nx = lane_next(u_reg, u_reg);
        if (v >= k && v < q - 1) { act_reg = a_nx; u_reg = u_nx; }
        if (v < k || v > q - 2) *reinterpret_cast<float2*>(&sh.u.gi.cs[2 * v]) = make_float2(1.f, 0.f);
        const bool in_c = v >= k && v <= q - 2;
        float top = in_c ? sh.P[rcol(v + 1) + k] : 0.f;
        tsync();
        for (int r = 0; r < k; r++) {
          const float x = in_c ? sh.P[rcol(v + 1) + r] : 0.f;
          tsync();
          if (in_c) sh.P[rcol(v) + r] = x;
          tsync();
        }
        for (int j = k; j <= q - 2; j++) {
          const bool on = in_c && v >= j;
          const float bot = on ? sh.P[rcol(v + 1) + j + 1] : 0.f;
          tsync();
          const float a0 = rl(top, j), b0 = rl(bot, j);
          const float hh = sqrtf(a0 * a0 + b0 * b0);
          float cc = 1.f, sn = 0.f;
          if (hh > 0.f) { const float ih = fast_rcp(hh); cc = a0 * ih; sn = b0 * ih; }
          if (on) {
            sh.P[rcol(v) + j] = fmaf(cc, top, sn * bot);
            top = fmaf(-sn, top, cc * bot);
          }
          if (v == 0) *reinterpret_cast<float2*>(&sh.u.gi.cs[2 * j]) = make_float2(cc, sn);
          tsync();
        }
        if (rinv_ok) {
          const int i = v;
          const bool live = i < q && i != k;
          const int i2 = (i > k) ? i - 1 : i;
          int j = (i > k) ? i - 1 : k;
          float carry = (live && j >= i) ? sh.P[S::RB + rcol(j) + i] : 0.f;
          for (int jj = k; jj <= q - 2; jj++) {
            const float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * jj]);
            const float b = (live && jj >= j && jj + 1 >= i) ? sh.P[S::RB + rcol(jj + 1) + i] : 0.f;
            tsync();
            if (live && jj >= j) {
              sh.P[S::RB + rcol(jj) + i2] = fmaf(cs2.x, carry, cs2.y * b);
              carry = fmaf(-cs2.y, carry, cs2.x * b);
            }
          }
        }
      }
      tsync();
      {
        // J <- J (I - beta w w') (no-op on a drop: beta = 0)
        f2v tacc = {0.f, 0.f};
        piped_sweep<0, NV, TAIL_PIPE_GRP>(
            [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
            [&](auto C, float4 w4) {
              constexpr int c = decltype(C)::value;
              T_DOT(tacc, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3], w4);
            });
        const float bt = -beta * (tacc.x + tacc.y);
        float ta = 0.f;
#pragma unroll
        for (int m = 0; m < SW; m++) ta = fmaf(jt[m], sh.vbuf()[SW * ts + m], ta);
        const float btt = -beta * group_sum<LPR>(ta);
        asm volatile("" ::: "memory");
        piped_sweep<0, NV, TAIL_PIPE_GRP>(
            [&](auto C) { return *reinterpret_cast<const float4*>(&sh.vbuf()[decltype(C)::value]); },
            [&](auto C, float4 w4) {
              constexpr int c = decltype(C)::value;
              axpy4(bt, w4, slot[c + 0], slot[c + 1], slot[c + 2], slot[c + 3]);
            });
#pragma unroll
        for (int m = 0; m < SW; m++) jt[m] = fmaf(btt, sh.vbuf()[SW * ts + m], jt[m]);
      }
      if (!add_u) {
        // J columns (j, j+1) <- Givens chain j = 0 .. 62 (q <= 64: pairs past 62 are identities)
        static_for<0, 63>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          const float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * j]);
          const float x0 = slot[j], x1 = slot[j + 1];
          slot[j] = fmaf(cs2.x, x0, cs2.y * x1);
          slot[j + 1] = fmaf(-cs2.y, x0, cs2.x * x1);
          if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
        // tail rows: segment by segment, the seam rotations between neighbouring lanes
        static_for<0, LPR>([&](auto SS) {
          constexpr int s = decltype(SS)::value;
          constexpr int j0 = SW * s;
          if constexpr (j0 <= 62) {
            static_for<0, SW - 1>([&](auto M) {
              constexpr int m = decltype(M)::value;
              constexpr int j = j0 + m;
              if constexpr (j <= 62) {
                float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * j]);
                if (ts != s) cs2 = make_float2(1.f, 0.f);
                const float x0 = jt[m], x1 = jt[m + 1];
                jt[m] = fmaf(cs2.x, x0, cs2.y * x1);
                jt[m + 1] = fmaf(-cs2.y, x0, cs2.x * x1);
              }
            });
            constexpr int js = j0 + SW - 1;
            if constexpr (js <= 62 && s + 1 < LPR) {
              const float2 cs2 = *reinterpret_cast<const float2*>(&sh.u.gi.cs[2 * js]);
              const float nxt = lane_next(0.f, jt[0]);        // lane + 1's first column
              const float prv = lane_prev(0.f, jt[SW - 1]);   // lane - 1's last column
              if (ts == s) jt[SW - 1] = fmaf(cs2.x, jt[SW - 1], cs2.y * nxt);
              if (ts == s + 1) jt[0] = fmaf(-cs2.y, prv, cs2.x * jt[0]);
            }
          }
        });
      }
      if (add) {
        q++;
        p = -1;
      } else {
        q--;
      }
      tsync();
    }
  }
  T_MARK(6);
  if (handoff) {  // the wide class solves this instance afresh
    if (v == 0) {
      if (ovf_list) ovf_list[atomicAdd(ovf_count, 1)] = inst;
      else st_out[0] = kHandoffStatus;
    }
    return;
  }

  // ---- scatter (q_soln layout 12 k + 3 leg + axis, swing -> 0) staged in LDS, coalesced out
  const bool ok = (status == CMPC_OK);
  tsync();
  for (int t = v; t < 12 * N; t += 64) sh.P[t] = 0.f;
  tsync();
  if (ok) sh.P[12 * sh.varblk[v] + sh.varcol[v]] = xv;
  if (ok && ts == 0 && 64 + ti < n) sh.P[12 * sh.varblk[64 + ti] + sh.varcol[64 + ti]] = xt;
  tsync();
  for (int t = 4 * v; t < P.out_cols; t += 256)  // (the leading steps kept, 12 N by default)
    *reinterpret_cast<float4*>(&fout[t]) = *reinterpret_cast<const float4*>(&sh.P[t]);
  if (v == 0) {
    st_out[0] = (uint8_t)status;
    if (it_out) it_out[0] = iters;
  }
#ifdef CMPC_PHASE_PROF
  T_MARK(7);
  if (v == 0) {
    ph[8] = 1;
    ph[9] = (unsigned long long)iters;
#pragma unroll
    for (int i = 0; i < 16; i++) atomicAdd(&g_t_phase[i], ph[i]);
  }
#endif
}

}  // namespace

// One workgroup per list entry (entries first + blockIdx.x). The grid covers the whole list
// (one workgroup per possible entry: surplus workgroups exit after reading the count) or, from
// 16384 instances, the count an earlier solve predicts (cmpc_launch.hip hint), followed by the
// looping form below over any entries past it. (A persistent form that dequeues the whole list
// measured worse everywhere: its resident 168-VGPR waves keep two class-1 waves off every SIMD
// they share for the whole run, profiles/r05_h, r05_i; a grid-stride loop in this kernel itself
// spills 24 B more and cost 4-6 % at 4096 instances, profiles/r06_hint2.)
__global__ __launch_bounds__(64, CMPC_TAIL_WAVES_PER_EU) void cmpc_solve_t_kernel(
    const float* __restrict__ recs, KParams P, float* __restrict__ forces, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, const int* __restrict__ in_list, const int* __restrict__ in_count,
    int* __restrict__ ovf_list, int* __restrict__ ovf_count, int first) {
  __shared__ SharedT<kTailRows> sh;
#if CMPC_TAIL_PRIO > 0
  __builtin_amdgcn_s_setprio(CMPC_TAIL_PRIO);
#endif
  const int b = first + (int)blockIdx.x;
  if (b >= *in_count) return;
  const int t = in_list[b];
  solve_t<kTailRows>(recs + (size_t)t * P.rec_words, P, sh, forces + (size_t)t * P.out_cols, status + t,
                     iters ? iters + t : nullptr, ovf_list, ovf_count, t);
}

// The entries past a predicted grid (normally none: its few workgroups exit at once), grid-stride.
__global__ __launch_bounds__(64, CMPC_TAIL_WAVES_PER_EU) void cmpc_solve_t_rest_kernel(
    const float* __restrict__ recs, KParams P, float* __restrict__ forces, uint8_t* __restrict__ status,
    int32_t* __restrict__ iters, const int* __restrict__ in_list, const int* __restrict__ in_count,
    int* __restrict__ ovf_list, int* __restrict__ ovf_count, int first) {
  __shared__ SharedT<kTailRows> sh;
  const int count = *in_count;
  for (int b = first + (int)blockIdx.x; b < count; b += (int)gridDim.x) {
    const int t = in_list[b];
    solve_t<kTailRows>(recs + (size_t)t * P.rec_words, P, sh, forces + (size_t)t * P.out_cols, status + t,
                       iters ? iters + t : nullptr, ovf_list, ovf_count, t);
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  }
}

// Self-classifying form (no classify list, so it can start ahead of class 1 instead of behind the
// classify pass): workgroup g scans chunks g, g + G, ... of `chunk` instances, lanes < chunk count
// the stance foot-steps of one instance each (the classify pass's test: eliminated iff
// |gait * f_max| < 0.01, SolverMPC.cpp:869-894), and solves the chunk's tail-class instances in
// turn with the same solve_t as the list forms (bitwise the same forces).
__global__ __launch_bounds__(64, CMPC_TAIL_WAVES_PER_EU) void cmpc_solve_t_self_kernel(
    const float* __restrict__ recs, int batch, KParams P, float* __restrict__ forces,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, int* __restrict__ ovf_list,
    int* __restrict__ ovf_count, int chunk) {
  __shared__ SharedT<kTailRows> sh;
#if CMPC_TAIL_PRIO > 0
  __builtin_amdgcn_s_setprio(CMPC_TAIL_PRIO);
#endif
  for (int c0 = (int)blockIdx.x * chunk; c0 < batch; c0 += (int)gridDim.x * chunk) {
    const int i = c0 + (int)threadIdx.x;
    bool mine = false;
    if ((int)threadIdx.x < chunk && i < batch) {
      const uint32_t* g = reinterpret_cast<const uint32_t*>(recs + (size_t)i * P.rec_words + CMPC_REC_GAIT(P.N));
      int nfs = 0;
      for (int k = 0; k < P.N; k++) {
        const uint32_t w = g[k];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const float ub = (float)((w >> (8 * j)) & 0xffu) * P.f_max;
          nfs += (ub < 0.01f && ub > -0.01f) ? 0 : 1;
        }
      }
      mine = tail_class(P, 3 * nfs);  // 64 < n <= 64 + kTailRows
    }
    unsigned long long m = __ballot(mine);
    while (m) {
      const int b = __ffsll((long long)m) - 1;
      m &= m - 1ull;
      const int t = c0 + b;
      solve_t<kTailRows>(recs + (size_t)t * P.rec_words, P, sh, forces + (size_t)t * P.out_cols, status + t,
                         iters ? iters + t : nullptr, ovf_list, ovf_count, t);
      __builtin_amdgcn_wave_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

hipError_t launch_tail_self(const float* d_recs, int batch, const KParams& P, float* d_forces, uint8_t* d_status,
                            int32_t* d_iters, int* ovf_list, int* ovf_count, int grid, int chunk,
                            hipStream_t stream) {
  if (grid <= 0 || batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_solve_t_self_kernel, dim3(grid), dim3(64), 0, stream, d_recs, batch, P, d_forces,
                     d_status, d_iters, ovf_list, ovf_count, chunk);
  return hipGetLastError();
}

hipError_t launch_tail(const float* d_recs, const KParams& P, float* d_forces, uint8_t* d_status,
                       int32_t* d_iters, const int* in_list, const int* in_count, int* ovf_list,
                       int* ovf_count, int grid, hipStream_t stream, int rest_grid) {
  if (grid <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_solve_t_kernel, dim3(grid), dim3(64), 0, stream, d_recs, P, d_forces, d_status, d_iters,
                     in_list, in_count, ovf_list, ovf_count, 0);
  if (rest_grid > 0)
    hipLaunchKernelGGL(cmpc_solve_t_rest_kernel, dim3(rest_grid), dim3(64), 0, stream, d_recs, P, d_forces,
                       d_status, d_iters, in_list, in_count, ovf_list, ovf_count, grid);
  return hipGetLastError();
}

}  // namespace cmpc

#ifdef CMPC_PHASE_PROF
// cycles per stage summed over solved tail-class instances: condensation, H load, main Cholesky,
// tail Cholesky, J, x = -J y, active set, scatter; [8] instances, [9] active-set iterations. Resets.
extern "C" int cmpc_debug_tphase_read(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t_phase), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
  unsigned long long z[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_t_phase), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
