// cmpc_wide.h — the wide size classes (template over the row width NV = 80, 96, 120, 128, 144, 192, 256):
// fused condensation + friction-cone QP for instances with more than 64 reduced force variables
// (random contact tables at N = 10; trot at N >= 11, the deployed N = 16 and config 5's N = 20;
// all-stance tables), over the classify pass's list of the class.
//
// Same computation as cmpc_class1.hip — one call of the reference's solve_mpc()
// (be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-982): stance table + swing
// elimination, model + closed-form c2qp, structured condensation of the reduced qH / qg,
// bordered Cholesky, J = L^-T, Goldfarb-Idnani dual active set on the friction pyramids
// (qpOASES QProblem::init in the reference, :955-969), scatter to q_soln.
//
// MI355X mapping: TWO lanes per matrix row, NV/32 wavefronts per instance.
//   * thread t: wave w = t / 64, lane l = t % 64, half h = l / 32, row r = 32 w + l % 32; the
//     two lanes of a row are partners across the wave's halves (v_permlane32_swap exchanges and
//     sums their registers in one VALU op, no LDS);
//   * each lane holds NV/2 columns of its row in registers (64 at NV = 128, against 128 when one
//     lane owns a whole row: no spills, <= 128 VGPRs, four waves per SIMD to hide the LDS and
//     barrier latency of the factorisation);
//   * factorisation phases (Cholesky, J = L^-T): half h owns columns c = 2j + h (interleaved, so
//     both halves keep work to the end). Each published pivot row of the factor is stored in LDS
//     as its even- and odd-column segments from column 2 j0(k) on, so every half reads its own
//     columns as contiguous ds_read_b128;
//   * active-set phase: J's columns are relabelled l = h NV/2 + j (any column permutation of
//     J keeps J J' = H^-1), so the Givens chains of a drop run along one lane's registers; only
//     an active set larger than NV/2 crosses between the halves (one exchange at the seam);
//   * the QP's triangular factor R is explicit, packed by columns in LDS, maintained by
//     wavefront 0 with readlane chains (RQ = NV/64 active-set positions per lane).
// Everything is fp32 (the reference condenses in fp32: common_types.h:14).
#pragma once
#include "cmpc_common.h"

#ifndef CMPC_DIAG_STOP
#define CMPC_DIAG_STOP 0
#endif
#ifndef CMPC_WIDE_WAVES_PER_EU
#define CMPC_WIDE_WAVES_PER_EU 3
#endif
// hard VGPR cap per row width (0: none); 128 = four waves per SIMD
// Cholesky and J = L^-T two pivots per step (rank-2 sweeps, half the barriers); 0: one
#ifndef CMPC_WIDE_CHOL2
#define CMPC_WIDE_CHOL2 1
#endif
#ifndef CMPC_WIDE_J2
#define CMPC_WIDE_J2 CMPC_WIDE_CHOL2
#endif
// wavefronts skip the factorisation steps that cannot change their rows (1); 0: every wave sweeps
#ifndef CMPC_WIDE_SKIP
#define CMPC_WIDE_SKIP 1
#endif
#ifndef CMPC_WIDE_VGPR_CAP
#define CMPC_WIDE_VGPR_CAP 0
#endif
// one mixed-precision refinement step of the converged active set (wide_refine below); 0: off
#ifndef CMPC_WIDE_REFINE
#define CMPC_WIDE_REFINE 1
#endif
// refinements per instance at most, and the constraint tolerance (x x_max) after one
#ifndef CMPC_TRIP_PRIO_AT  // active-set trips after which the N <= 10 builds raise their priority
#define CMPC_TRIP_PRIO_AT 0
#endif
#ifndef CMPC_WIDE_TRIP_PRIO
#define CMPC_WIDE_TRIP_PRIO 3
#endif
// the active set's half-row dot products (z, |d2|^2, J_r . w) as two interleaved FMA chains (A/B)
#ifndef CMPC_WIDE_DOT2
#define CMPC_WIDE_DOT2 0
#endif
#if CMPC_WIDE_DOT2
#define W_DOT dot4x2
#else
#define W_DOT dot4
#endif
#ifndef CMPC_WIDE_PRIO  // s_setprio of the wide classes' waves (0: the default priority)
#define CMPC_WIDE_PRIO 0
#endif
#ifndef CMPC_DIAG_REF_LDSREC
#define CMPC_DIAG_REF_LDSREC 0
#endif
#ifndef CMPC_DIAG_REF_SKIP  // diagnostic builds: skip refinement phases (bit 0..4 = A..E; wrong results)
#define CMPC_DIAG_REF_SKIP 0
#endif
#ifndef CMPC_REF_BFA_MAX  // phases A / D branch-free over the feet / rows up to this width
#define CMPC_REF_BFA_MAX 96
#endif
#ifndef CMPC_REF_BFD_MAX
#define CMPC_REF_BFD_MAX 96
#endif
#ifndef CMPC_REFINE_MAX
#define CMPC_REFINE_MAX 4
#endif
#ifndef CMPC_REFINE_TOL
#define CMPC_REFINE_TOL 2e-7f
#endif


namespace cmpc {
namespace {

constexpr int kNoneW = 0x7fffffff;
typedef __attribute__((address_space(1))) float gfloat;

template <int NV>
struct WGeo {
  static_assert(NV % 8 == 0, "row width (each half's columns in 16-B chunks)");
  static constexpr int NH = NV / 2;             // columns per lane
  static constexpr int NW = (NV + 31) / 32;     // wavefronts (32 rows each)
  static constexpr int NT = 64 * NW;            // threads
  static constexpr int RQ = (NV + 63) / 64;     // active-set positions per lane of wave 0
  static constexpr int HOFF = NH + 8;           // half 1's base in logical-order LDS vectors
  static constexpr int VL = HOFF + NH;
  // condensation: H as packed upper rows (row r holds columns [r & ~3, NV), 16-B aligned)
  static constexpr int NG = NV / 4;
  static constexpr int PSZ_H = 4 * NG * NV - 8 * NG * (NG - 1);
  __host__ __device__ static constexpr int prow(int r) {
    return 4 * (r >> 2) * NV - 8 * (r >> 2) * ((r >> 2) - 1) + (r & 3) * (NV - 4 * (r >> 2));
  }
  __host__ __device__ static constexpr int prow0(int r) { return prow(r) - (r & ~3); }
  // H's exchange between the condensation and the row loads: the plain packed upper triangle,
  // element (r, c >= r) at tri(r) + c (unaligned row starts spread a half-wave's rows over the
  // banks; the 16-B aligned prow rows gave 16 bank groups)
  __host__ __device__ static constexpr int tri(int r) { return r * NV - ((r * (r + 1)) >> 1); }
  // factor rows: row k = even-column segment then odd-column segment, columns 2 j0(k) + h on
  __host__ __device__ static constexpr int j0(int k) { return (k >> 1) & ~3; }
  __host__ __device__ static constexpr int seg(int k) {  // segment stride (words)
    return (NH - j0(k)) + (((NH - j0(k)) % 64 == 0) ? 4 : 0);
  }
  __host__ __device__ static constexpr int fbase(int k) {
    int b = 0;
    for (int i = 0; i < k; i++) b += 2 * seg(i);
    return b;
  }
  static constexpr int PSZ_F = fbase(NV);
  static constexpr int PSZ_R = NV * (NV + 1) / 2;
  static constexpr int mx(int a, int b) { return a > b ? a : b; }
  static constexpr int PSZ = mx(mx(PSZ_H, PSZ_F), PSZ_R);
  // stage buffers behind P (offsets into SharedW::P). Prep + condensation: BdtT at PSZ;
  // Cholesky, J, x = -J y: ibuf, gbuf, ybuf at PSZ; active set: vbuf, bufA, bufB, dfull, xs, cs
  // from PSZ_R on (the factor rows are dead by then and R never reaches past PSZ_R). At NV = 128
  // this is 39 KB in place of 43: four workgroups per CU instead of three
  static constexpr int O_IBUF = PSZ, O_GBUF = PSZ + NV, O_YBUF = PSZ + 2 * NV;
  static constexpr int CH = 2 * NV + 2 * (NH + 4);
  static constexpr int O_VBUF = PSZ_R, O_BUFA = O_VBUF + VL, O_BUFB = O_BUFA + VL;
  static constexpr int O_DFULL = O_BUFB + VL, O_XS = O_DFULL + NV, O_CS = O_XS + NV;
  static constexpr int GI_END = O_CS + 2 * NV + 8;
  // R^-1 beside R for the first QI active-set positions (sized to keep each class's workgroups
  // per CU: 80 / 96 six, 120 / 128 four; at 80 the LDS it does not take lets class 1's one-wave
  // workgroups share the CU: QI 56 -> 36 config 3 +1.7 %, profiles/r04_ab/r04_ab80q2)
#ifdef CMPC_WIDE_QI
  static constexpr int QI = CMPC_WIDE_QI;
#else
  static constexpr int QI = (NV == 80) ? 36 : (NV == 96) ? 40 : (NV == 120) ? 48 : (NV == 128) ? 32
                            : (NV == 144) ? 40 : 64;
#endif
  static constexpr int O_RINV = (GI_END + 3) & ~3;
  static constexpr int PTOT = (mx(mx(PSZ + 12 * 16, PSZ + CH), O_RINV + QI * (QI + 1) / 2) + 3) & ~3;
  // the refinement's fp64 scratch (refine_gradient_seq: 18 + 12 N doubles) in the R^-1 area,
  // which the active set no longer reads once it has converged
  static_assert(2 * (24 + 12 * MAXN) <= QI * (QI + 1) / 2, "refinement scratch must fit the R^-1 area");
  static_assert(12 * MAXN <= 2 * NT && 6 * MAXN <= NT && 3 * MAXN <= NT - 20, "refinement phases: threads per step");
  static_assert(PSZ % 4 == 0 && PSZ_R % 4 == 0 && VL % 4 == 0, "16-B aligned stage buffers");
};

// logical-order LDS index (half 1 starts HOFF words in: the halves' ds_read_b128 never share a bank)
template <int NV>
__device__ __forceinline__ int lidx(int l) {
  return l + ((l >= WGeo<NV>::NH) ? (WGeo<NV>::HOFF - WGeo<NV>::NH) : 0);
}
__device__ __forceinline__ int rcol_w(int j) { return (j * (j + 1)) >> 1; }

constexpr int W_OFF_E = 0;
constexpr int W_OFF_ZE = W_OFF_E + 16 * MAXN;
constexpr int W_OFF_REC = W_OFF_ZE + 16 * MAXN;   // LDS copy of the instance record

template <int NV>
struct SharedW {
  using G = WGeo<NV>;
  alignas(16) float P[G::PTOT];  // H / factor / R, then the stage buffers (WGeo offsets)
  float redf[16];
  int redi[16];
  float sub[4 * MAXN];        // ub of each stance foot-step (gait * f_max)
  int sfs[4 * MAXN];          // stance foot-step ids, in order
  int blkbase[MAXN + 2];      // first reduced variable of each horizon step
  unsigned char varblk[G::NT], varcol[G::NT];
  alignas(4) unsigned char stance[4 * MAXN];
  unsigned char cflag[2 * NV + 8];  // active flag per constraint id (6 per stance foot-step)
  int deq_b;                  // list entry dequeued by the workgroup (persistent launches)
  __device__ __forceinline__ float (*BdtT())[16] { return reinterpret_cast<float(*)[16]>(&P[G::PSZ]); }
  __device__ __forceinline__ float* ibuf() { return &P[G::O_IBUF]; }    // 1 / sqrt(d_k) of pivot k
  __device__ __forceinline__ float* gbuf() { return &P[G::O_GBUF]; }    // gradient border of pivot row k
  // y = L^-1 g, de-interleaved: ybuf(h)[j] = y[2 j + h]
  __device__ __forceinline__ float* ybuf(int h) { return &P[G::O_YBUF + h * (G::NH + 4)]; }
  __device__ __forceinline__ float* vbuf() { return &P[G::O_VBUF]; }    // masked d, then the Householder vector
  __device__ __forceinline__ float* bufA() { return &P[G::O_BUFA]; }    // J rows ia, iz (logical order)
  __device__ __forceinline__ float* bufB() { return &P[G::O_BUFB]; }
  __device__ __forceinline__ float* dfull() { return &P[G::O_DFULL]; }  // d = J' n+ (logical index)
  __device__ __forceinline__ float* xs() { return &P[G::O_XS]; }        // x by reduced variable
  __device__ __forceinline__ float* cs() { return &P[G::O_CS]; }        // Givens (c, s), half 1 at +4 words
};
static_assert(W_OFF_REC + CMPC_REC_WORDS(MAXN) <= WGeo<80>::PSZ, "prep scratch must fit in P");

__device__ __forceinline__ void wbar() { __syncthreads(); }
__device__ __forceinline__ void wlsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ float wdiv(float a, float b) { return a * fast_rcp(b); }

// partner exchange across the halves of the wavefront: returns (own + partner)
__device__ __forceinline__ float pair_sum(float x) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// the partner lane's value (lane l ^ 32)
__device__ __forceinline__ float pair_other(float x, int h) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(h ? r[0] : r[1]);
}

template <int M>
__device__ __forceinline__ void wpin(float (&x)[M]) {
#pragma unroll
  for (int c = 0; c < M; c++) asm volatile("" : "+v"(x[c]));
}

// rank-2 sweeps (two loads per chunk): a fence every 8 columns keeps the in-flight loads at 16
// VGPRs (at 16 columns the 128-column class spilled 129 VGPRs)
#define CMPC_WSWEEP2_FENCE(c)                               \
  do {                                                      \
    if (((c) & 7) == 4) __builtin_amdgcn_sched_barrier(0);  \
  } while (0)
#define CMPC_WSWEEP_FENCE(c)                                 \
  do {                                                       \
    if (((c) & 15) == 12) __builtin_amdgcn_sched_barrier(0); \
  } while (0)
// the active-set loop's sweeps over LDS vectors: 8 columns between fences for half rows of <= 48
// columns (the 16 loaded values of a 16-column chunk were the loop's register peak: w96 fits
// 96 VGPRs, five waves per SIMD, without spills), 16 otherwise (kGiFence in solve_w)
#define CMPC_WGI_FENCE(c)                                                      \
  do {                                                                         \
    if (((c) & (kGiFence - 1)) == kGiFence - 4) __builtin_amdgcn_sched_barrier(0); \
  } while (0)

// readlane of position i (0 <= i < 64 RQ) of a per-lane array of RQ registers (i uniform)
template <int RQ>
__device__ __forceinline__ float rl_pos(const float (&a)[RQ], int i) {
  float x = 0.f;
  static_for<0, RQ>([&](auto M) {
    constexpr int m = decltype(M)::value;
    if ((i >> 6) == m) x = rl(a[m], i & 63);
  });
  return x;
}
template <int RQ>
__device__ __forceinline__ int rli_pos(const int (&a)[RQ], int i) {
  int x = 0;
  static_for<0, RQ>([&](auto M) {
    constexpr int m = decltype(M)::value;
    if ((i >> 6) == m) x = rli(a[m], i & 63);
  });
  return x;
}

// the lane's thread id, row and half, re-derived where needed (lane_opq): the ids of the top of
// solve_w would otherwise stay live across the unrolled factorisation (at five waves per SIMD
// they were spilled and reloaded from scratch once per pivot step)
#define CMPC_WIDE_IDS()                              \
  const int t = 64 * wave + lane_opq();              \
  const int lane = t & 63;                           \
  const int h = lane >> 5;                           \
  const int r = 32 * wave + (lane & 31);             \
  (void)t;                                           \
  (void)lane;                                        \
  (void)h;                                           \
  (void)r

// Mixed-precision refinement of the converged active set, one step. With the working set W of the
// dual active set, x minimises the fp32-condensed QP on the face {C_W x = b_W}; the minimiser of
// the exact QP on that face is x - J2 J2' r, where r = H x + g is the exact QP's gradient at x and
// J2 the columns of J past the q active positions (Goldfarb-Idnani: J2 J2' = Z (Z' H Z)^-1 Z',
// Z spanning the null space of C_W; C_W J2 = 0, so the step keeps the active constraints). r is
// evaluated in fp64 without H or g (SolverMPC.cpp:806-814):
//   r = H x + g = 2 B_qp' S (A_qp x0 + B_qp x + Q_qp f - X_d) + 2 alpha x,
// by one forward simulation of the discretised model driven by the forces x and one backward
// (adjoint) recursion. A_c^3 = 0, so Adt = I + dt A + dt^2/2 A^2 and Bdt = (dt I + dt^2/2 A +
// dt^3/6 A^2) B_c act as a few sparse operations (ct_ss_mats, SolverMPC.cpp:260-279: A[0:3][6:9]
// = R', A[3:6][9:12] = I, A(11,9) = x_drag, A(11,12) = 1; B[6:9][3b..] = I_w^-1 [r_b]x, B[9:12]
// [3b..] = I / m). The forward pass runs on the deviations z_k+1 = x_k+1 - X_d,k (= e_k, the
// tracking error the cost weighs):
//   z_k+1 = Adt z_k + d_k,  d_k = Bdt u_k + Qdt f + Adt X_d,k-1 - X_d,k  (X_d,-1 = x0, z_0 = 0),
// the backward pass on mu_k = S e_k + Adt' mu_k+1, and the gradient entry of force (k, 3 b + a) is
//   2 ((y_k x r_b)_a + nu_k[9 + a] / m) + 2 alpha x,  nu_k = (dt I + dt^2/2 A' + dt^3/6 A'^2) mu_k,
//   y_k = I_w^-1 nu_k[6:9]  (B_c' nu_k; I_w^-1 symmetric).
// Phases (fp64 scratch in the R^-1 area, 18 + 12 N doubles: R, I_w^-1, then 12 per step):
//   A  thread (k, a), a < 3: t_a = sum_b (r_b x u_b)_a and s_a = sum_b u_b,a of step k;
//   B  thread (k, j), j < 12: d_k,j (w = B_c u_k from t, s);
//   C  wave 0, lane j < 12 owns component j: the two recursions, the cross terms by v_readlane;
//   D  thread (k, i), i < 6: y_k (i < 3) and nu_k[9 + i - 3] / m;
//   E  row r: its gradient entry, then u = J2' r (the columns of J summed over the rows, by DPP
//      within a wave and over the waves in order through the LDS: deterministic) and x -= J2 u.
// The reference's own fp32 pipeline (dense-S GEMMs) is up to ~1e-4 from its QP's exact optimum at
// N >= 16; after this step the solution lands within ~1e-6 of it.
// Phases A-D of wide_refine: the exact QP's gradient at x (xs[] in LDS) into the refinement
// scratch (24 + 12 N doubles in the R^-1 area). (Out of line, the call saved 95 VGPRs of the J
// rows around it: N = 16 10.0 -> 8.8 M QP/s, abr2.)
template <int NV>
__device__ __forceinline__ void refine_residual(const float* __restrict__ rec_in, const KParams& P,
                                                     SharedW<NV>& sh, int wave) {
  using G = WGeo<NV>;
  constexpr int S0 = 24;  // [0..8] R, [9..17] I_w^-1, [18] x_drag, [19] f_est term, [20] x0[12], [21..23] rpy
  // an opaque record pointer keeps its loads (and the arithmetic on them) from being hoisted out
  // of the active-set loop and kept live across every trip. The fp64 scalars come from the kernel
  // arguments (SGPRs) or the LDS, never long-lived VGPRs: the 96-column class has 48 VGPRs beside
  // its J row
#if CMPC_DIAG_REF_LDSREC  // diagnostic: the phases read LDS garbage in place of the record (timing only)
  const float* rec = reinterpret_cast<const float*>(&sh.P[0]);
  (void)rec_in;
#else
  // global address space: the opaque pointer would otherwise be generic (flat loads, which wait
  // on the LDS counter too)
  const gfloat* rec = (const gfloat*)(rec_in);
  asm volatile("" : "+s"(rec));
#endif
  double* scr = reinterpret_cast<double*>(&sh.P[G::O_RINV]);
  const int N = P.N;
  const double dt = P.dt64, dth = P.dth64, dt3 = P.dt3_64;
  const float* xs = sh.xs();
  // ---- A: per step and axis, sum_b r_b x u_b and sum_b u_b; R, I_w^-1 and the instance scalars
  if (!(CMPC_DIAG_REF_SKIP & 1)) {
    const int t = 64 * wave + lane_opq();
    if (t < 3 * N) {
      const int k = t / 3, a = t - 3 * (t / 3);
      const int a1 = (a == 2) ? 0 : a + 1, a2 = (a == 0) ? 2 : a - 1;
      double tc = 0.0, sc = 0.0;
      if constexpr (NV <= CMPC_REF_BFA_MAX) {
        // branch-free over the feet: the lever arms (one global round trip for all eight) and the
        // step's four stance bytes (one LDS word) first, so every x read's address is known up front
        // (per-lane stance branches had serialised a load round trip per foot)
        float ra1[4], ra2[4];
#pragma unroll
        for (int f = 0; f < 4; f++) {
          ra1[f] = rec[CMPC_REC_R + 4 * a1 + f];
          ra2[f] = rec[CMPC_REC_R + 4 * a2 + f];
        }
        const uint32_t st4 = *reinterpret_cast<const uint32_t*>(&sh.stance[4 * k]);
        int v = sh.blkbase[k];
#pragma unroll
        for (int f = 0; f < 4; f++) {
          const bool on = ((st4 >> (8 * f)) & 0xffu) != 0u;
          // (r x u)_a = r_a1 u_a2 - r_a2 u_a1 (a swing foot's reads land on the next foot's
          // variables, or past x's end inside the LDS block, and are discarded)
          const double u0 = xs[v + a], u1 = xs[v + a1], u2 = xs[v + a2];
          const double tf = (double)ra1[f] * u2 - (double)ra2[f] * u1;
          tc += on ? tf : 0.0;
          sc += on ? u0 : 0.0;
          v += on ? 3 : 0;
        }
      } else {  // the per-foot branches (the branch-free form cost config 5 1.3 %, r04_l5)
        int v = sh.blkbase[k];
#pragma unroll
        for (int f = 0; f < 4; f++) {
          if (sh.stance[4 * k + f]) {
            // (r x u)_a = r_a1 u_a2 - r_a2 u_a1
            tc += (double)rec[CMPC_REC_R + 4 * a1 + f] * (double)xs[v + a2] -
                  (double)rec[CMPC_REC_R + 4 * a2 + f] * (double)xs[v + a1];
            sc += (double)xs[v + a];
            v += 3;
          }
        }
      }
      scr[S0 + 12 * k + a] = tc;
      scr[S0 + 12 * k + 3 + a] = sc;
    } else if (t >= G::NT - 18) {
      // R (Eigen toRotationMatrix, RobotState.cpp:36) entry i, or I_w^-1 = R diag(1/I_body) R'
      // entry i - 9 (I_body: RobotState.h:25), in fp64 from the fp32 quaternion
      const int e = t - (G::NT - 18);
      const double qw = rec[CMPC_REC_Q + 0], qx = rec[CMPC_REC_Q + 1], qy = rec[CMPC_REC_Q + 2],
                   qz = rec[CMPC_REC_Q + 3];
      auto rot = [&](int i, int j) -> double {
        const double vi = (i == 0) ? qx : (i == 1) ? qy : qz;
        const double vj = (j == 0) ? qx : (j == 1) ? qy : qz;
        if (i == j) {
          const double o1 = (i == 0) ? qy : qx, o2 = (i == 2) ? qy : qz;
          return 1.0 - 2.0 * (o1 * o1 + o2 * o2);
        }
        const int k = 3 - i - j;
        const double vk = (k == 0) ? qx : (k == 1) ? qy : qz;
        const double sg = ((j - i + 3) % 3 == 1) ? 1.0 : -1.0;  // epsilon_ijk
        return 2.0 * (vi * vj - sg * qw * vk);
      };
      double val;
      if (e < 9) {
        val = rot(e / 3, e - 3 * (e / 3));
      } else {
        const int i = (e - 9) / 3, j = (e - 9) - 3 * ((e - 9) / 3);
        val = rot(i, 0) * (1.0 / 0.07) * rot(j, 0) + rot(i, 1) * (1.0 / 0.26) * rot(j, 1) +
              rot(i, 2) * (1.0 / 0.242) * rot(j, 2);
      }
      scr[e] = val;
    } else if (t == G::NT - 19) {
      const uint32_t flags = __float_as_uint(rec[CMPC_REC_FLAGS]);
      scr[18] = (double)rec[CMPC_REC_XDRAG];
      scr[19] = (flags & 1u) ? (double)rec[CMPC_REC_FEST3] : 0.0;  // Q_qp f (SolverMPC.cpp:808-811)
      scr[20] = (double)vopq(-9.8f);
    } else if (t == G::NT - 20) {
      float rpy[3];  // x0's rpy as the fp32 solve computes it (quat_to_rpy)
      quat_to_rpy(rec, rpy);
      scr[21] = rpy[0];
      scr[22] = rpy[1];
      scr[23] = rpy[2];
    }
  }
  wbar();
  // ---- B: d_k,j = (Bdt u_k + Qdt f)_j + (Adt X_d,k-1)_j - X_d,k,j  (X_d,-1 = x0; component 12 = g)
  if (!(CMPC_DIAG_REF_SKIP & 2)) {
    const double* R = scr;
    const double* Ii = scr + 9;
    const auto traj = rec + CMPC_REC_HDR;
    double dv[2] = {0.0, 0.0};
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int t = 64 * wave + lane_opq() + it * G::NT;
      if (t < 12 * N) {
        const int k = t / 12, j = t - 12 * (t / 12);
        const double* ts = scr + S0 + 12 * k;
        const double xd = scr[18];
        // w = B_c u_k (+ Q_c f: f_est(3) into row 9)
        const double w9 = ts[3] * (1.0 / 12.0) + scr[19];
        double c;
        if (j < 3 || (j >= 6 && j < 9)) {
          // j < 3: dt^2/2 (R' w[6:9])_j; 6..8: dt w_j, w[6:9] = I_w^-1 t
          c = 0.0;
#pragma unroll
          for (int m = 0; m < 3; m++) {
            const double wm = Ii[3 * m] * ts[0] + Ii[3 * m + 1] * ts[1] + Ii[3 * m + 2] * ts[2];
            c += (j < 3) ? dth * R[3 * m + j] * wm : ((j - 6 == m) ? dt * wm : 0.0);
          }
        } else if (j == 3 || j == 9) {
          c = ((j == 3) ? dth : dt) * w9;
        } else if (j == 4 || j == 10) {
          c = ((j == 4) ? dth : dt) * ts[4] * (1.0 / 12.0);
        } else if (j == 5) {
          c = dth * ts[5] * (1.0 / 12.0) + dt3 * xd * w9;
        } else {
          c = dt * ts[5] * (1.0 / 12.0) + dth * xd * w9;
        }
        // X_d,k-1 (x0 for k = 0: [rpy, p, w, v], rpy as quat_to_rpy in fp32)
        auto vprev = [&](int i) -> double {
          if (k > 0) return (double)traj[12 * (k - 1) + i];
          if (i < 3) return scr[21 + i];
          return (double)rec[(i < 6) ? CMPC_REC_P + i - 3 : (i < 9) ? CMPC_REC_W + i - 6 : CMPC_REC_V + i - 9];
        };
        double av = vprev(j);
        if (j < 3) {
          av += dt * (R[j] * vprev(6) + R[3 + j] * vprev(7) + R[6 + j] * vprev(8));
        } else if (j < 6) {
          av += dt * vprev(j + 6);
          if (j == 5) av += dth * (xd * vprev(9) + scr[20]);
        } else if (j == 11) {
          av += dt * (xd * vprev(9) + scr[20]);
        }
        dv[it] = c + av - (double)traj[12 * k + j];
      }
    }
    wbar();  // every read of t, s is done before the step slots are overwritten
#pragma unroll
    for (int it = 0; it < 2; it++) {
      const int t = 64 * wave + lane_opq() + it * G::NT;
      if (t < 12 * N) scr[S0 + t] = dv[it];
    }
  }
  wbar();
  // ---- C: wave 0, lane j < 12 owns component j of z, then of mu. Each step's coefficients are
  // re-read from the LDS (R) and the kernel arguments: nothing but z / mu stays live
  if (wave == 0 && !(CMPC_DIAG_REF_SKIP & 4)) {
    const int j = lane_opq();
    const int jj = (j < 12) ? j : 11;
    const double* R = scr;
    float wf = 0.f;  // P.wts[jj] by uniform selects (a dynamic index would build a VGPR array)
#pragma unroll
    for (int i = 0; i < 12; i++) wf = (jj == i) ? P.wts[i] : wf;
    // forward: z_j += (N1 z)_j + d_k,j   (N1 = Adt - I: rows 0..2 dt R' z[6:9], 3, 4 dt z9, z10,
    // 5 dt z11 + dt^2/2 x_drag z9, 11 dt x_drag z9; z12 = 0)
    double z = 0.0;
    // per-lane coefficients of (z6 .. z11): one branch-free FMA chain per step (per-lane branches
    // measured 5 % slower at N = 16, 3.5 % at config 5: same-box A/B abr1)
    double c6 = 0.0, c7 = 0.0, c8 = 0.0, c9 = 0.0, c10 = 0.0, c11 = 0.0;
    if (jj < 3) { c6 = dt * R[jj]; c7 = dt * R[3 + jj]; c8 = dt * R[6 + jj]; }
    if (jj == 3) c9 = dt;
    if (jj == 4) c10 = dt;
    if (jj == 5) { c11 = dt; c9 = dth * scr[18]; }
    if (jj == 11) c9 = dt * scr[18];
    for (int k = 0; k < N; k++) {
      const double dk = scr[S0 + 12 * k + jj];
      const double z6 = rl_d(z, 6), z7 = rl_d(z, 7), z8 = rl_d(z, 8);
      const double z9 = rl_d(z, 9), z10 = rl_d(z, 10), z11 = rl_d(z, 11);
      z += c6 * z6 + c7 * z7 + c8 * z8 + c9 * z9 + c10 * z10 + c11 * z11 + dk;
      if (j < 12) scr[S0 + 12 * k + j] = (double)wf * z;  // S e_k
    }
    // backward: mu_j += (N1' mu)_j + S e_k,j  (rows 6..8 dt R mu[0:3], 9 dt (mu3 + x_drag mu11) +
    // dt^2/2 x_drag mu5, 10 dt mu4, 11 dt mu5)
    double mu = 0.0;
    double e0 = 0.0, e1 = 0.0, e2 = 0.0, e3 = 0.0, e4 = 0.0, e5 = 0.0, e11 = 0.0;
    if (jj >= 6 && jj < 9) { e0 = dt * R[3 * (jj - 6)]; e1 = dt * R[3 * (jj - 6) + 1]; e2 = dt * R[3 * (jj - 6) + 2]; }
    if (jj == 9) { e3 = dt; e11 = dt * scr[18]; e5 = dth * scr[18]; }
    if (jj == 10) e4 = dt;
    if (jj == 11) e5 = dt;
    for (int k = N - 1; k >= 0; k--) {
      const double sk = scr[S0 + 12 * k + jj];
      const double m0 = rl_d(mu, 0), m1 = rl_d(mu, 1), m2 = rl_d(mu, 2), m3 = rl_d(mu, 3);
      const double m4 = rl_d(mu, 4), m5 = rl_d(mu, 5), m11 = rl_d(mu, 11);
      mu += e0 * m0 + e1 * m1 + e2 * m2 + e3 * m3 + e4 * m4 + e5 * m5 + e11 * m11 + sk;
      if (j < 12) scr[S0 + 12 * k + j] = mu;
    }
  }
  wbar();
  // ---- D: per step, y_k = I_w^-1 nu_k[6:9] and nu_k[9:12] / m into the step's first 6 slots
  if (!(CMPC_DIAG_REF_SKIP & 8)) {
    const int t = 64 * wave + lane_opq();
    double ev = 0.0;
    if (t < 6 * N) {
      const int k = t / 6, i = t - 6 * (t / 6);
      const double* mu = scr + S0 + 12 * k;
      const double* R = scr;
      const double* Ii = scr + 9;
      const double xd = scr[18];
      if constexpr (NV <= CMPC_REF_BFD_MAX) {
        // branch-free over i (one instruction stream per wave; per-row branches cost 1 % at N = 16,
        // r04_k16): i < 3 y_k,i = (I_w^-1 nu[6:9])_i; 3..5 nu[9 + i - 3] / m
        // (scheduling fences between the terms: with every LDS load hoisted to the top, the 30-odd
        // fp64 operands were the refining builds' register peak and spilled the J rows' neighbours)
        const int ic = (i < 3) ? i : 0, il = (i < 3) ? 0 : i - 3;
        const double x3 = (i == 3) ? xd : 0.0;
        const double e2 = (dt * mu[9 + il] + dth * (mu[3 + il] + x3 * mu[11]) + dt3 * x3 * mu[5]) * (1.0 / 12.0);
        __builtin_amdgcn_sched_barrier(0);
        double e1 = 0.0;
#pragma unroll
        for (int m = 0; m < 3; m++) {
          const double nu = dt * mu[6 + m] + dth * (R[3 * m] * mu[0] + R[3 * m + 1] * mu[1] + R[3 * m + 2] * mu[2]);
          e1 += Ii[3 * ic + m] * nu;
          __builtin_amdgcn_sched_barrier(0);
        }
        ev = (i < 3) ? e1 : e2;
      } else {
        if (i < 3) {
#pragma unroll
          for (int m = 0; m < 3; m++) {
            const double nu = dt * mu[6 + m] + dth * (R[3 * m] * mu[0] + R[3 * m + 1] * mu[1] + R[3 * m + 2] * mu[2]);
            ev += Ii[3 * i + m] * nu;
          }
        } else if (i == 3) {
          ev = (dt * mu[9] + dth * (mu[3] + xd * mu[11]) + dt3 * xd * mu[5]) * (1.0 / 12.0);
        } else if (i == 4) {
          ev = (dt * mu[10] + dth * mu[4]) * (1.0 / 12.0);
        } else {
          ev = (dt * mu[11] + dth * mu[5]) * (1.0 / 12.0);
        }
      }
    }
    wbar();
    if (t < 6 * N) scr[S0 + 12 * (t / 6) + t - 6 * (t / 6)] = ev;
  }
  wbar();
}

template <int NV>
__device__ __forceinline__ void wide_refine(const float* __restrict__ rec_in, const KParams& P, SharedW<NV>& sh,
                                            float (&slot)[WGeo<NV>::NH], float& xv, int q, int n, int wave) {
  using G = WGeo<NV>;
  constexpr int NH = G::NH;
  constexpr int NC = (NH + 63) / 64;
  const gfloat* rec = (const gfloat*)(rec_in);
  asm volatile("" : "+s"(rec));
  double* scr = reinterpret_cast<double*>(&sh.P[G::O_RINV]);
  refine_residual<NV>(rec_in, P, sh, wave);
  // ---- E: row r's gradient entry, u = J2' r, x -= J2 u
  float rr = 0.f;
  {
    CMPC_WIDE_IDS();
    if (r < n) {
      const int k = sh.varblk[r], c = sh.varcol[r];
      const int b = c / 3, a = c - 3 * (c / 3);
      const int a1 = (a == 2) ? 0 : a + 1, a2 = (a == 0) ? 2 : a - 1;
      const double* yk = scr + 24 + 12 * k;
      // (y x r_b)_a = y_a1 r_a2 - y_a2 r_a1
      const double cr = yk[a1] * (double)rec[CMPC_REC_R + 4 * a2 + b] - yk[a2] * (double)rec[CMPC_REC_R + 4 * a1 + b];
      rr = (float)(2.0 * (cr + yk[3 + a]) + (double)sopq(P.alpha2) * (double)xv);
    }
  }
  float pa[NC], pb[NC];
#pragma unroll
  for (int m = 0; m < NC; m++) { pa[m] = 0.f; pb[m] = 0.f; }
  if (!(CMPC_DIAG_REF_SKIP & 16)) {
    const int ln = lane_opq();
    static_for<0, NH>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      float v = slot[j] * rr;
      v += dppf<kDppQuadSwap1>(0.f, v);
      v += dppf<kDppQuadSwap2>(0.f, v);
      v += dppf<kDppRowHalfMirror>(0.f, v);
      v += dppf<kDppRowMirror>(0.f, v);
      v += dppf<kDppRowBcast15, 0xa>(0.f, v);  // rows 1 / 3 += row 0 / 2: the two halves' sums
      const float s0 = rl(v, 31), s1 = rl(v, 63);
      if (ln == (j & 63)) { pa[j >> 6] = s0; pb[j >> 6] = s1; }
      if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    });
    // the waves' partials summed in wave order, masked to the columns q <= l < n
    float* ub = sh.vbuf();
    for (int w = 0; w < G::NW; w++) {
      if (wave == w) {
        const bool last = (w == G::NW - 1);
#pragma unroll
        for (int m = 0; m < NC; m++) {
          const int l = 64 * m + ln;
          if (l < NH) {
            float u0 = pa[m] + (w ? ub[l] : 0.f);
            float u1 = pb[m] + (w ? ub[G::HOFF + l] : 0.f);
            if (last) {
              u0 = (l >= q && l < n) ? u0 : 0.f;
              u1 = (NH + l >= q && NH + l < n) ? u1 : 0.f;
            }
            ub[l] = u0;
            ub[G::HOFF + l] = u1;
          }
        }
      }
      wbar();
    }
  }
  {
    CMPC_WIDE_IDS();
    f2v acc = {0.f, 0.f};
    const float* vb = &sh.vbuf()[h * G::HOFF];
#pragma unroll
    for (int j = 0; j < NH; j += 4) {
      const float4 u4 = *reinterpret_cast<const float4*>(vb + j);
      dot4(acc, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3], u4);
      CMPC_WSWEEP_FENCE(j);
    }
    const float dx = pair_sum(acc.x + acc.y);
    if (r < n && !(CMPC_DIAG_REF_SKIP & 16)) xv -= dx;
  }
}

template <int NV, bool REFINE>
__device__ __forceinline__ void solve_w(const float* __restrict__ rec, const KParams& P,
                                        SharedW<NV>& sh, float* __restrict__ fout,
                                        uint8_t* __restrict__ st_out, int32_t* __restrict__ it_out) {
  using G = WGeo<NV>;
  constexpr int NH = G::NH;
  constexpr int RQ = G::RQ;
  constexpr int kGiFence = (NH <= 48) ? 8 : 16;
  const int t = tid_opq();  // opaque: nothing lane-dependent is hoisted out of the persistent loop
  const int lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int h = lane >> 5;
  const int r = 32 * wave + (lane & 31);   // matrix row of this lane (rows >= NV: idle lanes)
  const int N = P.N;
  // ---- stage the record in LDS (16-B loads, one HBM round trip for the whole prep)
  {
    const float4* src = reinterpret_cast<const float4*>(rec);
    float4* dst = reinterpret_cast<float4*>(&sh.P[W_OFF_REC]);
    for (int i = t; i < (P.rec_words >> 2); i += G::NT) dst[i] = src[i];
  }
  wbar();
  const float* srec = &sh.P[W_OFF_REC];
  // ---- stance table + elimination (SolverMPC.cpp:869-894); every wave compacts, wave 0 stores
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(srec + CMPC_REC_HDR + 12 * N);
  int nfs = 0;
  unsigned long long msk0 = 0ull, msk1 = 0ull;
  for (int c0 = 0; c0 < 4 * N; c0 += 64) {
    const int s = c0 + lane;
    float ub = 0.f;
    bool f = false;
    if (s < 4 * N) {
      ub = (float)gait[s] * P.f_max;
      f = !(ub < 0.01f && ub > -0.01f);
      if (wave == 0) sh.stance[s] = f ? 1 : 0;
    }
    const unsigned long long m = __ballot(f);
    if (c0 == 0) msk0 = m; else msk1 = m;
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (f && wave == 0) {
      sh.sfs[nfs + pre] = s;
      sh.sub[nfs + pre] = ub;
    }
    nfs += __popcll(m);
  }
  const int n = 3 * nfs;
  if (n > NV) {  // not this class's instance (classify guarantees it never happens)
    if (t == 0) { st_out[0] = CMPC_BAD_INPUT; if (it_out) it_out[0] = 0; }
    return;
  }
  wbar();
  {
    int kb = 0, kc = 0;
    if (t < n) {
      const int fs = sh.sfs[t / 3];
      kb = fs >> 2;
      kc = 3 * (fs & 3) + t % 3;
    }
    sh.varblk[t] = (unsigned char)kb;
    sh.varcol[t] = (unsigned char)kc;
    if (t <= N) {
      const int b0 = 4 * t, b1 = 4 * t - 64;
      const unsigned long long lo = (b0 >= 64) ? msk0 : (msk0 & ((1ull << b0) - 1ull));
      const unsigned long long hi = (b1 <= 0) ? 0ull : (msk1 & ((1ull << b1) - 1ull));
      sh.blkbase[t] = 3 * (__popcll(lo) + __popcll(hi));
    }
    for (int i = t; i < 6 * nfs; i += G::NT) sh.cflag[i] = 0;
  }
  Model md;
  make_model(srec, P.dt, md);
  make_bdt<G::NT>(srec, md, t, sh.BdtT());
  wbar();
  if (t < N) {
    float e[13];
    state_error(srec, md, t, srec + CMPC_REC_HDR + 12 * t, e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.P[W_OFF_E + 16 * t + j] = e[j];
  }
  wbar();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  // gradient recursion ze_i = S e_i + Adt' ze_{i+1} (uniform; thread j < 13 stores component j)
  {
    float ze[13];
#pragma unroll
    for (int j = 0; j < 13; j++) ze[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      float e[13];
#pragma unroll
      for (int j = 0; j < 13; j++) e[j] = sh.P[W_OFF_E + 16 * i + j];
      recur(md, wts, e, ze);
      float mine = 0.f;
#pragma unroll
      for (int j = 0; j < 13; j++) mine = (t == j) ? ze[j] : mine;
      if (t < 13) sh.P[W_OFF_ZE + 16 * i + t] = mine;
    }
  }
  wbar();

  // ---- condensation: row r's lanes build H[r][w], w >= r (half h takes every other w of a
  // block), into packed upper rows of P; both compute the gradient g_r
  const bool real = r < n;
  const int rr = (r < NV) ? r : 0;
  float gv;
  {
    const int kv = real ? sh.varblk[r] : 0;
    const int cv = real ? sh.varcol[r] : 0;
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = real ? sh.BdtT()[cv][j] : 0.f;
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.P[W_OFF_ZE + 16 * kv + j];
      gv = real ? 2.f * dot13(b, zk) : 0.f;  // qg = 2 B_qp' S (A_qp x0 + Q_qp f - X_d)
    }
    wbar();  // every ZE read is done before P is overwritten
    const int myrow = G::tri(rr);
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    // (stopping each wavefront below the smallest block of its rows, whose steps build nothing,
    // measured 0.5-1 % slower on every workload: profiles/r03_ab/r03_o)
    for (int i = N - 1; i >= 0; i--) {
      // z_i = S Adt^{i-kv} b_r + Adt' z_{i+1}  (the S term only for i >= kv)
      const bool act = real && (i >= kv);
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = act ? fmaf(k2, u2[j], fmaf(k, u1[j], b[j])) : 0.f;
      recur(md, wts, gk, z);
      const int wb = __builtin_amdgcn_readfirstlane(sh.blkbase[i]);
      const int we = __builtin_amdgcn_readfirstlane(sh.blkbase[i + 1]);
      // half h takes every other column of the step (the per-foot unrolled form of class 1, with
      // both halves computing every column, measured 2-5 % slower at N = 16 / 20)
      for (int w0 = wb; w0 < we; w0 += 2) {
        const int w = w0 + h;
        const int cw = sh.varcol[w];
        float bw[13];
#pragma unroll
        for (int j = 0; j < 13; j++) bw[j] = sh.BdtT()[cw][j];
        float val = 2.f * dot13(bw, z);
        if (w == r) val += P.alpha2;  // qH = 2 (B'SB + alpha I), SolverMPC.cpp:806
        if (act && w < we && w >= r) sh.P[myrow + w] = val;
      }
    }
  }
  wbar();

  // ---- my half-row of H into registers: columns c = 2 j + h (identity padding)
  float slot[NH];
  float gb = gv;  // border: g_r, then y_r (both halves keep it)
  {
    const int myrow = G::tri(rr);
    static_for<0, NH>([&](auto J) {
      constexpr int j = decltype(J)::value;
      const int c = 2 * j + h;
      const int addr = (c >= rr) ? myrow + c : G::tri(c) + rr;
      const float x = sh.P[addr];
      slot[j] = (real && c < n) ? x : ((c == r) ? 1.f : 0.f);
      if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
  }
  wbar();

  // ---- bordered Cholesky [H | g]: pivot column k = register k/2 of half k%2 of every row,
  // published into P's row k (even / odd segments), one s_barrier per step
  int status = CMPC_OK;
  float my_inv = 1.f;
#if CMPC_DIAG_STOP != 3  // diagnostic build 3: stop after the condensation and the H-row load
#if CMPC_WIDE_CHOL2
  // Two pivots per step (k even, k+1: register k/2 of half 0 and of half 1 of every row), one
  // s_barrier per step instead of per pivot. Each lane publishes its own pivot column entry
  // (half 0: raw column k, half 1: raw column k+1), then every row applies both steps as one
  // rank-2 sweep over the two raw columns:
  //   beta = H[k+1][k] / d_k, d_k+1 = H[k+1][k+1] - beta H[k+1][k], s1 = H[r][k+1] - beta H[r][k],
  //   a1 = -s1 / d_k+1, a0 = -H[r][k] / d_k - beta a1   (coefficient of the raw column k)
  // J = L^-T below applies the same beta to the stored raw column k+1. Odd n: the last step's
  // second pivot is the identity padding row.
  static_for<0, NV / 2>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value, k1 = k + 1;
    constexpr int kj = k >> 1;
    constexpr int j0 = G::j0(k);  // = j0(k + 1)
    constexpr int base = G::fbase(k), base1 = G::fbase(k1);
    constexpr int st = G::seg(k);  // = seg(k + 1)
    if (k < n) {
      // row / half re-derived from an opaque thread index each step: a row index kept live
      // across the unrolled steps was spilled at five waves per SIMD (wide 96) and reloaded from
      // scratch twice per step
      CMPC_WIDE_IDS();
      const float mine = slot[kj];
      const float other = pair_other(mine, h);
      const float hk = h ? other : mine;    // H[r][k]
      const float hk1 = h ? mine : other;   // H[r][k+1]
      // two stores with constant bases (one store with a per-lane base select made the 128-column
      // class spill 129 VGPRs)
      if (h == 0 && r >= 2 * j0 && r < NV) sh.P[base + (r & 1) * st + (r >> 1) - j0] = (r >= k) ? mine : 0.f;
      if (h == 1 && r >= 2 * j0 && r < NV) sh.P[base1 + (r & 1) * st + (r >> 1) - j0] = (r >= k1) ? mine : 0.f;
      if (h == 0 && (r == k || r == k1)) sh.gbuf()[r] = gb;
      wbar();
      float d0 = sh.P[base + kj - j0];
      const float h10 = sh.P[base + st + kj - j0];
      const float d1r = sh.P[base1 + st + kj - j0];
      const float g0 = sh.gbuf()[k], g1 = sh.gbuf()[k1];
      if (!(d0 > 0.f)) { status = CMPC_NOT_PD; d0 = 1e-30f; }
      const float i0 = __builtin_amdgcn_rsqf(d0);  // raw v_rsq: d is a normal positive pivot
      const float beta = h10 * (i0 * i0);
      float d1 = fmaf(-h10, beta, d1r);
      if (!(d1 > 0.f)) { status = CMPC_NOT_PD; d1 = 1e-30f; }
      const float i1 = __builtin_amdgcn_rsqf(d1);
      if (r == k) { my_inv = i0; if (h == 0) sh.ibuf()[k] = i0; }
      if (r == k1) { my_inv = i1; if (h == 0) sh.ibuf()[k1] = i1; }
      const float s1 = fmaf(-hk, beta, hk1);
      const float a1 = (r > k1 && r < NV) ? -s1 * (i1 * i1) : 0.f;
      const float a0 = (r > k && r < NV) ? fmaf(-a1, beta, -hk * (i0 * i0)) : 0.f;
      // a wavefront whose rows are all factored (r <= k) or all padding (r >= n) has a0 = a1 = 0:
      // it skips the sweep (scalar branch; 20 % of the sweep reads at NV = 120, more with more waves)
      if (CMPC_WIDE_SKIP == 0 || (32 * wave + 31 > k && 32 * wave < n)) {
        const float* prow0 = &sh.P[base + h * st - j0];
        const float* prow1 = &sh.P[base1 + h * st - j0];
#pragma unroll
        for (int j = j0; j < NH; j += 4) {
          const float4 r0 = *reinterpret_cast<const float4*>(prow0 + j);
          const float4 r1 = *reinterpret_cast<const float4*>(prow1 + j);
          axpy4(a0, r0, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
          axpy4(a1, r1, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
          CMPC_WSWEEP2_FENCE(j);
        }
        gb = fmaf(a1, g1, fmaf(a0, g0, gb));
      }
      wpin(slot);
    }
  });
#else
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int kj = k >> 1, kh = k & 1;
    constexpr int j0 = G::j0(k);
    constexpr int base = G::fbase(k);
    constexpr int st = G::seg(k);
    if (k < n) {
      const float mine = slot[kj];
      const float other = pair_other(mine, h);
      const float hrk = (h == kh) ? mine : other;          // H[r][k] of the trailing matrix
      if (h == kh && r >= 2 * j0 && r < NV)
        sh.P[base + (r & 1) * st + (r >> 1) - j0] = (r >= k) ? mine : 0.f;
      if (r == k && h == 0) sh.gbuf()[k] = gb;
      wbar();
      float d = sh.P[base + kh * st + kj - j0];
      if (!(d > 0.f)) { status = CMPC_NOT_PD; d = 1e-30f; }
      const float inv = __builtin_amdgcn_rsqf(d);  // raw v_rsq: d is a normal positive pivot
      if (r == k) { my_inv = inv; if (h == 0) sh.ibuf()[k] = inv; }
      const float a = (r > k && r < NV) ? -hrk * (inv * inv) : 0.f;
      const float* prow = &sh.P[base + h * st - j0];
#pragma unroll
      for (int j = j0; j < NH; j += 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(prow + j);
        axpy4(a, r4, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
        CMPC_WSWEEP_FENCE(j);
      }
      gb = fmaf(a, sh.gbuf()[k], gb);
      wpin(slot);
    }
  });
#endif
#endif  // CMPC_DIAG_STOP != 3
  float yv;
  {
    CMPC_WIDE_IDS();
    yv = (r < n) ? gb * my_inv : 0.f;  // L y = g
    if (h == 0 && r < NV) sh.ybuf(r & 1)[r >> 1] = yv;
  }
  wbar();

#if CMPC_DIAG_STOP != 1 && CMPC_DIAG_STOP != 3  // diagnostic builds: stop after the Cholesky (1) / after J (2)
  // ---- J = L^-T: row r solves L x = e_r over its half of the columns (LDS reads only; the
  // pivot value x_k lives in the half holding column k: one partner exchange per step)
  {
    // the unit row from an opaque thread index: with the plain (h, r) the NH per-lane column
    // ids 2 j + h are shared (CSE) with the H-row load above and stay live across the whole
    // Cholesky (64 VGPRs at NV = 128)
    const int to = 64 * wave + lane_opq();
    const int lr = ((to & 63) >> 5) - 32 * (to >> 6) - (to & 31);  // h - r
    static_for<0, NH>([&](auto J) {
      constexpr int j = decltype(J)::value;
      slot[j] = (lr == -2 * j) ? 1.f : 0.f;
    });
  }
#if CMPC_WIDE_J2
  // two columns per step, as the factorisation (the stored column k+1 is raw: beta corrects it)
  static_for<0, NV / 2>([&](auto KB) {
    constexpr int k = 2 * decltype(KB)::value, k1 = k + 1;
    constexpr int kj = k >> 1;
    constexpr int j0 = G::j0(k);
    constexpr int base = G::fbase(k), base1 = G::fbase(k1);
    constexpr int st = G::seg(k);
    // rows r > k + 1 have x_k = x_k+1 = 0 (L is lower triangular): a wavefront whose rows all lie
    // past the pivot pair skips the step (its slot k stays the +0 the step would store)
    if (k < n && (CMPC_WIDE_SKIP == 0 || k1 >= 32 * wave)) {
      wlsync();
      const int h = (lane_opq() >> 5) & 1;
      const float i0 = sh.ibuf()[k], i1 = sh.ibuf()[k1];
      const float h10 = sh.P[base + st + kj - j0];
      const float beta = h10 * (i0 * i0);
      const float mine = slot[kj];
      const float other = pair_other(mine, h);
      const float x0 = (h ? other : mine) * i0;
      const float x1 = fmaf(-h10 * i0, x0, h ? mine : other) * i1;
      const float a1 = -x1 * i1;
      const float a0 = fmaf(-a1, beta, -x0 * i0);
      const float* prow0 = &sh.P[base + h * st - j0];
      const float* prow1 = &sh.P[base1 + h * st - j0];
#pragma unroll
      for (int j = j0; j < NH; j += 4) {
        const float4 r0 = *reinterpret_cast<const float4*>(prow0 + j);
        const float4 r1 = *reinterpret_cast<const float4*>(prow1 + j);
        axpy4(a0, r0, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
        axpy4(a1, r1, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
        CMPC_WSWEEP2_FENCE(j);
      }
      slot[kj] = h ? x1 : x0;
      wpin(slot);
    }
  });
#else
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int kj = k >> 1, kh = k & 1;
    constexpr int j0 = G::j0(k);
    constexpr int base = G::fbase(k);
    constexpr int st = G::seg(k);
    if (k < n) {
      wlsync();
      const float inv = sh.ibuf()[k];
      const float mine = slot[kj];
      const float other = pair_other(mine, h);
      const float xk = ((h == kh) ? mine : other) * inv;
      const float a = -xk * inv;
      const float* prow = &sh.P[base + h * st - j0];
#pragma unroll
      for (int j = j0; j < NH; j += 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(prow + j);
        axpy4(a, r4, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
        CMPC_WSWEEP_FENCE(j);
      }
      if (h == kh) slot[kj] = xk;
      wpin(slot);
    }
  });

#endif
#endif
  // ---- unconstrained minimiser x = -J y
  float xv;
  {
    CMPC_WIDE_IDS();
    f2v xacc = {0.f, 0.f};
    const float* yb = sh.ybuf(h);
#pragma unroll
    for (int j = 0; j < NH; j += 4) {
      const float4 y4 = *reinterpret_cast<const float4*>(yb + j);
      dot4(xacc, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3], y4);
      CMPC_WSWEEP_FENCE(j);
    }
    const float xs2 = pair_sum(xacc.x + xacc.y);
    xv = (r < n) ? -xs2 : 0.f;
  }
  wbar();  // the factor rows in P are dead from here; P holds R

  // ---- Goldfarb-Idnani dual active set on the friction pyramids, J's columns relabelled
  // l = h NH + j. One flat loop, one active-set step per trip; R in P, maintained by wave 0
  const float mui = P.mu_inv;
  const float fnorm = rsqrtf(mui * mui + 1.f);
  int q = 0;
  bool rinv_ok = true;  // R^-1 kept beside R (wave-uniform)
  int iters = 0;
  float u_a[RQ], r_a[RQ];
  int a_a[RQ];
#pragma unroll
  for (int m = 0; m < RQ; m++) { u_a[m] = 0.f; r_a[m] = 0.f; a_a[m] = 0; }
  int p = -1;
  Cons cp{};
  float up = 0.f;
  int it_refined = -1;  // active-set trips at the last refinement
  int passes = 0;       // refinements so far
  if (status == CMPC_OK && CMPC_DIAG_STOP == 0) {
   for (;;) {
    for (;;) {
      wpin(slot);
      CMPC_WIDE_IDS();
      if (p < 0) {
        if (h == 0 && r < NV) sh.xs()[r] = xv;
        wbar();
        // most violated constraint (normalised slack); every wave scans the same foot-steps
        float best = 0.f, xm = 0.f;
        int bid = kNoneW;
#pragma unroll
        for (int m = 0; m < 2; m++) {
          const int s = lane + 64 * m;
          if (s < nfs) {
            const float fx = sh.xs()[3 * s], fy = sh.xs()[3 * s + 1], fz = sh.xs()[3 * s + 2];
            xm = fmaxf(xm, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz))));
            float sl[6];
            sl[0] = (mui * fx + fz) * fnorm;
            sl[1] = (-mui * fx + fz) * fnorm;
            sl[2] = (mui * fy + fz) * fnorm;
            sl[3] = (-mui * fy + fz) * fnorm;
            sl[4] = fz;
            sl[5] = sh.sub[s] - fz;
#pragma unroll
            for (int u = 0; u < 6; u++)
              if (!sh.cflag[6 * s + u] && sl[u] < best) { best = sl[u]; bid = 6 * s + u; }
          }
        }
        const float xmax = wave_max(xm);
        wave_argmin(best, bid);
        // after a refinement x is the exact QP's optimum on the working set up to fp32 rounding:
        // the constraints are held to that (a face the fp32 solve left for a nearly active
        // constraint shows here as a violation of ~1e-6 x_max, and joins the working set)
        const float tol = (passes ? CMPC_REFINE_TOL : 1e-5f) * fmaxf(1.f, xmax);
        if (bid == kNoneW || best >= -tol) break;
        p = __builtin_amdgcn_readfirstlane(bid);
        cp = decode_cons(p, mui, sh.sub[p / 6]);
        cp.bp = rfl(cp.bp);  // uniform: SGPRs, not loop-carried VGPRs
        up = 0.f;
      }
      if (++iters > P.max_iter + 2 * n) { status = CMPC_MAX_ITER; break; }
#if CMPC_WIDE_PRIO > 0 && CMPC_TRIP_PRIO_AT > 0
      if (iters == CMPC_TRIP_PRIO_AT) __builtin_amdgcn_s_setprio(CMPC_WIDE_TRIP_PRIO);
#endif
      // d = J' n+ : rows ia, iz of J through LDS (logical order)
      if (r == cp.ia && cp.ia != cp.iz) {
#pragma unroll
        for (int j = 0; j < NH; j++) sh.bufA()[h * G::HOFF + j] = slot[j];
      }
      if (r == cp.iz) {
#pragma unroll
        for (int j = 0; j < NH; j++) sh.bufB()[h * G::HOFF + j] = slot[j];
      }
      if (h == 0 && r < NV) sh.xs()[r] = xv;
      wbar();
      // thread t < NV: logical column t
      float dv = 0.f, dm = 0.f;
      if (t < NV) {
        const int li = lidx<NV>(t);
        dv = (cp.ia != cp.iz) ? fmaf(cp.ca, sh.bufA()[li], cp.cb * sh.bufB()[li]) : cp.cb * sh.bufB()[li];
        dm = (t >= q) ? dv : 0.f;
        sh.vbuf()[li] = dm;
        sh.dfull()[t] = dv;
      }
      {
        const float dw = wave_sum(dv * dv);
        if (lane == 0) sh.redf[wave] = dw;
      }
      const float spv = fmaf(cp.ca, sh.xs()[cp.ia], fmaf(cp.cb, sh.xs()[cp.iz], -cp.bp));
      wbar();
      // z_r = J_r . dm (primal step direction), zn = |dm|^2 = z' n+, dn = |d|^2
      float zv, zn, dn = 0.f;
      {
        f2v zacc = {0.f, 0.f}, nacc = {0.f, 0.f};
        const float* vb = &sh.vbuf()[h * G::HOFF];
#pragma unroll
        for (int j = 0; j < NH; j += 4) {
          const float4 m4 = *reinterpret_cast<const float4*>(vb + j);
          W_DOT(zacc, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3], m4);
          W_DOT(nacc, m4.x, m4.y, m4.z, m4.w, m4);
          CMPC_WGI_FENCE(j);
        }
        zv = pair_sum(zacc.x + zacc.y);
        zn = pair_sum(nacc.x + nacc.y);
        // materialise both sums here: otherwise the FMAs sink below wave 0's back substitution
        // and the NV/2 loaded values of vbuf stay live across it
        asm volatile("" : "+v"(zv), "+v"(zn));
#pragma unroll
        for (int w = 0; w < G::NW; w++) dn += sh.redf[w];
      }
      // r = R^-1 d1 by back substitution (wave 0), then the dual step t1 = min u_j / r_j
      if (wave == 0 && rinv_ok) {
        // R^-1 kept (only adds so far, q <= QI): r = R^-1 d1 as a matvec, four columns per trip
        float ra[RQ];
#pragma unroll
        for (int m = 0; m < RQ; m++) ra[m] = 0.f;
        int j = 0;
        for (; j + 4 <= q; j += 4) {
          const float4 d4 = *reinterpret_cast<const float4*>(&sh.dfull()[j]);
          const float dj[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const int off = G::O_RINV + rcol_w(j + e);
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int pos = lane + 64 * m;
              const float x = sh.P[off + ((pos <= j + e) ? pos : j + e)];
              ra[m] = fmaf((pos <= j + e) ? x : 0.f, dj[e], ra[m]);
            }
          }
        }
        for (; j < q; j++) {
          const int off = G::O_RINV + rcol_w(j);
          const float dj = sh.dfull()[j];
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int pos = lane + 64 * m;
            const float x = sh.P[off + ((pos <= j) ? pos : j)];
            ra[m] = fmaf((pos <= j) ? x : 0.f, dj, ra[m]);
          }
        }
#pragma unroll
        for (int m = 0; m < RQ; m++) r_a[m] = (lane + 64 * m < q) ? ra[m] : 0.f;
      }
      if (wave == 0 && !rinv_ok) {
        float acc[RQ];
#pragma unroll
        for (int m = 0; m < RQ; m++) {
          acc[m] = (lane + 64 * m < NV) ? sh.dfull()[(lane + 64 * m) < NV ? lane + 64 * m : 0] : 0.f;
          r_a[m] = 0.f;
        }
#if CMPC_WIDE_WAVES_PER_EU <= 4
        // software-pipelined: the LDS reads of step i - 1 are issued before step i's chain (the
        // five-waves-per-SIMD builds keep the plain loop: 96 VGPRs leave no room for it)
        float pd = 1.f, pv[RQ];
#pragma unroll
        for (int m = 0; m < RQ; m++) pv[m] = 0.f;
        if (q > 0) {
          const int off = rcol_w(q - 1);
          pd = sh.P[off + q - 1];
#pragma unroll
          for (int m = 0; m < RQ; m++) pv[m] = (lane + 64 * m < q - 1) ? sh.P[off + lane + 64 * m] : 0.f;
        }
        for (int i = q - 1; i >= 0; i--) {
          float pd_n = 1.f, pv_n[RQ];
#pragma unroll
          for (int m = 0; m < RQ; m++) pv_n[m] = 0.f;
          if (i > 0) {
            const int offn = rcol_w(i - 1);
            pd_n = sh.P[offn + i - 1];
#pragma unroll
            for (int m = 0; m < RQ; m++) pv_n[m] = (lane + 64 * m < i - 1) ? sh.P[offn + lane + 64 * m] : 0.f;
          }
          const float ri = wdiv(rl_pos<RQ>(acc, i), pd);
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int pos = lane + 64 * m;
            if (pos < i) acc[m] = fmaf(-pv[m], ri, acc[m]);
            r_a[m] = (pos == i) ? ri : r_a[m];
            pv[m] = pv_n[m];
          }
          pd = pd_n;
        }
#else
        for (int i = q - 1; i >= 0; i--) {
          const int off = rcol_w(i);
          const float ri = wdiv(rl_pos<RQ>(acc, i), sh.P[off + i]);
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int pos = lane + 64 * m;
            if (pos < i) acc[m] = fmaf(-sh.P[off + pos], ri, acc[m]);
            r_a[m] = (pos == i) ? ri : r_a[m];
          }
        }
#endif
      }
      if (wave == 0) {
        float t1w = kBigF;
        int kw = kNoneW;
#pragma unroll
        for (int m = 0; m < RQ; m++) {
          const int pos = lane + 64 * m;
          if (pos < q && r_a[m] > 0.f) {
            const float th = fmaxf(wdiv(u_a[m], r_a[m]), 0.f);
            if (th < t1w) { t1w = th; kw = pos; }
          }
        }
        wave_argmin(t1w, kw);
        if (lane == 0) { sh.redf[8] = t1w; sh.redi[8] = kw; }
      }
      wbar();
      const float t1 = sh.redf[8];
      const int kk = __builtin_amdgcn_readfirstlane(sh.redi[8]);
      const bool zero_step = !(zn > 1e-9f * dn);
      const float t2 = zero_step ? kBigF : -wdiv(spv, zn);
      const float tt = fminf(t1, t2);
      if (tt >= kBigF) { status = CMPC_INFEASIBLE; break; }
      if (wave == 0) {
#pragma unroll
        for (int m = 0; m < RQ; m++)
          if (lane + 64 * m < q) u_a[m] = fmaf(-tt, r_a[m], u_a[m]);
      }
      up = rfl(up + tt);
      if (!zero_step) xv = fmaf(tt, zv, xv);
      const bool add = !zero_step && t2 <= t1;
      const bool add_u = __builtin_amdgcn_readfirstlane((int)add) != 0;  // wave-uniform copy
      float beta = 0.f;
      bool seam = false;   // a drop whose Givens chain crosses into half 1
      if (add) {
        // ---- add p: Householder reflection on logical columns q.., R gains column (d1, -sgn ts)
        const float ts = sqrtf(zn);
        const float dq = sh.dfull()[q];
        const float sgn = (dq >= 0.f) ? 1.f : -1.f;
        beta = fast_rcp(ts * (ts + fabsf(dq)));  // 2 / (w'w)
        if (t < NV) {
          sh.vbuf()[lidx<NV>(t)] = (t == q) ? dq + sgn * ts : dm;
          const int offq = rcol_w(q);
          if (t < q) sh.P[offq + t] = dv;
          if (t == q) sh.P[offq + q] = -sgn * ts;
        }
        if (wave == 0) {
          // R^-1 gains the column (-r / rho, 1 / rho), rho = R's new diagonal
          const bool keep = rinv_ok && q < G::QI;
          const float irho = 1.f / (-sgn * ts);
          const int offi = G::O_RINV + rcol_w(q);
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int pos = lane + 64 * m;
            if (lane + 64 * m == q) { u_a[m] = up; a_a[m] = p; }
            if (keep && pos < q) sh.P[offi + pos] = -r_a[m] * irho;
            if (keep && pos == q) sh.P[offi + q] = irho;
          }
        }
        if (q >= G::QI) rinv_ok = false;
        if (t == 0) sh.cflag[p] = 1;
      } else {
        // ---- drop active constraint kk: shift positions kk+1..q-1 down, remove column kk of R,
        // re-triangularise rows kk..q-1 with Givens rotations (wave 0, in place)
        const int k = kk;
        seam = (q > NH);
        if (t < NV) {
          sh.vbuf()[lidx<NV>(t)] = 0.f;
          if (t < k || t > q - 2)
            *reinterpret_cast<float2*>(&sh.cs()[2 * t + (t >= NH ? 4 : 0)]) = make_float2(vopq(1.f), vopq(0.f));
        }
        if (wave == 0) {
          const int ak = rli_pos<RQ>(a_a, k);
          if (lane == 0) sh.cflag[ak] = 0;
          // position j <- j + 1 for k <= j < q - 1
          int a_nx[RQ];
          float u_nx[RQ];
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            a_nx[m] = lane_next_i(a_a[m], a_a[m]);
            u_nx[m] = lane_next(u_a[m], u_a[m]);
            if (m + 1 < RQ) {
              const int a0 = rli(a_a[m + 1 < RQ ? m + 1 : m], 0);
              const float u0 = rl(u_a[m + 1 < RQ ? m + 1 : m], 0);
              if (lane == 63) { a_nx[m] = a0; u_nx[m] = u0; }
            }
          }
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int pos = lane + 64 * m;
            if (pos >= k && pos < q - 1) { a_a[m] = a_nx[m]; u_a[m] = u_nx[m]; }
          }
          // new column c (k <= c <= q-2) = old column c+1; lane handles c = lane + 64 m. Every
          // read of an old entry precedes, in this wavefront's LDS order, the write reusing it
          float top[RQ];
          bool in_c[RQ];
#pragma unroll
          for (int m = 0; m < RQ; m++) {
            const int c = lane + 64 * m;
            in_c[m] = c >= k && c <= q - 2;
            top[m] = in_c[m] ? sh.P[rcol_w(c + 1) + k] : 0.f;
          }
          wlsync();
          for (int rw = 0; rw < k; rw++) {
            float xr[RQ];
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int c = lane + 64 * m;
              xr[m] = in_c[m] ? sh.P[rcol_w(c + 1) + rw] : 0.f;
            }
            wlsync();
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int c = lane + 64 * m;
              if (in_c[m]) sh.P[rcol_w(c) + rw] = xr[m];
            }
            wlsync();
          }
          for (int j = k; j <= q - 2; j++) {
            float bot[RQ];
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int c = lane + 64 * m;
              bot[m] = (in_c[m] && c >= j) ? sh.P[rcol_w(c + 1) + j + 1] : 0.f;
            }
            wlsync();
            const float a0 = rl_pos<RQ>(top, j), b0 = rl_pos<RQ>(bot, j);
            const float hh = sqrtf(a0 * a0 + b0 * b0);
            float cc = 1.f, sn = 0.f;
            if (hh > 0.f) { const float ih = fast_rcp(hh); cc = a0 * ih; sn = b0 * ih; }
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int c = lane + 64 * m;
              if (in_c[m] && c >= j) {
                sh.P[rcol_w(c) + j] = fmaf(cc, top[m], sn * bot[m]);
                top[m] = fmaf(-sn, top[m], cc * bot[m]);
              }
            }
            if (lane == 0)
              *reinterpret_cast<float2*>(&sh.cs()[2 * j + (j >= NH ? 4 : 0)]) = make_float2(cc, sn);
            wlsync();
          }
          // R^-1 through the drop: R'^-1 = E' R^-1 G[:, 0:q-1] (row k removed, the rotations of
          // the chain above applied to its columns as to J's, the last column dropped; class 1
          // derives it). Lane row i = lane + 64 m streams through the chain with one carried value
          if (rinv_ok) {
#pragma unroll
            for (int m = 0; m < RQ; m++) {
              const int i = lane + 64 * m;
              const bool live = i < q && i != k;
              const int i2 = (i > k) ? i - 1 : i;
              const int j0 = (i > k) ? i - 1 : k;  // first rotation that touches row i
              float carry = (live && j0 >= i) ? sh.P[G::O_RINV + rcol_w(j0) + i] : 0.f;
              for (int jj = k; jj <= q - 2; jj++) {
                const float2 cs2 = *reinterpret_cast<const float2*>(&sh.cs()[2 * jj + (jj >= NH ? 4 : 0)]);
                const float b = (live && jj >= j0) ? sh.P[G::O_RINV + rcol_w(jj + 1) + i] : 0.f;
                wlsync();
                if (live && jj >= j0) {
                  sh.P[G::O_RINV + rcol_w(jj) + i2] = fmaf(cs2.x, carry, cs2.y * b);
                  carry = fmaf(-cs2.y, carry, cs2.x * b);
                }
              }
              wlsync();
            }
          }
        }
      }
      wbar();
      // J <- J (I - beta w w'): tw = J_r . w over both halves, J_r -= beta tw w (no-op on a drop)
      {
        f2v tacc = {0.f, 0.f};
        const float* vb = &sh.vbuf()[h * G::HOFF];
#pragma unroll
        for (int j = 0; j < NH; j += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(vb + j);
          W_DOT(tacc, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3], w4);
          CMPC_WGI_FENCE(j);
        }
        const float bt = -beta * pair_sum(tacc.x + tacc.y);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < NH; j += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(vb + j);
          axpy4(bt, w4, slot[j + 0], slot[j + 1], slot[j + 2], slot[j + 3]);
          CMPC_WGI_FENCE(j);
        }
      }
      // J columns (l, l+1) <- Givens chain, ascending l (identity on an add)
      // (drops only: on an add every rotation is the identity)
      const float* csb = &sh.cs()[h * (2 * NH + 4)];
      if (add_u) {
      } else if (!seam) {
        // every rotation lies in half 0 (active set <= NV/2); half 1 reads identities
        static_for<0, NH - 1>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          const float2 c2 = *reinterpret_cast<const float2*>(csb + 2 * j);
          const float x0 = slot[j], x1 = slot[j + 1];
          slot[j] = fmaf(c2.x, x0, c2.y * x1);
          slot[j + 1] = fmaf(-c2.y, x0, c2.x * x1);
          if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
      } else {
        // half 0's chain, the seam rotation (logical NH-1, NH), then half 1's chain
        static_for<0, NH - 1>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          float2 c2 = *reinterpret_cast<const float2*>(csb + 2 * j);
          if (h) c2 = make_float2(1.f, 0.f);
          const float x0 = slot[j], x1 = slot[j + 1];
          slot[j] = fmaf(c2.x, x0, c2.y * x1);
          slot[j + 1] = fmaf(-c2.y, x0, c2.x * x1);
          if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
        {
          const float2 c2 = *reinterpret_cast<const float2*>(&sh.cs()[2 * (NH - 1)]);
          const float mine = h ? slot[0] : slot[NH - 1];
          const float other = pair_other(mine, h);
          if (h == 0) slot[NH - 1] = fmaf(c2.x, mine, c2.y * other);
          else slot[0] = fmaf(-c2.y, other, c2.x * mine);
        }
        static_for<0, NH - 1>([&](auto JC) {
          constexpr int j = decltype(JC)::value;
          float2 c2 = *reinterpret_cast<const float2*>(csb + 2 * j);
          if (!h) c2 = make_float2(1.f, 0.f);
          const float x0 = slot[j], x1 = slot[j + 1];
          slot[j] = fmaf(c2.x, x0, c2.y * x1);
          slot[j + 1] = fmaf(-c2.y, x0, c2.x * x1);
          if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
        });
      }
      if (add) {
        q++;
        p = -1;
      } else {
        q--;
      }
    }
    // converged: a refinement step (from N = 11), then the constraints are checked again (to
    // the refined tolerance above). A step that violates one continues the dual active set from
    // the refined point, whose new steps are fp32 again: the new face is refined in turn (at most
    // four refinements; none when the working set did not move since the last one)
    if (passes >= CMPC_REFINE_MAX || (passes > 0 && iters == it_refined) || !(REFINE && P.refine) ||
        status != CMPC_OK)
      break;
    rinv_ok = false;  // the R^-1 area is the refinement's scratch from here on
    it_refined = iters;
    passes++;
    wide_refine<NV>(rec, P, sh, slot, xv, q, n, wave);
   }
  }

  // ---- scatter (q_soln layout 12 k + 3 leg + axis, swing -> 0) staged in LDS, coalesced out
  const bool ok = (status == CMPC_OK);
  {
    CMPC_WIDE_IDS();
    wbar();
    for (int i = t; i < 12 * N; i += G::NT) sh.P[i] = 0.f;
    wbar();
    // A stance foot-step whose own working-set rows pin all three forces (a vertex of its
    // pyramid: fz = 0 or fz = ub, or two opposite faces, with fx and fy each on a face) takes them
    // from those rows exactly. The fp32 steps of the active set leave x there at ~1e-6 of the
    // unconstrained minimiser: on an all-zero vertex reached from hundreds of N that was 4e-4 N
    // (the tail class's hand-offs, tests/test_gpu_parity.py), beyond 1e-4 x max(|f|, 1 N). Each
    // variable's thread decides for its own component.
    if (ok && h == 0 && r < n) {
      const int fs = r / 3, ax = r - 3 * fs;
      // the foot-step's six flags as one 4-byte and one 2-byte load (six byte loads here had the
      // refining wide 96 build spill 12 B more)
      unsigned int f4;
      unsigned short f2;
      __builtin_memcpy(&f4, &sh.cflag[6 * fs], 4);
      __builtin_memcpy(&f2, &sh.cflag[6 * fs + 4], 2);
      const bool c0 = f4 & 0xffu, c1 = f4 & 0xff00u, c2 = f4 & 0xff0000u, c3 = f4 & 0xff000000u;
      const bool c4 = f2 & 0xffu, c5 = f2 & 0xff00u;
      const bool z0 = c4 || (c0 && c1) || (c2 && c3);
      float out = xv;
      if ((z0 || c5) && (c0 || c1) && (c2 || c3)) {
        const float fz = z0 ? 0.f : sh.sub[fs];
        const float fxy = wdiv(vopq(fz), sopq(P.mu_inv));  // +-mui f + fz = 0 on an active face
        const bool neg = (ax == 0) ? c0 : c2;
        out = (ax == 2) ? fz : (z0 ? 0.f : (neg ? -fxy : fxy));
      }
      sh.P[12 * sh.varblk[r] + sh.varcol[r]] = out;
    }
    wbar();
    for (int i = 4 * t; i < P.out_cols; i += 4 * G::NT)  // (the leading steps kept, 12 N by default)
      *reinterpret_cast<float4*>(&fout[i]) = *reinterpret_cast<const float4*>(&sh.P[i]);
    if (t == 0) {
      st_out[0] = (uint8_t)status;
      if (it_out) it_out[0] = iters;
    }
  }
}

}  // namespace

// Two launch forms per class (CMPC_WIDE_BUILD per width unit: 1 one-per-entry, 2 persistent,
// 3 both):
//   * one workgroup per possible list entry (the list length is only known on the device);
//     surplus workgroups exit after one load. No loop around the solve, so nothing is carried
//     across instances. But an empty or sparse class drains up to `batch` empty workgroups: 3.5 ms
//     for the one-per-CU 146-KB workgroups of the 256 class at config 5, 1.2 ms for the 192 class;
//   * persistent: as many workgroups as fit the GPU at the kernel's occupancy
//     (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs), each dequeuing list entries with one
//     global atomic until the list is exhausted. The loop costs the populous classes registers
//     (80 / 96 / 128: 11 / 20 / 4 spilled VGPRs).
// launch_solve asks for the one-per-entry form (deq == nullptr) only for the class that holds the
// trot size n = 6N (the mode of any contact mix: every instance at config 3 / N = 16 / N = 20
// trot), the persistent form for every other class. The 144 / 192 / 256 classes are built
// persistent only (no spills at their occupancy); their single-instance path runs the loop once
// (deq == nullptr: workgroup i takes entry i).
#ifndef CMPC_WIDE_BUILD
#define CMPC_WIDE_BUILD 1
#endif
#if CMPC_WIDE_VGPR_CAP > 0
#define CMPC_WIDE_VGPR_ATTR __attribute__((amdgpu_num_vgpr(CMPC_WIDE_VGPR_CAP)))
#else
#define CMPC_WIDE_VGPR_ATTR
#endif
struct WideArgs {
  const float* recs;
  float* forces;
  uint8_t* status;
  int32_t* iters;
  const int* in_list;
  const int* in_count;
  int* deq;
  KParams P;
  int base;  // persistent form: first list entry it takes (0, or the grid of a one-per-entry launch)
};

// REFINE is part of the kernel's name: the refining and plain builds of a class live in different
// units, and one instantiation name would let the linker keep only one of them
template <int NV, bool PERSIST, bool REFINE>
__global__ __launch_bounds__(WGeo<NV>::NT, CMPC_WIDE_WAVES_PER_EU) CMPC_WIDE_VGPR_ATTR void cmpc_solve_w_kernel(
    WideArgs A) {
  __shared__ SharedW<NV> sh;
#if CMPC_WIDE_PRIO > 0
  // issue priority of this workgroup's waves over the class-1 waves sharing their SIMDs
  __builtin_amdgcn_s_setprio(CMPC_WIDE_PRIO);
#endif
  const int count = *A.in_count;
  if constexpr (!PERSIST) {  // one workgroup per possible list entry
    const int b = blockIdx.x;
    if (b >= count) return;
    const int inst = A.in_list[b];
    solve_w<NV, REFINE>(A.recs + (size_t)inst * A.P.rec_words, A.P, sh, A.forces + (size_t)inst * A.P.out_cols,
                        A.status + inst, A.iters ? A.iters + inst : nullptr);
  } else {
    for (int round = 0;; round++) {
      // deq == nullptr (single-instance path): workgroup i takes entry i, once
      // base: entries below it belong to a one-per-entry launch of a predicted grid (this launch
      // takes the rest, cmpc_launch.hip hint); 0 otherwise
      if (threadIdx.x == 0) sh.deq_b = A.base + (A.deq ? atomicAdd(A.deq, 1) : (round == 0 ? (int)blockIdx.x : count));
      wbar();
      const int b = __builtin_amdgcn_readfirstlane(sh.deq_b);
      if (b >= count) break;
      const int inst = A.in_list[b];
      solve_w<NV, REFINE>(A.recs + (size_t)inst * A.P.rec_words, A.P, sh, A.forces + (size_t)inst * A.P.out_cols,
                          A.status + inst, A.iters ? A.iters + inst : nullptr);
      wbar();  // every wave is done with this instance's LDS before the next record lands there
    }
  }
}

template <int NV, bool PERSIST, bool REFINE>
int wide_grid_cap() {
  static const int cap = [] {
    int nb = 0, dev = 0, cus = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, cmpc_solve_w_kernel<NV, PERSIST, REFINE>, WGeo<NV>::NT,
                                                     0) != hipSuccess ||
        nb <= 0)
      nb = 1;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    return nb * cus;
  }();
  return cap;
}

// deq != nullptr: persistent form (if built) with that dequeue counter; nullptr: one workgroup per
// entry (if built; the persistent-only classes then run the loop once per workgroup). Internal
// linkage: the width units compile it with different CMPC_WIDE_BUILD, and one shared
// instantiation would serve both launch forms with whichever the linker kept.
namespace {
template <int NV>
hipError_t launch_wide_impl(const float* d_recs, const KParams& P, float* d_forces,
                            uint8_t* d_status, int32_t* d_iters, const int* in_list,
                            const int* in_count, int* deq, int grid, hipStream_t stream, int base = 0) {
  if (grid <= 0) return hipSuccess;
  constexpr bool kOne = (CMPC_WIDE_BUILD & 1) != 0, kPersist = (CMPC_WIDE_BUILD & 2) != 0;
  const bool persist = kPersist && (deq != nullptr || !kOne);
  WideArgs A{d_recs, d_forces, d_status, d_iters, in_list, in_count, persist ? deq : nullptr, P, base};
  if (persist) {
    if constexpr (kPersist) {
      constexpr bool kRef = CMPC_WIDE_REFINE != 0;
      if (deq) grid = grid < wide_grid_cap<NV, true, kRef>() ? grid : wide_grid_cap<NV, true, kRef>();
      hipLaunchKernelGGL((cmpc_solve_w_kernel<NV, true, CMPC_WIDE_REFINE != 0>), dim3(grid), dim3(WGeo<NV>::NT), 0,
                         stream, A);
    }
  } else {
    if constexpr (kOne)
      hipLaunchKernelGGL((cmpc_solve_w_kernel<NV, false, CMPC_WIDE_REFINE != 0>), dim3(grid), dim3(WGeo<NV>::NT), 0,
                         stream, A);
  }
  return hipGetLastError();
}
}  // namespace

}  // namespace cmpc
