// cmpc_class2.h — size class 2 (template over the row width NV): fused condensation + friction-cone QP for instances
// with 64 < n <= NV reduced force variables (NV = 80, 96, 128: random contact tables at N = 10,
// trot at N = 11..16, trot at N = 17..21), one 128-lane workgroup (two wavefronts) per
// instance, over the previous class's overflow list. The row width NV is a
// template parameter: rows of 80 / 96 fit the 256-VGPR budget of a 2-wave/SIMD kernel without
// spilling, a 128-wide one does not, so class-2 work at N = 10 (n <= 78 in 99 % of the
// random-contact instances) runs in the narrowest kernel. One translation unit per width
// (cmpc_class2_w*.hip) so the unrolled kernels compile in parallel.
//
// Same computation as cmpc_class1.hip — one call of the reference's solve_mpc()
// (be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-982) — with the same mapping:
// lane v owns reduced variable v (row v of H, of the Cholesky working matrix, then of J = L^-T,
// in 129 VGPRs), the packed upper-row LDS matrix P holds H and then the raw Cholesky columns.
// What changes with two wavefronts:
//   * each Cholesky step publishes its pivot column (slot[k] of every lane) and crosses ONE
//     s_barrier; J = L^-T and x = -J y only read LDS, so they run barrier-free;
//   * the QP's triangular factor R is kept EXPLICITLY, as packed upper columns in the region
//     that held L (dead once J is formed). The back substitution r = R^-1 d1 and the
//     re-triangularisation after a drop then run inside wavefront 0 with readlanes only, where
//     the implicit R of class 1 would need a cross-wave reduction per active constraint;
//   * cross-wave scalars (|x| max, |d|^2, the dual step) go through a few LDS words.
// Everything is fp32 (the reference condenses in fp32: common_types.h:14).
#pragma once
#include "cmpc_common.h"

#ifndef CMPC_W2_WAVES_PER_EU
#define CMPC_W2_WAVES_PER_EU 2
#endif
// Rows of 128 do not fit 256 VGPRs. At one wave per SIMD (-DCMPC_W128_WAVES_PER_EU=1) the kernel
// may use the whole unified register file (299 VGPRs + 43 AGPRs, no scratch), but that was
// measured slower than two waves per SIMD with scratch spills: 2.05 vs 2.67 M QP/s at N = 20 trot.
#ifndef CMPC_W128_WAVES_PER_EU
#define CMPC_W128_WAVES_PER_EU 2
#endif

namespace cmpc {
namespace {

constexpr int NT = 128;  // threads per workgroup: two wavefronts, lane v < NV owns row v
constexpr int kNone = 0x7fffffff;

// packed upper-row storage of an NV x NV matrix: row r holds columns [r & ~3, NV), 16-B aligned
template <int NV>
struct Geo {
  static constexpr int NG = NV / 4;
  static constexpr int PSZ = 4 * NG * NV - 8 * NG * (NG - 1);
  __host__ __device__ static constexpr int prow(int r) {
    return 4 * (r >> 2) * NV - 8 * (r >> 2) * ((r >> 2) - 1) + (r & 3) * (NV - 4 * (r >> 2));
  }
  __host__ __device__ static constexpr int prow0(int r) { return prow(r) - (r & ~3); }
  static_assert(NV % 4 == 0 && NV <= NT, "row width");
  static_assert(NV * (NV + 1) / 2 <= PSZ, "R must fit in P");
};
// R (upper triangular, q x q) packed by columns: R[i][j] at rcol(j) + i, i <= j
__device__ __forceinline__ int rcol(int j) { return (j * (j + 1)) >> 1; }

constexpr int OFF_E = 0;
constexpr int OFF_ZE = OFF_E + 16 * MAXN;
constexpr int OFF_REC = OFF_ZE + 16 * MAXN;  // LDS copy of the instance record (16-B aligned)
static_assert(OFF_REC + CMPC_REC_WORDS(MAXN) <= Geo<80>::PSZ, "prep scratch must fit in P");

// per-thread arrays are NT long (lanes v >= NV write them too); 19 / 25 / 40 KB (NV = 80 / 96 / 128)
template <int NV>
struct SharedC2 {
  float P[Geo<NV>::PSZ];
  float BdtT[12][16];
  float ibuf[NT];          // 1 / sqrt(d_k) of pivot k
  float vbuf[NT];          // y, then the masked d (v >= q, v < n)
  float dfull[NT];         // d = J' n+
  float bufA[NT], bufB[NT];  // gradient border of pivot k (Cholesky); J rows ia, iz (QP)
  float xs[NT];
  float cs[2 * NT];        // Givens (c, s) per column pair
  float redf[8];
  int redi[8];
  float sub[4 * MAXN];     // ub of each stance foot-step (gait * f_max)
  int sfs[4 * MAXN];       // stance foot-step ids, in order
  int blkbase[MAXN + 2];   // first reduced variable of each horizon step
  unsigned char varblk[NT], varcol[NT];
  unsigned char stance[4 * MAXN];
  unsigned char cflag[2 * NV + 8];  // active flag per constraint id (6 per stance foot-step)
};

__device__ __forceinline__ void bar() { __syncthreads(); }
// compiler-only ordering point for LDS traffic inside one wavefront
__device__ __forceinline__ void lsync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float fdiv(float a, float b) { return a * fast_rcp(b); }

template <int M>
__device__ __forceinline__ void pin(float (&x)[M]) {
#pragma unroll
  for (int c = 0; c < M; c++) asm volatile("" : "+v"(x[c]));
}

#define CMPC_SWEEP_FENCE(c)                                  \
  do {                                                       \
    if (((c) & 15) == 12) __builtin_amdgcn_sched_barrier(0); \
  } while (0)

template <int NV>
__device__ __forceinline__ void solve_c2(const float* __restrict__ rec, const KParams& P,
                                         SharedC2<NV>& sh, float* __restrict__ fout,
                                         uint8_t* __restrict__ st_out, int32_t* __restrict__ it_out,
                                         int* __restrict__ ovf_list, int* __restrict__ ovf_count,
                                         int inst) {
  using G = Geo<NV>;
  const int v = threadIdx.x;
  const int lane = v & 63;
  const int wave = __builtin_amdgcn_readfirstlane(v >> 6);  // wave-uniform: scalar branches
  const int N = P.N;
  // ---- stage the record in LDS: one 16-B load per lane, so the whole prep waits on a single
  // HBM round trip (record words are a multiple of 4, records 16-B aligned)
  {
    const float4* src = reinterpret_cast<const float4*>(rec);
    float4* dst = reinterpret_cast<float4*>(&sh.P[OFF_REC]);
    for (int t = v; t < (P.rec_words >> 2); t += NT) dst[t] = src[t];
  }
  bar();
  const float* srec = &sh.P[OFF_REC];
  // ---- stance table + elimination (SolverMPC.cpp:869-894): both wavefronts compact it (same
  // result), wavefront 0 stores it
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(srec + CMPC_REC_HDR + 12 * N);
  int nfs = 0;
  unsigned long long msk0 = 0ull, msk1 = 0ull;  // stance ballots of foot-steps 0..63, 64..127
  for (int c0 = 0; c0 < 4 * N; c0 += 64) {
    const int t = c0 + lane;
    float ub = 0.f;
    bool f = false;
    if (t < 4 * N) {
      ub = (float)gait[t] * P.f_max;
      f = !(ub < 0.01f && ub > -0.01f);
      if (wave == 0) sh.stance[t] = f ? 1 : 0;
    }
    const unsigned long long m = __ballot(f);
    if (c0 == 0) msk0 = m; else msk1 = m;
    const int pre = __popcll(m & ((1ull << lane) - 1ull));
    if (f && wave == 0) {
      sh.sfs[nfs + pre] = t;
      sh.sub[nfs + pre] = ub;
    }
    nfs += __popcll(m);
  }
  const int n = 3 * nfs;
  if (n > NV) {  // hand the instance to the next (wider) class
    if (v == 0 && ovf_list) ovf_list[atomicAdd(ovf_count, 1)] = inst;
    return;
  }
  bar();
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
    for (int t = v; t < 6 * nfs; t += NT) sh.cflag[t] = 0;
  }
  Model md;
  make_model(srec, P.dt, md);
  make_bdt<NT>(srec, md, v, sh.BdtT);
  bar();
  if (v < N) {
    float e[13];
    state_error(srec, md, v, srec + CMPC_REC_HDR + 12 * v, e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.P[OFF_E + 16 * v + j] = e[j];
  }
  bar();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  // gradient recursion ze_i = S e_i + Adt' ze_{i+1} (uniform; lane j < 13 stores component j)
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
  bar();

  // ---- condensation: lane v builds H[v][w] for w >= v into packed P, and its gradient g_v
  const bool real = v < n;
  float gv;
  {
    const int kv = real ? sh.varblk[v] : 0;
    const int cv = real ? sh.varcol[v] : 0;
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = real ? sh.BdtT[cv][j] : 0.f;
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.P[OFF_ZE + 16 * kv + j];
      gv = real ? 2.f * dot13(b, zk) : 0.f;  // qg = 2 B_qp' S (A_qp x0 + Q_qp f - X_d)
    }
    bar();  // every ZE read is done before P is overwritten
    const int myrow = G::prow0(v);
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
      const int wb = __builtin_amdgcn_readfirstlane(sh.blkbase[i]);
      const int we = __builtin_amdgcn_readfirstlane(sh.blkbase[i + 1]);
      for (int w = wb; w < we; w++) {
        const int cw = sh.varcol[w];
        float bw[13];
#pragma unroll
        for (int j = 0; j < 13; j++) bw[j] = sh.BdtT[cw][j];
        float val = 2.f * dot13(bw, z);
        if (w == v) val += P.alpha2;  // qH = 2 (B'SB + alpha I), SolverMPC.cpp:806
        if (act && w >= v) sh.P[myrow + w] = val;
      }
    }
  }
  bar();

  // ---- row v of H into registers (full symmetric; identity padding for v >= n) ----------
  float slot[NV + 1];
  {
    const int myrow = G::prow0(v);
    static_for<0, NV>([&](auto C) {
      constexpr int c = decltype(C)::value;
      const int addr = (c >= v) ? myrow + c : G::prow0(c) + v;
      const float x = sh.P[addr];
      slot[c] = (real && c < n) ? x : ((c == v) ? 1.f : 0.f);
      if ((c & 7) == 7) __builtin_amdgcn_sched_barrier(0);
    });
    slot[NV] = gv;
  }
  bar();

  // ---- bordered Cholesky [H | g]: raw column k = slot[k] of every lane -> P row k ----------
  int status = CMPC_OK;
  float my_inv = 1.f;
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int c0 = k & ~3;
    constexpr int rk = G::prow(k);
    if (k < n) {
      if (v >= c0 && v < NV) sh.P[rk + v - c0] = (v >= k) ? slot[k] : 0.f;
      if (v == k) sh.bufA[k] = slot[NV];
      bar();
      float d = sh.P[rk + k - c0];
      if (!(d > 0.f)) { status = CMPC_NOT_PD; d = 1e-30f; }
      const float inv = rsqrtf(d);
      if (v == k) { my_inv = inv; sh.ibuf[k] = inv; }
      const float a = (v > k) ? -slot[k] * (inv * inv) : 0.f;
#pragma unroll
      for (int c = c0; c < NV; c += 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        slot[c + 0] = fmaf(a, r4.x, slot[c + 0]);
        slot[c + 1] = fmaf(a, r4.y, slot[c + 1]);
        slot[c + 2] = fmaf(a, r4.z, slot[c + 2]);
        slot[c + 3] = fmaf(a, r4.w, slot[c + 3]);
        CMPC_SWEEP_FENCE(c);
      }
      slot[NV] = fmaf(a, sh.bufA[k], slot[NV]);
      pin(slot);
    }
  });
  const float yv = (v < n) ? slot[NV] * my_inv : 0.f;  // L y = g
  bar();

  // ---- J = L^-T: lane v solves L x = e_v (column v of L^-1 = row v of J); LDS reads only ----
  static_for<0, NV>([&](auto C) {
    constexpr int c = decltype(C)::value;
    slot[c] = (c == v) ? 1.f : 0.f;
  });
  static_for<0, NV>([&](auto KC) {
    constexpr int k = decltype(KC)::value;
    constexpr int c0 = k & ~3;
    constexpr int rk = G::prow(k);
    if (k < n) {
      lsync();
      const float inv = sh.ibuf[k];
      const float xk = slot[k] * inv;
      const float a = -xk * inv;
#pragma unroll
      for (int c = c0; c < NV; c += 4) {
        const float4 r4 = *reinterpret_cast<const float4*>(&sh.P[rk + c - c0]);
        slot[c + 0] = fmaf(a, r4.x, slot[c + 0]);
        slot[c + 1] = fmaf(a, r4.y, slot[c + 1]);
        slot[c + 2] = fmaf(a, r4.z, slot[c + 2]);
        slot[c + 3] = fmaf(a, r4.w, slot[c + 3]);
        CMPC_SWEEP_FENCE(c);
      }
      slot[k] = xk;
      pin(slot);
    }
  });

  // ---- unconstrained minimiser x = -J y ----------------------------------------------------
  sh.vbuf[v] = yv;
  bar();
  float xv = 0.f;
#pragma unroll
  for (int c = 0; c < NV; c += 4) {
    const float4 y4 = *reinterpret_cast<const float4*>(&sh.vbuf[c]);
    xv = fmaf(slot[c + 0], y4.x, xv);
    xv = fmaf(slot[c + 1], y4.y, xv);
    xv = fmaf(slot[c + 2], y4.z, xv);
    xv = fmaf(slot[c + 3], y4.w, xv);
    CMPC_SWEEP_FENCE(c);
  }
  xv = (v < n) ? -xv : 0.f;
  bar();  // L (in P) and y are dead from here; P holds R

  // ---- Goldfarb-Idnani dual active set on the friction pyramids -----------------------------
  // One flat loop, one active-set step per trip (class 1's structure): the J rows see the same
  // straight-line code on every trip (Householder reflection for an add, beta = 0 on a drop;
  // ascending Givens chain for a drop, identity rotations on an add), so their registers carry
  // through the loop without copies. R lives in P, maintained by wavefront 0.
  const float mui = P.mu_inv;
  const float fnorm = rsqrtf(mui * mui + 1.f);
  int q = 0;
  int iters = 0;
  // wavefront 0, lane l: active-set positions l and l + 64 (dual u, constraint id, dual step r)
  float u_lo = 0.f, u_hi = 0.f, r_lo = 0.f, r_hi = 0.f;
  int a_lo = 0, a_hi = 0;
  int p = -1;          // constraint being added (-1: pick the most violated one)
  Cons cp{};
  float up = 0.f;
  if (status == CMPC_OK) {
    for (;;) {
      pin(slot);
      // lane ids re-materialised per trip (tid_opq): keeps per-lane LDS addresses out of the
      // loop preheader, where they would be spilled
      const int v = tid_opq();
      const int lane = v & 63;
      if (p < 0) {
        sh.xs[v] = xv;
        {
          const float wm = wave_max(fabsf(xv));
          if (lane == 0) sh.redf[wave] = wm;
        }
        bar();
        // most violated constraint (normalised slack): both wavefronts scan the same foot-steps
        float best = 0.f;
        int bid = kNone;
        if (lane < nfs) {
          const float fx = sh.xs[3 * lane], fy = sh.xs[3 * lane + 1], fz = sh.xs[3 * lane + 2];
          float sl[6];
          sl[0] = (mui * fx + fz) * fnorm;
          sl[1] = (-mui * fx + fz) * fnorm;
          sl[2] = (mui * fy + fz) * fnorm;
          sl[3] = (-mui * fy + fz) * fnorm;
          sl[4] = fz;
          sl[5] = sh.sub[lane] - fz;
#pragma unroll
          for (int t = 0; t < 6; t++)
            if (!sh.cflag[6 * lane + t] && sl[t] < best) { best = sl[t]; bid = 6 * lane + t; }
        }
        const float xmax = fmaxf(sh.redf[0], sh.redf[1]);
        wave_argmin(best, bid);
        const float tol = 1e-5f * fmaxf(1.f, xmax);
        if (bid == kNone || best >= -tol) break;
        p = __builtin_amdgcn_readfirstlane(bid);
        cp = decode_cons(p, mui, sh.sub[p / 6]);
        up = 0.f;
      }
      if (++iters > P.max_iter + 2 * n) { status = CMPC_MAX_ITER; break; }
      // d = J' n+ : rows ia, iz of J through LDS (dword stores: 128-bit stores would tie the
      // row registers into quads)
      if (v == cp.ia && cp.ia != cp.iz) {
#pragma unroll
        for (int c = 0; c < NV; c++) sh.bufA[c] = slot[c];
      }
      if (v == cp.iz) {
#pragma unroll
        for (int c = 0; c < NV; c++) sh.bufB[c] = slot[c];
      }
      sh.xs[v] = xv;
      bar();
      const float dv = (cp.ia != cp.iz) ? fmaf(cp.ca, sh.bufA[v], cp.cb * sh.bufB[v]) : cp.cb * sh.bufB[v];
      const float dm = (v >= q && v < n) ? dv : 0.f;
      sh.vbuf[v] = dm;
      sh.dfull[v] = dv;
      {
        const float dw = wave_sum((v < n) ? dv * dv : 0.f);
        if (lane == 0) sh.redf[2 + wave] = dw;
      }
      const float spv = fmaf(cp.ca, sh.xs[cp.ia], fmaf(cp.cb, sh.xs[cp.iz], -cp.bp));
      bar();
      // z = J2 d2 (primal step direction), zn = |d2|^2 = z' n+, dn = |d|^2
      float zv = 0.f, zn = 0.f;
#pragma unroll
      for (int c = 0; c < NV; c += 4) {
        const float4 m4 = *reinterpret_cast<const float4*>(&sh.vbuf[c]);
        zv = fmaf(slot[c + 0], m4.x, zv);
        zv = fmaf(slot[c + 1], m4.y, zv);
        zv = fmaf(slot[c + 2], m4.z, zv);
        zv = fmaf(slot[c + 3], m4.w, zv);
        zn += m4.x * m4.x + m4.y * m4.y + m4.z * m4.z + m4.w * m4.w;
        CMPC_SWEEP_FENCE(c);
      }
      const float dn = sh.redf[2] + sh.redf[3];
      // r = R^-1 d1 by back substitution over the packed columns of R (wavefront 0), then the
      // partial (dual) step t1 = min_{r_j > 0} u_j / r_j
      if (wave == 0) {
        float acc_lo = dv;
        float acc_hi = sh.dfull[lane + 64];
        r_lo = 0.f;
        r_hi = 0.f;
        for (int i = q - 1; i >= 0; i--) {
          const int off = rcol(i);
          const float rii = sh.P[off + i];
          const float ai = (i < 64) ? rl(acc_lo, i) : rl(acc_hi, i - 64);
          const float ri = fdiv(ai, rii);
          if (lane < i) acc_lo = fmaf(-sh.P[off + lane], ri, acc_lo);
          if (lane + 64 < i) acc_hi = fmaf(-sh.P[off + lane + 64], ri, acc_hi);
          r_lo = (lane == i) ? ri : r_lo;
          r_hi = (lane + 64 == i) ? ri : r_hi;
        }
        float t1w = kBigF;
        int kw = kNone;
        if (lane < q && r_lo > 0.f) { t1w = fmaxf(fdiv(u_lo, r_lo), 0.f); kw = lane; }
        if (lane + 64 < q && r_hi > 0.f) {
          const float th = fmaxf(fdiv(u_hi, r_hi), 0.f);
          if (th < t1w) { t1w = th; kw = lane + 64; }
        }
        wave_argmin(t1w, kw);
        if (lane == 0) { sh.redf[4] = t1w; sh.redi[4] = kw; }
      }
      bar();
      const float t1 = sh.redf[4];
      const int kk = __builtin_amdgcn_readfirstlane(sh.redi[4]);
      const bool zero_step = !(zn > 1e-9f * dn);
      const float t2 = zero_step ? kBigF : -fdiv(spv, zn);
      const float t = fminf(t1, t2);
      if (t >= kBigF) { status = CMPC_INFEASIBLE; break; }
      if (wave == 0) {
        if (lane < q) u_lo = fmaf(-t, r_lo, u_lo);
        if (lane + 64 < q) u_hi = fmaf(-t, r_hi, u_hi);
      }
      up += t;
      if (!zero_step) xv = fmaf(t, zv, xv);
      const bool add = !zero_step && t2 <= t1;
      float beta = 0.f;
      if (add) {
        // ---- add p: the Householder reflection I - beta w w' on columns q..n-1 maps
        // d[q..n-1] to -sgn(d_q) |d[q..n-1]| e_q; R gains the column (d[0..q-1], -sgn ts)
        const float ts = sqrtf(zn);
        const float dq = sh.dfull[q];
        const float sgn = (dq >= 0.f) ? 1.f : -1.f;
        beta = fast_rcp(ts * (ts + fabsf(dq)));  // 2 / (w'w)
        sh.vbuf[v] = (v == q) ? dq + sgn * ts : dm;
        *reinterpret_cast<float2*>(&sh.cs[2 * v]) = make_float2(1.f, 0.f);
        const int offq = rcol(q);
        if (v < q) sh.P[offq + v] = dv;
        if (v == q) sh.P[offq + q] = -sgn * ts;
        if (wave == 0) {
          if (lane == q) { u_lo = up; a_lo = p; }
          if (lane + 64 == q) { u_hi = up; a_hi = p; }
        }
        if (v == 0) sh.cflag[p] = 1;
      } else {
        // ---- drop active constraint kk: shift positions kk+1..q-1 down, remove column kk of
        // R and re-triangularise rows kk..q-1 with Givens rotations (wavefront 0, in place)
        sh.vbuf[v] = 0.f;
        const int k = kk;
        // identity rotations outside k <= j <= q-2 (wavefront 0 writes the others below)
        if (v < k || v > q - 2) *reinterpret_cast<float2*>(&sh.cs[2 * v]) = make_float2(1.f, 0.f);
        if (wave == 0) {
          const int ak = (k < 64) ? rli(a_lo, k) : rli(a_hi, k - 64);
          if (lane == 0) sh.cflag[ak] = 0;
          const int alo_nx = lane_next_i(a_lo, a_lo);
          const float ulo_nx = lane_next(u_lo, u_lo);
          const int ahi_nx = lane_next_i(a_hi, a_hi);
          const float uhi_nx = lane_next(u_hi, u_hi);
          const int ahi0 = rli(a_hi, 0);
          const float uhi0 = rl(u_hi, 0);
          if (lane >= k && lane < q - 1) {
            a_lo = (lane == 63) ? ahi0 : alo_nx;
            u_lo = (lane == 63) ? uhi0 : ulo_nx;
          }
          if (lane + 64 >= k && lane + 64 < q - 1) { a_hi = ahi_nx; u_hi = uhi_nx; }
          // new column c (k <= c <= q-2) = old column c+1. Lane l handles c = l and l + 64.
          // Every read of an old entry precedes, in this wavefront's LDS order, the write that
          // reuses its word (new column c overlays old column c).
          const int clo = lane, chi = lane + 64;
          const bool in_lo = clo >= k && clo <= q - 2;
          const bool in_hi = chi >= k && chi <= q - 2;
          float top_lo = in_lo ? sh.P[rcol(clo + 1) + k] : 0.f;
          float top_hi = in_hi ? sh.P[rcol(chi + 1) + k] : 0.f;
          lsync();
          for (int r = 0; r < k; r++) {
            const float xlo = in_lo ? sh.P[rcol(clo + 1) + r] : 0.f;
            const float xhi = in_hi ? sh.P[rcol(chi + 1) + r] : 0.f;
            lsync();
            if (in_lo) sh.P[rcol(clo) + r] = xlo;
            if (in_hi) sh.P[rcol(chi) + r] = xhi;
            lsync();
          }
          for (int j = k; j <= q - 2; j++) {
            const bool on_lo = in_lo && clo >= j, on_hi = in_hi && chi >= j;
            const float bot_lo = on_lo ? sh.P[rcol(clo + 1) + j + 1] : 0.f;
            const float bot_hi = on_hi ? sh.P[rcol(chi + 1) + j + 1] : 0.f;
            lsync();
            const float a0 = (j < 64) ? rl(top_lo, j) : rl(top_hi, j - 64);
            const float b0 = (j < 64) ? rl(bot_lo, j) : rl(bot_hi, j - 64);
            const float h = sqrtf(a0 * a0 + b0 * b0);
            float cc = 1.f, sn = 0.f;
            if (h > 0.f) { const float ih = fast_rcp(h); cc = a0 * ih; sn = b0 * ih; }
            if (on_lo) {
              sh.P[rcol(clo) + j] = fmaf(cc, top_lo, sn * bot_lo);
              top_lo = fmaf(-sn, top_lo, cc * bot_lo);
            }
            if (on_hi) {
              sh.P[rcol(chi) + j] = fmaf(cc, top_hi, sn * bot_hi);
              top_hi = fmaf(-sn, top_hi, cc * bot_hi);
            }
            if (lane == 0) *reinterpret_cast<float2*>(&sh.cs[2 * j]) = make_float2(cc, sn);
            lsync();
          }
        }
      }
      bar();
      // J <- J (I - beta w w'): tw = J_v . w, J_v -= beta tw w  (no-op on a drop: beta = 0)
      {
        float tw = 0.f;
#pragma unroll
        for (int c = 0; c < NV; c += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(&sh.vbuf[c]);
          tw = fmaf(slot[c + 0], w4.x, tw);
          tw = fmaf(slot[c + 1], w4.y, tw);
          tw = fmaf(slot[c + 2], w4.z, tw);
          tw = fmaf(slot[c + 3], w4.w, tw);
          CMPC_SWEEP_FENCE(c);
        }
        const float bt = -beta * tw;
        // re-read w from LDS: without this point the compiler keeps all NV values of the first
        // sweep's loads live for the second (a whole row of extra VGPRs)
        asm volatile("" ::: "memory");
#pragma unroll
        for (int c = 0; c < NV; c += 4) {
          const float4 w4 = *reinterpret_cast<const float4*>(&sh.vbuf[c]);
          slot[c + 0] = fmaf(bt, w4.x, slot[c + 0]);
          slot[c + 1] = fmaf(bt, w4.y, slot[c + 1]);
          slot[c + 2] = fmaf(bt, w4.z, slot[c + 2]);
          slot[c + 3] = fmaf(bt, w4.w, slot[c + 3]);
          CMPC_SWEEP_FENCE(c);
        }
      }
      // J columns (j, j+1) <- Givens chain j = 0 .. NV-2 (identity on an add)
      static_for<0, NV - 1>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        const float2 cs2 = *reinterpret_cast<const float2*>(&sh.cs[2 * j]);
        const float x0 = slot[j], x1 = slot[j + 1];
        slot[j] = fmaf(cs2.x, x0, cs2.y * x1);
        slot[j + 1] = fmaf(-cs2.y, x0, cs2.x * x1);
        if ((j & 7) == 7) __builtin_amdgcn_sched_barrier(0);
      });
      if (add) {
        q++;
        p = -1;
      } else {
        q--;
      }
    }
  }

  // ---- scatter (q_soln layout 12 k + 3 leg + axis, swing -> 0) staged in LDS, coalesced out
  const bool ok = (status == CMPC_OK);
  bar();
  for (int t = v; t < 12 * N; t += NT) sh.P[t] = 0.f;
  bar();
  if (ok && v < n) sh.P[12 * sh.varblk[v] + sh.varcol[v]] = xv;
  bar();
  for (int t = 4 * v; t < 12 * N; t += 4 * NT)
    *reinterpret_cast<float4*>(&fout[t]) = *reinterpret_cast<const float4*>(&sh.P[t]);
  if (v == 0) {
    st_out[0] = (uint8_t)status;
    if (it_out) it_out[0] = iters;
  }
}

}  // namespace

// One workgroup per entry of the class's list; the grid is sized for the worst case (the list
// length is only known on the device) and surplus workgroups exit at once. (A persistent grid
// looping over the list was measured slower: it serialises the long class-2 solves.)
template <int NV>
__global__ __launch_bounds__(NT, (NV >= 128 ? CMPC_W128_WAVES_PER_EU : CMPC_W2_WAVES_PER_EU)) void
cmpc_solve_c2_kernel(
    const float* __restrict__ recs, KParams P, float* __restrict__ forces,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, const int* __restrict__ in_list,
    const int* __restrict__ in_count, int* __restrict__ ovf_list, int* __restrict__ ovf_count) {
  __shared__ SharedC2<NV> sh;
  const int t = blockIdx.x;
  if (t >= *in_count) return;
  const int inst = in_list[t];
  solve_c2<NV>(recs + (size_t)inst * P.rec_words, P, sh, forces + (size_t)inst * 12 * P.N,
               status + inst, iters ? iters + inst : nullptr, ovf_list, ovf_count, inst);
}

template <int NV>
hipError_t launch_class2_impl(const float* d_recs, const KParams& P, float* d_forces,
                              uint8_t* d_status, int32_t* d_iters, const int* in_list,
                              const int* in_count, int* ovf_list, int* ovf_count, int grid,
                              hipStream_t stream) {
  hipLaunchKernelGGL(cmpc_solve_c2_kernel<NV>, dim3(grid), dim3(NT), 0, stream, d_recs, P, d_forces,
                     d_status, d_iters, in_list, in_count, ovf_list, ovf_count);
  return hipGetLastError();
}

}  // namespace cmpc
