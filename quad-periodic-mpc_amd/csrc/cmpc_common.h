#pragma once
// cmpc_common.h — device building blocks shared by every solver kernel:
//   * wavefront reductions / lane helpers (64-wide wavefronts, gfx950);
//   * the per-instance model of solve_mpc(): RobotState::set + quat_to_rpy
//     (RobotState.cpp:9-50, SolverMPC.cpp:352-361), ct_ss_mats (SolverMPC.cpp:260-279) and the
//     closed-form discretisation of c2qp (SolverMPC.cpp:96-107; A_c^3 = 0 so
//     expm(dt [A B Q; 0]) = I + M + M^2/2 + M^3/6 exactly);
//   * the stance table / swing elimination (SolverMPC.cpp:859-894) and the condensation
//     recursions that build the reduced qH / qg (SolverMPC.cpp:806-814) without ever forming
//     A_qp, B_qp or the dense 13N x 13N weight matrix S.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "cmpc_kernels.h"

namespace cmpc {
namespace {

constexpr int MAXN = CMPC_MAX_HORIZON;
constexpr float kBigF = 3.0e38f;

// ---------------------------------------------------------------------------------------------
// wavefront helpers. Reductions use DPP lane permutes inside the VALU (row permutes, then the
// row_bcast15 / row_bcast31 steps across the four 16-lane rows) and hand back a wave-uniform
// result through v_readlane: no ds_bpermute round trips through the LDS crossbar and no
// per-lane shuffle addresses for the optimiser to hoist out of loops.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float rl(float x, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), lane));
}
__device__ __forceinline__ int rli(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }

// DPP16 controls (GFX9 encoding)
constexpr int kDppQuadSwap1 = 0xB1;   // quad_perm [1,0,3,2]
constexpr int kDppQuadSwap2 = 0x4E;   // quad_perm [2,3,0,1]
constexpr int kDppRowShl = 0x100;     // + n: lane i <- lane i + n of the same row
constexpr int kDppRowShr = 0x110;     // + n: lane i <- lane i - n of the same row
constexpr int kDppWaveShl1 = 0x130;   // lane i <- lane i + 1
constexpr int kDppWaveShr1 = 0x138;   // lane i <- lane i - 1
constexpr int kDppRowMirror = 0x140;
constexpr int kDppRowHalfMirror = 0x141;
constexpr int kDppRowBcast15 = 0x142;
constexpr int kDppRowBcast31 = 0x143;

// lanes whose source is outside the row/wave, or whose row is masked off, get `old`
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dppf(float old, float src) {
  return __int_as_float(
      __builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(src), CTRL, ROW_MASK, 0xf, false));
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dppi(int old, int src) {
  return __builtin_amdgcn_update_dpp(old, src, CTRL, ROW_MASK, 0xf, false);
}

// sum over the 64 lanes (uniform result)
__device__ __forceinline__ float wave_sum(float v) {
  v += dppf<kDppQuadSwap1>(0.f, v);
  v += dppf<kDppQuadSwap2>(0.f, v);
  v += dppf<kDppRowHalfMirror>(0.f, v);
  v += dppf<kDppRowMirror>(0.f, v);
  v += dppf<kDppRowBcast15, 0xa>(0.f, v);
  v += dppf<kDppRowBcast31, 0xc>(0.f, v);
  return rl(v, 63);
}
// max over the 64 lanes (uniform result)
__device__ __forceinline__ float wave_max(float v) {
  constexpr float ninf = -__builtin_huge_valf();
  v = fmaxf(v, dppf<kDppQuadSwap1>(ninf, v));
  v = fmaxf(v, dppf<kDppQuadSwap2>(ninf, v));
  v = fmaxf(v, dppf<kDppRowHalfMirror>(ninf, v));
  v = fmaxf(v, dppf<kDppRowMirror>(ninf, v));
  v = fmaxf(v, dppf<kDppRowBcast15, 0xa>(ninf, v));
  v = fmaxf(v, dppf<kDppRowBcast31, 0xc>(ninf, v));
  return rl(v, 63);
}
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ void argmin_step(float& v, int& i) {
  const float ov = dppf<CTRL, ROW_MASK>(__builtin_huge_valf(), v);
  const int oi = dppi<CTRL, ROW_MASK>(0x7fffffff, i);
  if (ov < v || (ov == v && oi < i)) { v = ov; i = oi; }
}
// lexicographic (value, index) minimum over the 64 lanes, i.e. argmin with a deterministic
// tie-break on the smaller index (uniform result)
__device__ __forceinline__ void wave_argmin(float& v, int& i) {
  argmin_step<kDppQuadSwap1>(v, i);
  argmin_step<kDppQuadSwap2>(v, i);
  argmin_step<kDppRowHalfMirror>(v, i);
  argmin_step<kDppRowMirror>(v, i);
  argmin_step<kDppRowBcast15, 0xa>(v, i);
  argmin_step<kDppRowBcast31, 0xc>(v, i);
  v = rl(v, 63);
  i = rli(i, 63);
}
// inclusive suffix sum over lanes: s_l = sum_{m >= l} v_m (a true suffix scan, no
// total-minus-prefix cancellation): row-local scan with row_shl, then the later rows' totals
__device__ __forceinline__ float wave_suffix_sum(float v, int lane) {
  v += dppf<kDppRowShl + 1>(0.f, v);
  v += dppf<kDppRowShl + 2>(0.f, v);
  v += dppf<kDppRowShl + 4>(0.f, v);
  v += dppf<kDppRowShl + 8>(0.f, v);
  const float r1 = rl(v, 16), r2 = rl(v, 32), r3 = rl(v, 48);
  const int row = lane >> 4;
  return v + ((row == 0) ? r1 + (r2 + r3) : (row == 1) ? r2 + r3 : (row == 2) ? r3 : 0.f);
}
// value of lane l - 1 (lane 0 gets `old`) / lane l + 1 (lane 63 gets `old`)
__device__ __forceinline__ float lane_prev(float old, float v) { return dppf<kDppWaveShr1>(old, v); }
__device__ __forceinline__ float lane_next(float old, float v) { return dppf<kDppWaveShl1>(old, v); }
__device__ __forceinline__ int lane_next_i(int old, int v) { return dppi<kDppWaveShl1>(old, v); }

// thread index the optimiser cannot treat as loop-invariant: per-lane addresses derived from it
// are recomputed where they are used instead of being hoisted out of long loops (and spilled)
__device__ __forceinline__ int tid_opq() {
  int x = threadIdx.x;
  asm volatile("" : "+v"(x));
  return x;
}

// lane id (0..63) from mbcnt, opaque to the optimiser: unlike threadIdx.x (v0 at entry, which
// has to stay live, or be spilled, to be re-read later) it needs no register between uses
#ifndef CMPC_LANE_ASM
#define CMPC_LANE_ASM 1
#endif
__device__ __forceinline__ int lane_opq() {
#if CMPC_LANE_ASM
  // the mbcnt pair inside the asm: every call recomputes the lane id (two VALU ops) instead of
  // sharing one CSE'd value that lives across the kernel (and was spilled and reloaded per call)
  int x;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
#else
  int x = (int)__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  asm volatile("" : "+v"(x));
#endif
  return x;
}

template <int I, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < E) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, E>(f);
  }
}
// Software-pipelined sweep over 16-B chunks c = C0, C0 + 4, ..., < CE: ld(c) loads chunk c's
// operands from LDS, f(c, v) consumes them; in groups of GRP chunks, the loads of group g + 1 are
// issued before the arithmetic of group g (scheduling fences keep that order and bound the live
// loads to two groups), so the wave meets the LDS latency once per sweep, not once per group.
template <int C0, int CE, int GRP, class Ld, class F>
__device__ __forceinline__ void piped_sweep(Ld&& ld, F&& f) {
  constexpr int NCH = (CE > C0) ? (CE - C0) / 4 : 0;
  if constexpr (NCH > 0) {
    using T = decltype(ld(std::integral_constant<int, C0>{}));
    constexpr int NG = (NCH + GRP - 1) / GRP;
    T cur[GRP], nxt[GRP];
    static_for<0, GRP>([&](auto I) {
      constexpr int ch = decltype(I)::value;
      if constexpr (ch < NCH) cur[ch] = ld(std::integral_constant<int, C0 + 4 * ch>{});
    });
    static_for<0, NG>([&](auto GI) {
      constexpr int g = decltype(GI)::value;
      static_for<0, GRP>([&](auto I) {
        constexpr int ch = (g + 1) * GRP + decltype(I)::value;
        if constexpr (ch < NCH) nxt[decltype(I)::value] = ld(std::integral_constant<int, C0 + 4 * ch>{});
      });
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, GRP>([&](auto I) {
        constexpr int ch = g * GRP + decltype(I)::value;
        if constexpr (ch < NCH) f(std::integral_constant<int, C0 + 4 * ch>{}, cur[decltype(I)::value]);
      });
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, GRP>([&](auto I) { cur[decltype(I)::value] = nxt[decltype(I)::value]; });
    });
  }
}
struct F4x2 {
  float4 a, b;
};
struct F4x4 {
  float4 a, b, c, d;
};

// An SGPR value the compiler cannot see through: keeps per-iteration scalar work of an unrolled
// loop inside its iteration (otherwise LICM hoists dozens of SGPRs out of it -> spills).
// a constant or kernel argument materialised at its use (volatile asm is never hoisted): keeps
// loop-invariant code motion from holding it in a register across a loop nest
__device__ __forceinline__ float vopq(float x) {
  asm volatile("" : "+v"(x));
  return x;
}
__device__ __forceinline__ float sopq(float x) {
  asm volatile("" : "+s"(x));
  return x;
}
__device__ __forceinline__ float rfl(float x) {  // a wave-uniform float into an SGPR
  return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}
__device__ __forceinline__ int opaque(int x) {
  x = __builtin_amdgcn_readfirstlane(x);
  asm volatile("" : "+s"(x));
  return x;
}
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// Row-sweep helpers: x[0..3] += a * r[0..3] and acc += x[0..3] . r[0..3] (acc is a lane pair,
// summed once at the end). Scalar FMAs: packed FP32 (v_pk_fma_f32) was measured 20 % slower in
// class 1 (2.47 vs 2.03 ms: packing the row registers into pairs costs more moves than the
// halved FMA count saves).
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void axpy4(float a, float4 r, float& x0, float& x1, float& x2, float& x3) {
  x0 = fmaf(a, r.x, x0);
  x1 = fmaf(a, r.y, x1);
  x2 = fmaf(a, r.z, x2);
  x3 = fmaf(a, r.w, x3);
}
__device__ __forceinline__ void dot4(f2v& acc, float x0, float x1, float x2, float x3, float4 r) {
  acc.x = fmaf(x0, r.x, acc.x);
  acc.x = fmaf(x1, r.y, acc.x);
  acc.x = fmaf(x2, r.z, acc.x);
  acc.x = fmaf(x3, r.w, acc.x);
}
// the same with two interleaved chains (acc.x: even columns, acc.y: odd): half the dependent FMA
// latency of a row-long dot product
__device__ __forceinline__ void dot4x2(f2v& acc, float x0, float x1, float x2, float x3, float4 r) {
  acc.x = fmaf(x0, r.x, acc.x);
  acc.y = fmaf(x1, r.y, acc.y);
  acc.x = fmaf(x2, r.z, acc.x);
  acc.y = fmaf(x3, r.w, acc.y);
}

// single-wavefront workgroup: orders this wave's LDS traffic without an s_barrier
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// ---------------------------------------------------------------------------------------------
// Discretised model (closed form). Adt = I + N1 with N1 = dt A_c + dt^2/2 A_c^2 (16 structural
// nonzeros); Adt^m = I + m N1 + m(m-1)/2 N1^2 exactly (N1^3 = 0).
// ---------------------------------------------------------------------------------------------
struct Model {
  float R[9];      // body rotation (Eigen toRotationMatrix of q, w-first); R_yaw = R (RobotState.cpp:44)
  float n1r[9];    // N1[0..2][6..8] = dt * R^T
  float dt, dth, xdrag;  // dt, dt^2/2, x_drag (A_c(11,9), SolverMPC.cpp:277)
};

// y = N1 x   (13-vectors)
__device__ __forceinline__ void n1_mul(const Model& m, const float* x, float* y) {
#pragma unroll
  for (int i = 0; i < 3; i++) y[i] = m.n1r[i * 3 + 0] * x[6] + m.n1r[i * 3 + 1] * x[7] + m.n1r[i * 3 + 2] * x[8];
  y[3] = m.dt * x[9];
  y[4] = m.dt * x[10];
  y[5] = m.dt * x[11] + (m.dth * m.xdrag) * x[9] + m.dth * x[12];
#pragma unroll
  for (int i = 6; i < 11; i++) y[i] = 0.f;
  y[11] = (m.dt * m.xdrag) * x[9] + m.dt * x[12];
  y[12] = 0.f;
}

// z <- w .* e + Adt' z   (in place on z; Adt' = I + N1')
__device__ __forceinline__ void recur(const Model& m, const float* wts, const float* e, float* z) {
  float t[13];
#pragma unroll
  for (int j = 0; j < 13; j++) t[j] = z[j];
  const float c6 = m.n1r[0] * t[0] + m.n1r[3] * t[1] + m.n1r[6] * t[2];
  const float c7 = m.n1r[1] * t[0] + m.n1r[4] * t[1] + m.n1r[7] * t[2];
  const float c8 = m.n1r[2] * t[0] + m.n1r[5] * t[1] + m.n1r[8] * t[2];
  const float c9 = m.dt * t[3] + (m.dt * m.xdrag) * t[11] + (m.dth * m.xdrag) * t[5];
  const float c10 = m.dt * t[4];
  const float c11 = m.dt * t[5];
  const float c12 = m.dt * t[11] + m.dth * t[5];
#pragma unroll
  for (int j = 0; j < 13; j++) z[j] = wts[j] * e[j] + t[j];
  z[6] += c6; z[7] += c7; z[8] += c8; z[9] += c9; z[10] += c10; z[11] += c11; z[12] += c12;
}

__device__ __forceinline__ float dot13(const float* a, const float* b) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 13; j++) s = fmaf(a[j], b[j], s);
  return s;
}

// stance mask of horizon step i (bit f: foot f in stance) from the two stance ballots over the
// foot-steps 4 i + f (m0: foot-steps 0..63, m1: 64..127); uniform
__device__ __forceinline__ unsigned step_mask(unsigned long long m0, unsigned long long m1, int i) {
  return (unsigned)(((i < 16) ? (m0 >> (4 * i)) : (m1 >> (4 * i - 64))) & 15ull);
}

// The H entries of horizon step i for one row: for every stance foot f of the step (uniform
// mask mi, ascending) and axis a, column c = 3 f + a of Bdt lands at reduced column
// w = wb + 3 rank(f) + a with value 2 b_c' z. Unrolled over the 4 feet x 3 axes with uniform
// branches: the Bdt columns are broadcast LDS reads at constant addresses, with no
// column-id -> column dependent-load chain (the dynamic loop over the step's columns waited on
// two LDS round trips per column). st(w, val) stores the entry.
template <class St>
__device__ __forceinline__ void step_columns(const float (*BdtT)[16], unsigned mi, int wb,
                                             const float* z, St&& st) {
  int w = wb;
  static_for<0, 4>([&](auto F) {
    constexpr int f = decltype(F)::value;
    if (mi & (1u << f)) {
      static_for<0, 3>([&](auto A) {
        constexpr int c = 3 * f + decltype(A)::value;
        float bw[16];
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const float4 b4 = *reinterpret_cast<const float4*>(&BdtT[c][4 * q]);
          bw[4 * q] = b4.x; bw[4 * q + 1] = b4.y; bw[4 * q + 2] = b4.z; bw[4 * q + 3] = b4.w;
        }
        st(w, 2.f * dot13(bw, z));
        w++;
      });
    }
  });
}

// quaternion (w,x,y,z) -> rotation matrix, as Eigen's toRotationMatrix (RobotState.cpp:36)
__device__ __forceinline__ void make_model(const float* __restrict__ rec, float dt, Model& md) {
  const float qw = rec[CMPC_REC_Q + 0], qx = rec[CMPC_REC_Q + 1], qy = rec[CMPC_REC_Q + 2],
              qz = rec[CMPC_REC_Q + 3];
  const float tx = 2.f * qx, ty = 2.f * qy, tz = 2.f * qz;
  const float twx = tx * qw, twy = ty * qw, twz = tz * qw;
  const float txx = tx * qx, txy = ty * qx, txz = tz * qx;
  const float tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
  md.R[0] = 1.f - (tyy + tzz); md.R[1] = txy - twz;         md.R[2] = txz + twy;
  md.R[3] = txy + twz;         md.R[4] = 1.f - (txx + tzz); md.R[5] = tyz - twx;
  md.R[6] = txz - twy;         md.R[7] = tyz + twx;         md.R[8] = 1.f - (txx + tyy);
  md.dt = dt;
  md.dth = dt * dt * 0.5f;
  md.xdrag = rec[CMPC_REC_XDRAG];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) md.n1r[i * 3 + j] = dt * md.R[j * 3 + i];
}

// Bdt[s][c] -> BdtT[c][s]: thread c < 12 (c = 3 leg + axis) builds column c, every row s
// unrolled (constant indices only: a row-strided mapping turned the R lookups into a private
// array on scratch). ct_ss_mats B_c rows 6..11: I_world^-1 [r]x, I/m; SolverMPC.cpp:267-276,
// m = 12 RobotState.h:26, I_body = diag(.07, .26, .242) RobotState.h:25;
// I_world = R I_body R^T, SolverMPC.cpp:593.
template <int NT>
__device__ __forceinline__ void make_bdt(const float* __restrict__ rec, const Model& md, int tid,
                                         float (*BdtT)[16]) {
  static_assert(NT >= 12, "one thread per force column");
  if (tid < 12) {
    const float Ib0 = .07f, Ib1 = 0.26f, Ib2 = 0.242f;
    float Iw[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int j = 0; j < 3; j++)
        Iw[i * 3 + j] = md.R[i * 3 + 0] * Ib0 * md.R[j * 3 + 0] + md.R[i * 3 + 1] * Ib1 * md.R[j * 3 + 1] +
                        md.R[i * 3 + 2] * Ib2 * md.R[j * 3 + 2];
    const float c00 = Iw[4] * Iw[8] - Iw[5] * Iw[7];
    const float c10 = Iw[5] * Iw[6] - Iw[3] * Iw[8];
    const float c20 = Iw[3] * Iw[7] - Iw[4] * Iw[6];
    const float idet = 1.f / (Iw[0] * c00 + Iw[1] * c10 + Iw[2] * c20);
    float Ii[9];
    Ii[0] = c00 * idet; Ii[1] = (Iw[2] * Iw[7] - Iw[1] * Iw[8]) * idet; Ii[2] = (Iw[1] * Iw[5] - Iw[2] * Iw[4]) * idet;
    Ii[3] = c10 * idet; Ii[4] = (Iw[0] * Iw[8] - Iw[2] * Iw[6]) * idet; Ii[5] = (Iw[2] * Iw[3] - Iw[0] * Iw[5]) * idet;
    Ii[6] = c20 * idet; Ii[7] = (Iw[1] * Iw[6] - Iw[0] * Iw[7]) * idet; Ii[8] = (Iw[0] * Iw[4] - Iw[1] * Iw[3]) * idet;
    const float im = 1.f / 12.0f;
    const float dt = md.dt, dt2 = md.dth, dt3 = md.dt * md.dt * md.dt / 6.f;
    const int c = tid;
    const int b = c / 3, a = c - 3 * (c / 3);
    const float r0 = rec[CMPC_REC_R + 0 * 4 + b], r1 = rec[CMPC_REC_R + 1 * 4 + b],
                r2 = rec[CMPC_REC_R + 2 * 4 + b];
    // column a of [r]x
    const float cx0 = (a == 0) ? 0.f : (a == 1) ? -r2 : r1;
    const float cx1 = (a == 0) ? r2 : (a == 1) ? 0.f : -r0;
    const float cx2 = (a == 0) ? -r1 : (a == 1) ? r0 : 0.f;
    float T[3];  // B_c[6+i][c] = (I_inv [r]x)[i][a]
#pragma unroll
    for (int i = 0; i < 3; i++) T[i] = Ii[i * 3 + 0] * cx0 + Ii[i * 3 + 1] * cx1 + Ii[i * 3 + 2] * cx2;
    const float e0 = (a == 0) ? im : 0.f, e1 = (a == 1) ? im : 0.f, e2 = (a == 2) ? im : 0.f;
    float* col = BdtT[c];
#pragma unroll
    for (int s = 0; s < 3; s++)  // dt^2/2 * N1-part: R^T (I_inv [r]x)
      col[s] = dt2 * (md.R[0 * 3 + s] * T[0] + md.R[1 * 3 + s] * T[1] + md.R[2 * 3 + s] * T[2]);
    col[3] = dt2 * e0;
    col[4] = dt2 * e1;
    col[5] = dt2 * e2 + dt3 * md.xdrag * e0;
#pragma unroll
    for (int s = 0; s < 3; s++) col[6 + s] = dt * T[s];
    col[9] = dt * e0;
    col[10] = dt * e1;
    col[11] = dt * e2 + dt2 * md.xdrag * e0;
    col[12] = 0.f;
    col[13] = 0.f;
    col[14] = 0.f;
    col[15] = 0.f;
  }
}

// rpy of the record's quaternion as the reference's quat_to_rpy (SolverMPC.cpp:352-361), fp32
template <typename RecPtr>  // const float* or a global-address-space pointer
__device__ __forceinline__ void quat_to_rpy(RecPtr rec, float* rpy) {
  const float qw = rec[CMPC_REC_Q + 0], qx = rec[CMPC_REC_Q + 1], qy = rec[CMPC_REC_Q + 2],
              qz = rec[CMPC_REC_Q + 3];
  float as = -2.f * (qx * qz - qw * qy);
  as = fminf(as, 0.99999f);  // only the upper clamp, as the reference
  rpy[0] = atan2f(2.f * (qy * qz + qw * qx), qw * qw - qx * qx - qy * qy + qz * qz);
  rpy[1] = asinf(as);
  rpy[2] = atan2f(2.f * (qx * qy + qw * qz), qw * qw + qx * qx - qy * qy - qz * qz);
}

// e_i = Adt^{i+1} x0 + sum_{k<=i} Adt^k Qdt f - X_d,i for step i (SolverMPC.cpp:592, 633-642,
// 808-814). x0 = [rpy, p, w, v, -9.8] with rpy from quat_to_rpy (SolverMPC.cpp:352-361).
__device__ __forceinline__ void state_error(const float* __restrict__ rec, const Model& md, int i,
                                            const float* traj_i, float* e) {
  float x0[13];
  {
    quat_to_rpy(rec, x0);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      x0[3 + k] = rec[CMPC_REC_P + k];
      x0[6 + k] = rec[CMPC_REC_W + k];
      x0[9 + k] = rec[CMPC_REC_V + k];
    }
    x0[12] = -9.8f;
  }
  float X1[13], X2[13], qf[13], F1[13], F2[13];
  n1_mul(md, x0, X1);
  n1_mul(md, X1, X2);
  // Q_qp f with f = (0,0,0,f_est(3),0,0) when the history flag is set (SolverMPC.cpp:808-811)
  const uint32_t flags = __float_as_uint(rec[CMPC_REC_FLAGS]);
  const float f3 = (flags & 1u) ? rec[CMPC_REC_FEST3] : 0.f;
#pragma unroll
  for (int j = 0; j < 13; j++) qf[j] = 0.f;
  // Qdt[:,3] = dt e9 + dt^2/2 (e3 + xdrag e11) + dt^3/6 xdrag e5
  qf[9] = md.dt * f3;
  qf[3] = md.dth * f3;
  qf[11] = md.dth * md.xdrag * f3;
  qf[5] = (md.dt * md.dt * md.dt / 6.f) * md.xdrag * f3;
  n1_mul(md, qf, F1);
  n1_mul(md, F1, F2);
  const float m1 = (float)(i + 1);
  const float m2 = 0.5f * m1 * (float)i;
  const float s2 = 0.5f * (float)i * (float)(i + 1);
  const float s3 = (float)(i + 1) * (float)i * (float)(i - 1) / 6.f;
#pragma unroll
  for (int j = 0; j < 13; j++) {
    float ev = x0[j] + m1 * X1[j] + m2 * X2[j] + m1 * qf[j] + s2 * F1[j] + s3 * F2[j];
    if (j < 12) ev -= traj_i[j];
    e[j] = ev;
  }
}

// v_readlane of a double (lane uniform)
__device__ __forceinline__ double rl_d(double x, int lane) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (long long)(unsigned)lo);
}

// Friction-pyramid constraint c = 6 s + t of stance foot-step s (reduced vars 3s, 3s+1, 3s+2):
//   t = 0..3: +-fx/mu + fz >= 0, +-fy/mu + fz >= 0 ; t = 4: fz >= 0 ; t = 5: -fz >= -ub
// (fmat rows of SolverMPC.cpp:657-665 with lb = 0, ub = BIG / gait*f_max)
struct Cons {
  int ia, iz;
  float ca, cb, bp;
};
__device__ __forceinline__ Cons decode_cons(int c, float mui, float sub_s) {
  Cons k;
  const int sft = c / 6, t = c - 6 * (c / 6);
  k.iz = 3 * sft + 2;
  if (t < 4) {
    k.ia = 3 * sft + (t >> 1);
    k.ca = (t & 1) ? -mui : mui;
    k.cb = 1.f;
    k.bp = 0.f;
  } else {
    k.ia = k.iz;
    k.ca = 0.f;
    k.cb = (t == 4) ? 1.f : -1.f;
    k.bp = (t == 4) ? 0.f : -sub_s;
  }
  return k;
}

}  // namespace
}  // namespace cmpc
