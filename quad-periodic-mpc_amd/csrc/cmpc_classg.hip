// cmpc_classg.hip — the general size class: any reduced size n <= 12 * CMPC_MAX_HORIZON.
//
// Instances too large for the register-resident classes (n > 128: e.g. N = 20 with more than
// 43 stance foot-steps, the all-stance edge cases) come here through the overflow list of the
// previous class. Same math as cmpc_class1.hip (solve_mpc(), SolverMPC.cpp:566-982), but with
// run-time loops and the n x n working matrices (H -> L, and J = L^-T) in a per-workgroup slab
// of global memory (L2-resident; hipMalloc'ed at handle creation), so it compiles in seconds and
// handles every size. One 256-thread workgroup per instance, persistent over the list.
#include "cmpc_common.h"

namespace cmpc {
namespace {

constexpr int NTG = 256;
constexpr int NWG = NTG / 64;
constexpr int NMAX = 12 * MAXN;

struct SharedG {
  float BdtT[12][16];
  float traj[12 * MAXN];
  float E[MAXN][16];
  float ZE[MAXN][16];
  float g[NMAX];        // gradient -> forward-solved y
  float lcol[NMAX];     // pivot column of the Cholesky / scratch vector
  float ivec[NMAX];     // 1 / L[k][k]
  float xs[NMAX];       // primal iterate
  float dvec[NMAX];     // d = J' n+
  float m[NMAX];        // back-substitution accumulator sum_{j>i} r_j n_j
  float rvec[NMAX];     // r = R^-1 d1
  float u[NMAX];        // duals of the active set
  int act[NMAX];        // active constraint ids
  float cs[2 * NMAX];   // Givens (c, s)
  float sub[4 * MAXN];
  int sfs[4 * MAXN];
  int blkbase[MAXN + 2];
  unsigned char varblk[NMAX], varcol[NMAX];
  unsigned char stance[4 * MAXN];
  unsigned char cflag[6 * 4 * MAXN];
  float red_f[NWG];
  int red_i[NWG];
  int ctrl[8];
  float fctrl[8];
};

__device__ __forceinline__ float block_sum(float v, SharedG& sh) {
  v = wave_sum(v);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh.red_f[wv] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NWG; i++) s += sh.red_f[i];
  __syncthreads();
  return s;
}
__device__ __forceinline__ float block_max(float v, SharedG& sh) {
  v = wave_max(v);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh.red_f[wv] = v;
  __syncthreads();
  float s = sh.red_f[0];
#pragma unroll
  for (int i = 1; i < NWG; i++) s = fmaxf(s, sh.red_f[i]);
  __syncthreads();
  return s;
}
__device__ __forceinline__ void block_argmin(float& v, int& idx, SharedG& sh) {
  wave_argmin(v, idx);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh.red_f[wv] = v; sh.red_i[wv] = idx; }
  __syncthreads();
  v = sh.red_f[0];
  idx = sh.red_i[0];
#pragma unroll
  for (int i = 1; i < NWG; i++) {
    const float ov = sh.red_f[i];
    const int oi = sh.red_i[i];
    if (ov < v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
  __syncthreads();
}

// One instance. A: n x n (stride ld) slab for H -> L (lower), J: n x n slab (row v = row v of J).
__device__ void solve_g(const float* __restrict__ rec, const KParams& P, SharedG& sh,
                        float* __restrict__ A, float* __restrict__ J, int ld,
                        float* __restrict__ fout, uint8_t* __restrict__ st_out,
                        int32_t* __restrict__ it_out, bool condense_only,
                        float* __restrict__ Hout, float* __restrict__ gout) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int N = P.N;
  const unsigned char* gait = reinterpret_cast<const unsigned char*>(rec + CMPC_REC_HDR + 12 * N);
  // ---- stance table (SolverMPC.cpp:869-894); condense_only keeps every variable ----------
  for (int t = tid; t < 4 * N; t += NTG) {
    const float ub = (float)gait[t] * P.f_max;
    sh.stance[t] = (condense_only || !(ub < 0.01f && ub > -0.01f)) ? 1 : 0;
  }
  for (int t = tid; t < 12 * N; t += NTG) sh.traj[t] = rec[CMPC_REC_HDR + t];
  __syncthreads();
  if (tid < 64) {
    int base = 0;
    for (int c0 = 0; c0 < 4 * N; c0 += 64) {
      const int t = c0 + lane;
      const bool f = (t < 4 * N) && sh.stance[t];
      const unsigned long long mk = __ballot(f);
      const int pre = __popcll(mk & ((1ull << lane) - 1ull));
      if (f) {
        sh.sfs[base + pre] = t;
        sh.sub[base + pre] = (float)gait[t] * P.f_max;
      }
      base += __popcll(mk);
    }
    if (lane == 0) sh.ctrl[0] = base;
  }
  __syncthreads();
  const int nfs = sh.ctrl[0];
  const int n = 3 * nfs;
  for (int t = tid; t < n; t += NTG) {
    const int fs = sh.sfs[t / 3];
    sh.varblk[t] = (unsigned char)(fs >> 2);
    sh.varcol[t] = (unsigned char)(3 * (fs & 3) + t % 3);
  }
  for (int i = tid; i <= N; i += NTG) {
    int c = 0;
    for (int s = 0; s < nfs; s++) c += (sh.sfs[s] < 4 * i) ? 1 : 0;
    sh.blkbase[i] = 3 * c;
  }
  for (int t = tid; t < 6 * nfs; t += NTG) sh.cflag[t] = 0;
  Model md;
  make_model(rec, P.dt, md);
  make_bdt<NTG>(rec, md, tid, sh.BdtT);
  __syncthreads();
  if (tid < N) {
    float e[13];
    state_error(rec, md, tid, &sh.traj[12 * tid], e);
#pragma unroll
    for (int j = 0; j < 13; j++) sh.E[tid][j] = e[j];
  }
  __syncthreads();
  float wts[13];
#pragma unroll
  for (int j = 0; j < 12; j++) wts[j] = P.wts[j];
  wts[12] = 0.f;
  if (tid < 64) {
    float ze[13];
#pragma unroll
    for (int j = 0; j < 13; j++) ze[j] = 0.f;
    for (int i = N - 1; i >= 0; i--) {
      float e[13];
#pragma unroll
      for (int j = 0; j < 13; j++) e[j] = sh.E[i][j];
      recur(md, wts, e, ze);
      if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 13; j++) sh.ZE[i][j] = ze[j];
      }
    }
  }
  __syncthreads();

  // ---- condensation: H (full symmetric, in A) and g -----------------------------------------
  for (int v = tid; v < n; v += NTG) {
    const int kv = sh.varblk[v], cv = sh.varcol[v];
    float b[13], u1[13], u2[13];
#pragma unroll
    for (int j = 0; j < 13; j++) b[j] = sh.BdtT[cv][j];
    n1_mul(md, b, u1);
    n1_mul(md, u1, u2);
    {
      float zk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) zk[j] = sh.ZE[kv][j];
      sh.g[v] = 2.f * dot13(b, zk);
    }
    float z[13];
#pragma unroll
    for (int j = 0; j < 13; j++) z[j] = 0.f;
    for (int i = N - 1; i >= kv; i--) {
      const float k = (float)(i - kv);
      const float k2 = 0.5f * k * (k - 1.f);
      float gk[13];
#pragma unroll
      for (int j = 0; j < 13; j++) gk[j] = fmaf(k2, u2[j], fmaf(k, u1[j], b[j]));
      recur(md, wts, gk, z);
      const int we = sh.blkbase[i + 1];
      for (int w = max(sh.blkbase[i], v); w < we; w++) {
        const int cw = sh.varcol[w];
        float bw[13];
#pragma unroll
        for (int j = 0; j < 13; j++) bw[j] = sh.BdtT[cw][j];
        float val = 2.f * dot13(bw, z);
        if (w == v) val += P.alpha2;  // qH = 2 (B'SB + alpha I)
        A[(size_t)v * ld + w] = val;
        A[(size_t)w * ld + v] = val;
      }
    }
  }
  __syncthreads();
  if (condense_only) {  // parity hook: the full qH / qg (nothing eliminated, v == 12 k + c)
    for (int e = tid; e < n * n; e += NTG) Hout[e] = A[(size_t)(e / n) * ld + e % n];
    for (int v = tid; v < n; v += NTG) gout[v] = sh.g[v];
    return;
  }

  // ---- right-looking Cholesky of A in place (lower), bordered with g -> y ------------------
  int status = CMPC_OK;
  const int wv = tid >> 6;
  for (int k = 0; k < n; k++) {
    float d = A[(size_t)k * ld + k];
    if (!(d > 0.f)) { status = CMPC_NOT_PD; d = 1e-30f; }
    const float inv = rsqrtf(d);
    for (int i = k + 1 + tid; i < n; i += NTG) {
      const float l = A[(size_t)i * ld + k] * inv;
      A[(size_t)i * ld + k] = l;
      sh.lcol[i] = l;
    }
    if (tid == 0) {
      sh.ivec[k] = inv;
      const float yk = sh.g[k] * inv;
      sh.g[k] = yk;
      A[(size_t)k * ld + k] = d * inv;
    }
    __syncthreads();
    const float yk = sh.g[k];
    for (int i = k + 1 + tid; i < n; i += NTG) sh.g[i] = fmaf(-sh.lcol[i], yk, sh.g[i]);
    // trailing update of the lower triangle, one row per wave, lanes along the row
    for (int i = k + 1 + wv; i < n; i += NWG) {
      const float li = sh.lcol[i];
      float* Ai = A + (size_t)i * ld;
      for (int j = k + 1 + lane; j <= i; j += 64) Ai[j] = fmaf(-li, sh.lcol[j], Ai[j]);
    }
    __syncthreads();
  }
  // ---- J = L^-T: thread v solves L x = e_v, x = row v of J ---------------------------------
  for (int v = tid; v < n; v += NTG) {
    float* Jv = J + (size_t)v * ld;
    for (int k = 0; k < v; k++) Jv[k] = 0.f;
    for (int k = v; k < n; k++) {
      const float* Lk = A + (size_t)k * ld;
      float s = (k == v) ? 1.f : 0.f;
      for (int j = v; j < k; j++) s = fmaf(-Lk[j], Jv[j], s);
      Jv[k] = s * sh.ivec[k];
    }
  }
  __syncthreads();
  // ---- x = -J y ------------------------------------------------------------------------------
  for (int v = tid; v < n; v += NTG) {
    const float* Jv = J + (size_t)v * ld;
    float s = 0.f;
    for (int c = v; c < n; c++) s = fmaf(Jv[c], sh.g[c], s);
    sh.xs[v] = -s;
  }
  __syncthreads();

  // ---- Goldfarb-Idnani dual active set (R[i][j] = J[:,i]' n_act_j, implicit) --------------
  const float mui = P.mu_inv;
  const float fnorm = rsqrtf(mui * mui + 1.f);
  int q = 0, iters = 0;
  if (status == CMPC_OK && n > 0) {
    for (;;) {
      float best = 0.f, xm = 0.f;
      int bid = 0x7fffffff;
      for (int s = tid; s < nfs; s += NTG) {
        const float fx = sh.xs[3 * s], fy = sh.xs[3 * s + 1], fz = sh.xs[3 * s + 2];
        xm = fmaxf(xm, fmaxf(fabsf(fx), fmaxf(fabsf(fy), fabsf(fz))));
        float sl[6];
        sl[0] = (mui * fx + fz) * fnorm;
        sl[1] = (-mui * fx + fz) * fnorm;
        sl[2] = (mui * fy + fz) * fnorm;
        sl[3] = (-mui * fy + fz) * fnorm;
        sl[4] = fz;
        sl[5] = sh.sub[s] - fz;
#pragma unroll
        for (int t = 0; t < 6; t++)
          if (!sh.cflag[6 * s + t] && sl[t] < best) { best = sl[t]; bid = 6 * s + t; }
      }
      const float xmax = block_max(xm, sh);
      block_argmin(best, bid, sh);
      const float tol = 1e-5f * fmaxf(1.f, xmax);
      if (bid == 0x7fffffff || best >= -tol) break;
      const int p = bid;
      const Cons cp = decode_cons(p, mui, sh.sub[p / 6]);
      float up = 0.f;
      for (;;) {
        if (++iters > P.max_iter + 2 * n) { status = CMPC_MAX_ITER; break; }
        // d = J' n+
        const float* Ja = J + (size_t)cp.ia * ld;
        const float* Jz = J + (size_t)cp.iz * ld;
        float dsq = 0.f, d2sq = 0.f;
        for (int i = tid; i < n; i += NTG) {
          const float di = (cp.ia != cp.iz) ? fmaf(cp.ca, Ja[i], cp.cb * Jz[i]) : cp.cb * Jz[i];
          sh.dvec[i] = di;
          dsq += di * di;
          d2sq += (i >= q) ? di * di : 0.f;
        }
        const float dn = block_sum(dsq, sh);
        const float zn = block_sum(d2sq, sh);
        // r = R^-1 d1 by back substitution through m = sum_{j>i} r_j n_j
        for (int v = tid; v < n; v += NTG) sh.m[v] = 0.f;
        __syncthreads();
        for (int i = q - 1; i >= 0; i--) {
          float part = 0.f;
          for (int v = tid; v < n; v += NTG) part = fmaf(J[(size_t)v * ld + i], sh.m[v], part);
          const float sdot = block_sum(part, sh);
          if (tid == 0) {
            const Cons ci = decode_cons(sh.act[i], mui, sh.sub[sh.act[i] / 6]);
            const float Rii = fmaf(ci.ca, J[(size_t)ci.ia * ld + i], ci.cb * J[(size_t)ci.iz * ld + i]);
            const float ri = (sh.dvec[i] - sdot) / Rii;
            sh.rvec[i] = ri;
            if (ci.ia != ci.iz) sh.m[ci.ia] += ci.ca * ri;
            sh.m[ci.iz] += ci.cb * ri;
          }
          __syncthreads();
        }
        // step lengths
        float t1 = kBigF;
        int kk = 0x7fffffff;
        for (int j = tid; j < q; j += NTG) {
          const float rj = sh.rvec[j];
          if (rj > 0.f) {
            const float tj = fmaxf(sh.u[j] / rj, 0.f);
            if (tj < t1) { t1 = tj; kk = j; }
          }
        }
        block_argmin(t1, kk, sh);
        const float spv = fmaf(cp.ca, sh.xs[cp.ia], fmaf(cp.cb, sh.xs[cp.iz], -cp.bp));
        const bool zero_step = !(zn > 1e-9f * dn);
        const float t2 = zero_step ? kBigF : -spv / zn;
        const float t = fminf(t1, t2);
        if (t >= kBigF) { status = CMPC_INFEASIBLE; break; }
        // z = J2 d2 (row dots) and the primal / dual updates
        if (!zero_step) {
          for (int v = tid; v < n; v += NTG) {
            const float* Jv = J + (size_t)v * ld;
            float z = 0.f;
            for (int c = q; c < n; c++) z = fmaf(Jv[c], sh.dvec[c], z);
            sh.xs[v] = fmaf(t, z, sh.xs[v]);
          }
        }
        for (int j = tid; j < q; j += NTG) sh.u[j] = fmaf(-t, sh.rvec[j], sh.u[j]);
        up += t;
        __syncthreads();
        if (!zero_step && t2 <= t1) {
          // add p: rotations zeroing d[q+1..n-1] into d[q] (bottom up), applied to J columns
          if (tid == 0) {
            float h = sh.dvec[n - 1];
            for (int j = n - 1; j > q; j--) {
              const float a0 = sh.dvec[j - 1];
              const float r = sqrtf(a0 * a0 + h * h);
              float c = 1.f, s = 0.f;
              if (r > 0.f) { c = a0 / r; s = h / r; }
              sh.cs[2 * j] = c;
              sh.cs[2 * j + 1] = s;
              h = r;
            }
            sh.act[q] = p;
            sh.u[q] = up;
            sh.cflag[p] = 1;
          }
          __syncthreads();
          for (int v = tid; v < n; v += NTG) {
            float* Jv = J + (size_t)v * ld;
            for (int j = n - 1; j > q; j--) {
              const float c = sh.cs[2 * j], s = sh.cs[2 * j + 1];
              const float a0 = Jv[j - 1], b0 = Jv[j];
              Jv[j - 1] = fmaf(c, a0, s * b0);
              Jv[j] = fmaf(-s, a0, c * b0);
            }
          }
          q++;
          __syncthreads();
          break;
        }
        // drop kk and re-triangularise (rotations on J columns kk..q-1)
        const int k = kk;
        if (tid == 0) {
          sh.cflag[sh.act[k]] = 0;
          for (int j = k; j < q - 1; j++) { sh.act[j] = sh.act[j + 1]; sh.u[j] = sh.u[j + 1]; }
        }
        __syncthreads();
        for (int j = k; j < q - 1; j++) {
          if (tid == 0) {
            const Cons cj = decode_cons(sh.act[j], mui, sh.sub[sh.act[j] / 6]);
            const float a0 = fmaf(cj.ca, J[(size_t)cj.ia * ld + j], cj.cb * J[(size_t)cj.iz * ld + j]);
            const float b0 = fmaf(cj.ca, J[(size_t)cj.ia * ld + j + 1], cj.cb * J[(size_t)cj.iz * ld + j + 1]);
            const float h = sqrtf(a0 * a0 + b0 * b0);
            float c = 1.f, s = 0.f;
            if (h > 0.f) { c = a0 / h; s = b0 / h; }
            sh.fctrl[0] = c;
            sh.fctrl[1] = s;
          }
          __syncthreads();
          const float c = sh.fctrl[0], s = sh.fctrl[1];
          for (int v = tid; v < n; v += NTG) {
            float* Jv = J + (size_t)v * ld;
            const float x0 = Jv[j], x1 = Jv[j + 1];
            Jv[j] = fmaf(c, x0, s * x1);
            Jv[j + 1] = fmaf(-s, x0, c * x1);
          }
          __syncthreads();
        }
        q--;
      }
      if (status != CMPC_OK) break;
    }
  }
  __syncthreads();
  // ---- scatter (staged in LDS, then one coalesced pass) ----------------------------------
  const bool ok = (status == CMPC_OK);
  for (int t = tid; t < 12 * N; t += NTG) sh.lcol[t] = 0.f;
  __syncthreads();
  if (ok)
    for (int v = tid; v < n; v += NTG) sh.lcol[12 * sh.varblk[v] + sh.varcol[v]] = sh.xs[v];
  __syncthreads();
  for (int t = tid; t < 12 * N; t += NTG) fout[t] = sh.lcol[t];
  if (tid == 0) {
    st_out[0] = (uint8_t)status;
    if (it_out) it_out[0] = iters;
  }
}

}  // namespace

// Persistent grid over an instance list (in_list == nullptr: instances 0..batch-1). Workgroup b
// owns the slab pair at scratch + b * 2 * ld * ld.
__global__ __launch_bounds__(NTG) void cmpc_solve_g_kernel(
    const float* __restrict__ recs, int batch, KParams P, float* __restrict__ forces,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, const int* __restrict__ in_list,
    const int* __restrict__ in_count, float* __restrict__ scratch, float* __restrict__ Hout,
    float* __restrict__ gout) {
  __shared__ SharedG sh;
  const int ld = 12 * P.N;
  float* A = scratch + (size_t)blockIdx.x * 2 * ld * ld;
  float* J = A + (size_t)ld * ld;
  const int count = in_list ? *in_count : batch;
  for (int t = blockIdx.x; t < count; t += gridDim.x) {
    const int inst = in_list ? in_list[t] : t;
    solve_g(recs + (size_t)inst * P.rec_words, P, sh, A, J, ld, forces + (size_t)inst * 12 * P.N,
            status + inst, iters ? iters + inst : nullptr, Hout != nullptr,
            Hout ? Hout + (size_t)inst * ld * ld : nullptr, gout ? gout + (size_t)inst * ld : nullptr);
    __syncthreads();
  }
}

size_t classg_scratch_floats(int horizon, int grid) {
  const size_t ld = 12 * (size_t)horizon;
  return 2 * ld * ld * (size_t)grid;
}

hipError_t launch_classg(const float* d_recs, int batch, const KParams& P, float* d_forces,
                         uint8_t* d_status, int32_t* d_iters, const int* in_list, const int* in_count,
                         float* scratch, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(cmpc_solve_g_kernel, dim3(grid), dim3(NTG), 0, stream, d_recs, batch, P,
                     d_forces, d_status, d_iters, in_list, in_count, scratch, nullptr, nullptr);
  return hipGetLastError();
}

hipError_t launch_condense(const float* d_recs, int batch, const KParams& P, float* d_H, float* d_g,
                           float* scratch, int grid, hipStream_t stream) {
  if (batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_solve_g_kernel, dim3(grid), dim3(NTG), 0, stream, d_recs, batch, P,
                     nullptr, nullptr, nullptr, nullptr, nullptr, scratch, d_H, d_g);
  return hipGetLastError();
}

}  // namespace cmpc
