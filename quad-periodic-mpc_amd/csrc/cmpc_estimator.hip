// cmpc_estimator.hip — config 5: the periodic-disturbance estimator of solve_mpc, batched.
//
// Per instance and per MPC step, what the reference does in globals of SolverMPC.cpp before it
// condenses (SolverMPC.cpp:688-811), preceded by the caller's residual when LogData records are
// given (ConvexMPCLocomotion.cpp:639-771):
//   f_ext = x_k - A_prev x_prev - B_prev u_prev  (continuous model of the logged step, no dt)
//   push (f_ext[3], simulation_time); while 400 <= count <= 500:
//     band = gaussian_filter(window, 7) - gaussian_filter(window, 27)   (SolverMPC.cpp:404-437)
//     fit_sin: peak |rfft| bin >= 1, amp = sqrt(2) std, offset = mean   (SolverMPC.cpp:478-541)
//   count >= 400: f_est(3) = est_amp + sin(2 pi t est_freq + est_phase)  (sic '+', :766)
//   qg uses f_est only when count > 500 (:808) -> record flag bit 0.
//
// MI355X mapping: one 128-thread workgroup (two wavefronts) per instance; the 400-sample window
// is staged in LDS as double. Everything is fp64, as the reference.
//   * band-pass: thread t < 100 produces the four consecutive output samples 4t..4t+3 of both
//     Gaussian FIRs (43 and 163 float taps, computed on the host exactly as the reference does,
//     widened to double in LDS). Per tap one LDS read extends a 4-sample sliding window in
//     registers and feeds four fp64 FMAs; taps are accumulated in ascending order per output,
//     as gaussian_filter does;
//   * DFT peak: a 400-point Stockham FFT of the band in LDS (radices 4, 4, 5, 5; twiddles from a
//     quarter-period table of 100 sincospi values, the other quarters by symmetry), then thread
//     t < 100 takes |X_k|^2 of bins t+1 and t+101; the first maximum over bins 1..200 (the
//     reference's rfft agrees to ~1e-13 relative on the magnitudes). It replaced round 2's 200
//     Goertzel recurrences (400 dependent fp64 steps each): 1.03 -> 0.75 ms at config 5;
//   * mean / std / argmax: wave butterflies plus one LDS exchange.
// Instances outside the estimation window only push their sample (a few words of HBM traffic)
// and evaluate the compensation.
#include "cmpc_common.h"

namespace cmpc {
namespace {

constexpr int W = CMPC_EST_WINDOW;
constexpr int NT = 128;
constexpr int NWV = NT / 64;
constexpr int NBIN = W / 2;  // bins 1..200 are searched (bin 0 excluded, SolverMPC.cpp:503-510)
constexpr int NOUT = 4;      // FIR outputs per thread
constexpr int NFIR = W / NOUT;
constexpr int NTAPS7 = 2 * kGaussR7 + 1, NTAPS27 = 2 * kGaussR27 + 1;
static_assert(W % NOUT == 0 && NFIR <= NT && NBIN <= 2 * NT, "estimator thread mapping");

// DFT of the band: mixed-radix Stockham FFT (radices 4, 4, 5, 5) in LDS, one pass per stage:
// thread j < W / R handles sub-transform j of a radix-R stage, so every stage needs W / 4 threads
static_assert(W == 400, "the FFT's radix plan is 4 * 4 * 5 * 5");
static_assert(NT >= W / 4, "fft_stage has no stride loop: one thread per radix-4 butterfly");
constexpr int QW = W / 4;  // quarter-period twiddle table

// LDS slots. Layout 2's XOR swizzles inside aligned 4- / 16-element groups (no padding), chosen
// with a bank model of every LDS access of this kernel (scripts/lds_bank_model.py; the rules of
// MI355X_MICROARCH.md §LDS: ds_read_b64 serves 32 lanes on 64 banks, ds_write_b64 16 lanes on 32,
// ds_read_b128 4 x 16 lanes on 64, ds_write_b128 8 x 8 lanes on 32). Modelled extra LDS cycles per
// instance: 541 with round 3's one pad slot per 8 window samples and plain band / FFT buffers (0.75
// conflicts per LDS instruction in the counters), 66 with these (+38 in the twiddle gathers):
//  * dslot (fp64 window and band): the FIR's lane t reads sample 4t + c (32 B apart) and the band
//    is stored the same way; the low two bits are XORed with bits 3 and 5 of the index, so a
//    32-lane read and a 16-lane store both land every lane on its own bank pair;
//  * fslot<1> (stage 1 / 3 outputs, 16 B): stage 1 stores element 4j + m (lanes 64 B apart): the low
//    two bits XOR bits 3-4, so 8 consecutive lanes hit 8 bank groups;
//  * fslot<2> (stage 2 / 4 outputs): stage 2 stores 16 (j / 4) + j % 4 + 4 m: bits 2-3 XOR bits 4-5.
// Contiguous reads stay conflict-free: each element stays in its aligned 4-group (16-block for
// fslot<2>), so a run's residues modulo the bank count are only permuted.
// Measured (config 5, rocprofv3 kernel stats + SQ_LDS_BANK_CONFLICT, scripts/gpu_est_ab.sh,
// profiles/r05_est): layout 0 (round 3: window padded 1 / 8, plain band and FFT buffers) 748 us at
// 0.754 conflicts per LDS instruction; 3 (+ the FFT swizzles) 760 us at 0.630; 1 (window and band
// padded 1 / 32 + FFT swizzles) 798 us at 0.466; 2 (XOR swizzles everywhere) 874 us at 0.140. The
// swizzles' address arithmetic (+800 VALU instructions per wave at layout 2) costs more than the
// conflicts they remove: the kernel is issue-bound (issue-stall 0.37-0.40 of its wave cycles), not
// LDS-bound, so layout 0 stays the product build.
#ifndef CMPC_EST_LAYOUT
#define CMPC_EST_LAYOUT 0
#endif
#if CMPC_EST_LAYOUT == 0 || CMPC_EST_LAYOUT == 3
constexpr int kDPad = W / 8;
__device__ __forceinline__ int dslot(int i) { return i + (i >> 3); }
__device__ __forceinline__ int bslot(int i) { return i; }
#elif CMPC_EST_LAYOUT == 1
constexpr int kDPad = W / 32 + 1;
__device__ __forceinline__ int dslot(int i) { return i + (i >> 5); }
__device__ __forceinline__ int bslot(int i) { return i + (i >> 5); }
#else
constexpr int kDPad = 0;
__device__ __forceinline__ int dslot(int i) { return i ^ (((i >> 3) ^ (i >> 5)) & 3); }
__device__ __forceinline__ int bslot(int i) { return dslot(i); }
#endif
template <int L>
__device__ __forceinline__ int fslot(int e) {
  if constexpr (CMPC_EST_LAYOUT == 0) return e;
  else if constexpr (L == 1) return e ^ ((e >> 3) & 3);
  else return e ^ (((e >> 4) & 3) << 2);
}

struct SharedE {
  union {
    struct {
      double d[W + kDPad];  // window, oldest first, at dslot(i)
      double k7[NTAPS7], k27[NTAPS27];
    } fir;
    double2 fa[W];  // FFT stages 1 / 3 output (the FIR's inputs are dead by then)
  };
  union {
    double band[W + kDPad];  // blur7 - blur27, at bslot(i)
    double2 fb[W];   // FFT stages 2 / 4 output (the band is dead after stage 1)
  };
  double2 tw[QW];  // e^{-2 pi i m / W}, m < W / 4 (the other quarters by symmetry)
  double redd[NWV];
  int redi[NWV];
  int count, head;
  float t_now, t0, t1;
};

__device__ __forceinline__ double block_sum_d(double x, SharedE& sh) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off, 64);
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh.redd[wv] = x;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < NWV; i++) s += sh.redd[i];
  __syncthreads();
  return s;
}


// one Gaussian FIR over outputs i0..i0+3, edge-clamped, taps ascending (SolverMPC.cpp:419-436)
template <int R>
__device__ __forceinline__ void fir4(const double* __restrict__ d, const double* __restrict__ k,
                                     int i0, double (&acc)[NOUT]) {
  double win[NOUT];
#pragma unroll
  for (int r = 0; r < NOUT - 1; r++) win[r + 1] = d[dslot(min(max(i0 - R + r, 0), W - 1))];
#pragma unroll 8
  for (int j = -R; j <= R; j++) {
#pragma unroll
    for (int r = 0; r < NOUT - 1; r++) win[r] = win[r + 1];
    win[NOUT - 1] = d[dslot(min(max(i0 + j + NOUT - 1, 0), W - 1))];
    const double kj = k[j + R];
#pragma unroll
    for (int r = 0; r < NOUT; r++) acc[r] = fma(win[r], kj, acc[r]);
  }
}

__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
  return make_double2(fma(a.x, b.x, -a.y * b.y), fma(a.x, b.y, a.y * b.x));
}
// e^{-2 pi i k / W}, 0 <= k < W, from the quarter table: e^{-i pi q / 2} = (-i)^q
__device__ __forceinline__ double2 twid(const double2* __restrict__ T, int k) {
  const int q = k / QW, m = k - QW * q;
  const double2 t = T[m];
  return (q == 0) ? t : (q == 1) ? make_double2(t.y, -t.x) : (q == 2) ? make_double2(-t.x, -t.y)
                                                                        : make_double2(-t.y, t.x);
}
// one Stockham autosort stage of radix R over sub-transforms of length NS (NS = product of the
// earlier radices): thread j < W / R twiddles its R inputs in[j + r W/R] by e^{-2 pi i (j % NS) r /
// (NS R)}, takes their length-R DFT and writes out[(j / NS) NS R + j % NS + m NS]. The band enters
// stage 1 as real input (REAL_IN)
template <int R, int NS, bool REAL_IN, int LIN, int LOUT>
__device__ __forceinline__ void fft_stage(const double2* __restrict__ in, const double* __restrict__ in_re,
                                          double2* __restrict__ out, const double2* __restrict__ T, int j) {
  constexpr int M = W / R;
  if (j >= M) return;
  const int k = j % NS;
  double2 v[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    double2 x = REAL_IN ? make_double2(in_re[bslot(j + r * M)], 0.0) : in[fslot<LIN>(j + r * M)];
    if (NS > 1 && r > 0) x = cmul(x, twid(T, (k * r * (W / (NS * R))) % W));
    v[r] = x;
  }
  const int d = (j / NS) * NS * R + k;
#pragma unroll
  for (int m = 0; m < R; m++) {
    double2 acc = v[0];
#pragma unroll
    for (int r = 1; r < R; r++) {
      const int e = (r * m) % R;
      if (e == 0) {
        acc.x += v[r].x; acc.y += v[r].y;
      } else if (R == 4 && e == 2) {  // -1
        acc.x -= v[r].x; acc.y -= v[r].y;
      } else if (R == 4 && e == 1) {  // -i
        acc.x += v[r].y; acc.y -= v[r].x;
      } else if (R == 4 && e == 3) {  // +i
        acc.x -= v[r].y; acc.y += v[r].x;
      } else {
        const double2 c = cmul(v[r], twid(T, e * (W / R)));
        acc.x += c.x; acc.y += c.y;
      }
    }
    out[fslot<LOUT>(d + m * NS)] = acc;
  }
}

// residual of ConvexMPCLocomotion.cpp:639-771 for one instance (one thread)
__device__ void residual(const float* __restrict__ lg, const float* __restrict__ rec, float f_ext[6]) {
  const float* R = lg + CMPC_LOG_ROT;  // R_yaw of the logged step, row-major
  const float Ib[3] = {0.07f, 0.26f, 0.242f};
  float Iw[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++)
      Iw[i * 3 + j] = R[i * 3 + 0] * Ib[0] * R[j * 3 + 0] + R[i * 3 + 1] * Ib[1] * R[j * 3 + 1] +
                      R[i * 3 + 2] * Ib[2] * R[j * 3 + 2];
  const float c00 = Iw[4] * Iw[8] - Iw[5] * Iw[7];
  const float c10 = Iw[5] * Iw[6] - Iw[3] * Iw[8];
  const float c20 = Iw[3] * Iw[7] - Iw[4] * Iw[6];
  const float idet = 1.f / (Iw[0] * c00 + Iw[1] * c10 + Iw[2] * c20);
  float Ii[9];
  Ii[0] = c00 * idet; Ii[1] = (Iw[2] * Iw[7] - Iw[1] * Iw[8]) * idet; Ii[2] = (Iw[1] * Iw[5] - Iw[2] * Iw[4]) * idet;
  Ii[3] = c10 * idet; Ii[4] = (Iw[0] * Iw[8] - Iw[2] * Iw[6]) * idet; Ii[5] = (Iw[2] * Iw[3] - Iw[0] * Iw[5]) * idet;
  Ii[6] = c20 * idet; Ii[7] = (Iw[1] * Iw[6] - Iw[0] * Iw[7]) * idet; Ii[8] = (Iw[0] * Iw[4] - Iw[1] * Iw[3]) * idet;
  // B_prev u_prev, u_prev = -logged forces: rows 6..8 sum_b I_inv [r_b]x u_b, rows 9..11 sum_b u_b / m
  float tq[3] = {0.f, 0.f, 0.f}, fs[3] = {0.f, 0.f, 0.f};
  for (int b = 0; b < 4; b++) {
    const float r0 = lg[CMPC_LOG_R + 0 * 4 + b], r1 = lg[CMPC_LOG_R + 1 * 4 + b], r2 = lg[CMPC_LOG_R + 2 * 4 + b];
    const float u0 = -lg[CMPC_LOG_FORCE + 3 * b + 0], u1 = -lg[CMPC_LOG_FORCE + 3 * b + 1],
                u2 = -lg[CMPC_LOG_FORCE + 3 * b + 2];
    const float cm[9] = {0.f, -r2, r1, r2, 0.f, -r0, -r1, r0, 0.f};
#pragma unroll
    for (int i = 0; i < 3; i++) {
      float m0 = 0.f, m1 = 0.f, m2 = 0.f;  // (I_inv cm)[i][:]
#pragma unroll
      for (int k = 0; k < 3; k++) {
        m0 += Ii[i * 3 + k] * cm[k * 3 + 0];
        m1 += Ii[i * 3 + k] * cm[k * 3 + 1];
        m2 += Ii[i * 3 + k] * cm[k * 3 + 2];
      }
      tq[i] += m0 * u0 + m1 * u1 + m2 * u2;
    }
    fs[0] += (1.f / 12.f) * u0;
    fs[1] += (1.f / 12.f) * u1;
    fs[2] += (1.f / 12.f) * u2;
  }
  // A_prev x_prev: rows 6..10 are zero; row 11 = x_drag * v_x + x(12)
  const float ax11 = lg[CMPC_LOG_XDRAG] * lg[CMPC_LOG_LIN + 0] + (-9.81f);
  const float e6 = rec[CMPC_REC_W + 0] - tq[0];
  const float e7 = rec[CMPC_REC_W + 1] - tq[1];
  const float e8 = rec[CMPC_REC_W + 2] - tq[2];
  const float e9 = rec[CMPC_REC_V + 0] - fs[0];
  const float e10 = rec[CMPC_REC_V + 1] - fs[1];
  const float e11 = (rec[CMPC_REC_V + 2] - ax11) - fs[2];
  f_ext[0] = -e6;
  f_ext[1] = -e7;
  f_ext[2] = e8;
  f_ext[3] = e9;
  f_ext[4] = e10;
  f_ext[5] = e11;
}

__global__ __launch_bounds__(NT) void cmpc_estimate_kernel(
    float* __restrict__ est, const float* __restrict__ logs, const float* __restrict__ fext3,
    const float* __restrict__ times, float sim_time, float* __restrict__ recs, int rec_words,
    float* __restrict__ fext6, const float* __restrict__ gauss, int batch, float* __restrict__ fest_out) {
  __shared__ SharedE sh;
  const int inst = blockIdx.x;
  if (inst >= batch) return;
  const int tid = threadIdx.x;
  float* st = est + (size_t)inst * CMPC_EST_WORDS;
  float* rec = recs + (size_t)inst * rec_words;
  int32_t* sti = reinterpret_cast<int32_t*>(st);
  if (tid == 0) {
    float f3;
    if (logs) {
      float fe[6];
      residual(logs + (size_t)inst * CMPC_LOG_WORDS, rec, fe);
      f3 = fe[3];
      if (fext6) {
#pragma unroll
        for (int i = 0; i < 6; i++) fext6[(size_t)inst * 6 + i] = fe[i];
      }
    } else {
      f3 = fext3[inst];
    }
    const float t = times ? times[inst] : sim_time;
    int count = sti[CMPC_EST_COUNT];
    int head = sti[CMPC_EST_HEAD];
    st[CMPC_EST_F + head] = f3;  // diff_history.push_back(f_ext(3))
    st[CMPC_EST_T + head] = t;   // time_history.push_back(simulation_time)
    head = (head + 1) % W;
    if (count < (1 << 30)) count++;
    sti[CMPC_EST_COUNT] = count;
    sti[CMPC_EST_HEAD] = head;
    sh.count = count;
    sh.head = head;
    sh.t_now = t;
  }
  __syncthreads();
  const int count = sh.count;
  double* prm = reinterpret_cast<double*>(st + CMPC_EST_PARAMS);  // stat, amp, freq, phase
  if (count >= W && count <= CMPC_EST_STOP) {
    const int head = sh.head;
    for (int i = tid; i < W; i += NT) sh.fir.d[dslot(i)] = (double)st[CMPC_EST_F + (head + i) % W];
    for (int i = tid; i < NTAPS7; i += NT) sh.fir.k7[i] = (double)gauss[i];  // float taps, exact
    for (int i = tid; i < NTAPS27; i += NT) sh.fir.k27[i] = (double)gauss[NTAPS7 + i];
    if (tid < QW) {
      double sn, cs;
      sincospi(2.0 * tid / W, &sn, &cs);
      sh.tw[tid] = make_double2(cs, -sn);
    }
    if (tid == 0) {
      sh.t0 = st[CMPC_EST_T + head];
      sh.t1 = st[CMPC_EST_T + (head + 1) % W];
    }
    __syncthreads();
    // band-pass: gaussian_filter(7) - gaussian_filter(27)
    if (tid < NFIR) {
      const int i0 = NOUT * tid;
      double a7[NOUT] = {0.0, 0.0, 0.0, 0.0}, a27[NOUT] = {0.0, 0.0, 0.0, 0.0};
      fir4<kGaussR7>(sh.fir.d, sh.fir.k7, i0, a7);
      fir4<kGaussR27>(sh.fir.d, sh.fir.k27, i0, a27);
#pragma unroll
      for (int r = 0; r < NOUT; r++) sh.band[bslot(i0 + r)] = a7[r] - a27[r];
    }
    __syncthreads();
    // mean and standard deviation of the band (fit_sin's amplitude and offset guesses)
    double part = 0.0;
    for (int i = tid; i < W; i += NT) part += sh.band[bslot(i)];
    const double mean = block_sum_d(part, sh) / W;
    part = 0.0;
    for (int i = tid; i < W; i += NT) part += (sh.band[bslot(i)] - mean) * (sh.band[bslot(i)] - mean);
    const double sd = sqrt(block_sum_d(part, sh) / W);
    double v = __builtin_huge_val();
    int bi = 0x7fffffff;
    // |DFT|^2 of bins tid+1 and tid+101 from a 400-point FFT of the band (4 stages, a barrier
    // each; the reference's rfft, SolverMPC.cpp:503, agrees to ~1e-13 relative on the magnitudes)
    fft_stage<4, 1, true, 0, 1>(nullptr, sh.band, sh.fa, sh.tw, tid);
    __syncthreads();
    fft_stage<4, 4, false, 1, 2>(sh.fa, nullptr, sh.fb, sh.tw, tid);
    __syncthreads();
    fft_stage<5, 16, false, 2, 1>(sh.fb, nullptr, sh.fa, sh.tw, tid);
    __syncthreads();
    fft_stage<5, 80, false, 1, 2>(sh.fa, nullptr, sh.fb, sh.tw, tid);
    __syncthreads();
    if (tid < NBIN / 2) {
      const int ka = tid + 1, kb = tid + 1 + NBIN / 2;
      const double2 xa = sh.fb[fslot<2>(ka)], xb = sh.fb[fslot<2>(kb)];
      const double ma = xa.x * xa.x + xa.y * xa.y;
      const double mb = xb.x * xb.x + xb.y * xb.y;
      if (mb > ma) { v = -mb; bi = kb; } else { v = -ma; bi = ka; }
    }
    // first maximum: reduce on (-|X|^2, k)
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const double ov = __shfl_xor(v, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (ov < v || (ov == v && oi < bi)) { v = ov; bi = oi; }
    }
    const int wv = tid >> 6;
    if ((tid & 63) == 0) { sh.redd[wv] = v; sh.redi[wv] = bi; }
    __syncthreads();
    if (tid == 0) {
      double bv = sh.redd[0];
      int bk = sh.redi[0];
      for (int w = 1; w < NWV; w++)
        if (sh.redd[w] < bv || (sh.redd[w] == bv && sh.redi[w] < bk)) { bv = sh.redd[w]; bk = sh.redi[w]; }
      const double dt = (double)sh.t1 - (double)sh.t0;
      const double guess_freq = fabs(bk / (W * dt));  // fftfreq(n, dt)[k], k <= n/2
      const double omega = 2 * M_PI * guess_freq;
      prm[0] = mean;               // est_stat = offset
      prm[1] = sd * sqrt(2.0);     // est_amp
      prm[2] = omega / (2 * M_PI); // est_freq
      prm[3] = 0.0;                // est_phase
    }
    __syncthreads();
  }
  if (tid == 0) {
    float f_est3 = st[CMPC_EST_FEST3];
    if (count >= W) {
      f_est3 = (float)(prm[1] + sin(2 * M_PI * (double)sh.t_now * prm[2] + prm[3]));
      st[CMPC_EST_FEST3] = f_est3;
    }
    rec[CMPC_REC_FEST3] = f_est3;
    reinterpret_cast<uint32_t*>(rec)[CMPC_REC_FLAGS] = (count > CMPC_EST_STOP) ? 1u : 0u;
    if (fest_out) fest_out[inst] = f_est3;
  }
}

}  // namespace

hipError_t launch_estimate(float* d_est, const float* d_logs, const float* d_fext3,
                           const float* d_time, float sim_time, float* d_records, int rec_words,
                           float* d_fext6, const float* d_gauss, int batch, hipStream_t stream,
                           float* d_fest_out) {
  if (batch <= 0) return hipSuccess;
  hipLaunchKernelGGL(cmpc_estimate_kernel, dim3(batch), dim3(NT), 0, stream, d_est, d_logs, d_fext3,
                     d_time, sim_time, d_records, rec_words, d_fext6, d_gauss, batch, d_fest_out);
  return hipGetLastError();
}

}  // namespace cmpc
