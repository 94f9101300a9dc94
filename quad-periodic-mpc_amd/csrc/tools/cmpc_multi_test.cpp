// cmpc_multi_test — a plain C++ caller of include/cmpc_multi.h (no Python, no torch): reads
// records from a file, solves them through cmpc_batch_solve (one handle) and through
// cmpc_multi_solve (world 1, and the loopback world 2 that sends a peer's block to the root
// itself over RCCL), and prints one JSON line: whether every multi solve equals the single-handle
// solve bit for bit, and ms per solve of each.
//   cmpc_multi_test <records.f32> <batch> <horizon> [reps]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/cmpc_multi.h"

#define CHK(x)                                                                                  \
  do {                                                                                          \
    if ((x) != 0) {                                                                             \
      std::fprintf(stderr, "%s failed: %s | %s\n", #x, cmpc_multi_last_error(), cmpc_last_error()); \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)
#define HCHK(x)                                                                                 \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                              \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s records.f32 batch horizon [reps]\n", argv[0]);
    return 2;
  }
  const int B = std::atoi(argv[2]), N = std::atoi(argv[3]);
  const int reps = argc > 4 ? std::atoi(argv[4]) : 10;
  const int W = cmpc_record_words(N);
  std::vector<float> recs((size_t)B * W);
  FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(recs.data(), sizeof(float), recs.size(), f) != recs.size()) {
    std::fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  std::fclose(f);
  cmpc_params prm{};
  prm.dt = 0.026f;
  prm.mu = 0.4f;
  prm.f_max = 120.f;
  prm.horizon = N;
  const float w[12] = {0.25f, 0.25f, 10.f, 10.f, 2.f, 50.f, 0.f, 0.f, 0.3f, 0.2f, 0.2f, 0.1f};
  std::memcpy(prm.weights, w, sizeof w);
  prm.alpha = 4e-5f;
  prm.max_iter = 100;
  HCHK(hipSetDevice(0));
  float *d_recs, *d_f0, *d_f;
  uint8_t *d_s0, *d_s;
  const size_t FC = (size_t)B * 12 * N;
  HCHK(hipMalloc(&d_recs, sizeof(float) * recs.size()));
  HCHK(hipMalloc(&d_f0, sizeof(float) * FC));
  HCHK(hipMalloc(&d_f, sizeof(float) * FC));
  HCHK(hipMalloc(&d_s0, B));
  HCHK(hipMalloc(&d_s, B));
  HCHK(hipMemcpy(d_recs, recs.data(), sizeof(float) * recs.size(), hipMemcpyHostToDevice));
  hipStream_t st;
  HCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  // reference: one handle
  cmpc_batch* h = nullptr;
  CHK(cmpc_batch_create(&h, &prm, B, st));
  CHK(cmpc_batch_solve(h, d_recs, B, d_f0, d_s0, nullptr));
  HCHK(hipStreamSynchronize(st));
  std::vector<float> f0(FC), f1(FC);
  std::vector<uint8_t> s0(B), s1(B);
  HCHK(hipMemcpy(f0.data(), d_f0, sizeof(float) * FC, hipMemcpyDeviceToHost));
  HCHK(hipMemcpy(s0.data(), d_s0, B, hipMemcpyDeviceToHost));
  auto timed = [&](auto&& fn) {
    fn();
    (void)hipStreamSynchronize(st);
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; r++) fn();
    (void)hipStreamSynchronize(st);
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
  };
  const double ms_single = timed([&] { cmpc_batch_solve(h, d_recs, B, d_f0, d_s0, nullptr); });
  cmpc_batch_destroy(h);
  int n_ok = 0, n_cases = 0;
  // the JSON line is assembled here and printed once at the end (RCCL prints its banner to stdout
  // when the first communicator is created)
  std::string js;
  char buf[512];
  std::snprintf(buf, sizeof buf, "{\"batch\": %d, \"horizon\": %d, \"ms_single_handle\": %.4f, \"cases\": [", B,
                N, ms_single);
  js += buf;
  const int dev0 = 0;
  const int devs[2] = {0, 0};
  struct Case {
    int G, flags;
    float share;
  } cases[] = {{1, 0, 0.f}, {2, CMPC_MULTI_LOOPBACK, 0.f}, {2, CMPC_MULTI_LOOPBACK, 1.f},
               {2, CMPC_MULTI_LOOPBACK, 3.5f}};
  for (const Case& c : cases) {
    cmpc_multi* m = nullptr;
    CHK(cmpc_multi_create(&m, &prm, c.G, c.G == 1 ? &dev0 : devs, B, c.share, 0, c.flags));
    HCHK(hipMemsetAsync(d_f, 0xff, sizeof(float) * FC, st));
    HCHK(hipMemsetAsync(d_s, 0xff, B, st));
    CHK(cmpc_multi_solve(m, d_recs, B, d_f, d_s, st));
    HCHK(hipStreamSynchronize(st));
    HCHK(hipMemcpy(f1.data(), d_f, sizeof(float) * FC, hipMemcpyDeviceToHost));
    HCHK(hipMemcpy(s1.data(), d_s, B, hipMemcpyDeviceToHost));
    const bool eq = std::memcmp(f0.data(), f1.data(), sizeof(float) * FC) == 0 &&
                    std::memcmp(s0.data(), s1.data(), B) == 0;
    const double ms = timed([&] { cmpc_multi_solve(m, d_recs, B, d_f, d_s, st); });
    // the same again after the timed solves (buffers reused across solves)
    HCHK(hipMemcpy(f1.data(), d_f, sizeof(float) * FC, hipMemcpyDeviceToHost));
    const bool eq2 = std::memcmp(f0.data(), f1.data(), sizeof(float) * FC) == 0;
    int rows[2] = {0, 0};
    cmpc_multi_rows(m, B, rows);
    std::snprintf(buf, sizeof buf, "%s{\"gpus\": %d, \"loopback\": %d, \"rows\": [%d, %d], \"bitwise\": %s, \"ms\": %.4f}",
                  n_cases ? ", " : "", c.G, c.flags, rows[0], c.G > 1 ? rows[1] : 0,
                  (eq && eq2) ? "true" : "false", ms);
    js += buf;
    n_ok += (eq && eq2);
    n_cases++;
    cmpc_multi_destroy(m);
  }
  std::fflush(stdout);
  std::printf("\n%s], \"all_bitwise\": %s}\n", js.c_str(), n_ok == n_cases ? "true" : "false");
  return n_ok == n_cases ? 0 : 3;
}
