// cmpc_multi.cpp — libcmpc_multi.so: the config-4 sharding as a C ABI over the
// batched solver (cmpc_solver.h) and RCCL, declared in include/cmpc_multi.h.
//
// One solve, for G participants (participant 0 is the root, which holds records and forces):
//   1. every peer's contiguous block of records goes root -> peer (ncclSend / ncclRecv, one group
//      over all communicators, on the per-communicator transfer streams);
//   2. every participant solves its block with its own cmpc_batch handle: the root in place, on
//      its solve stream, concurrently with the transfers (it moves nothing, so it takes
//      root_share times a peer's rows);
//   3. every peer's forces and status bytes go peer -> root, straight into the root's arrays.
// The caller's stream waits for the root's solve and the root's receives; nothing blocks the
// host. The plan is parallel.RootPipeline's with one piece per rank (auto_chunks gives one piece
// from 4 ranks at 262144 instances).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/cmpc_multi.h"

namespace {
thread_local std::string g_err;

int fail(const std::string& what) {
  g_err = what;
  return -1;
}
#define HIPCHK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) return fail(std::string(#x) + ": " + hipGetErrorString(e_));            \
  } while (0)
#define NCCLCHK(x)                                                                                 \
  do {                                                                                             \
    ncclResult_t r_ = (x);                                                                         \
    if (r_ != ncclSuccess) return fail(std::string(#x) + ": " + ncclGetErrorString(r_));          \
  } while (0)

// what one xGMI link (153 GB/s per direction) carries in the marginal solve time of one instance
// at N = 10 (21 ns on one MI355X between 59192 and 84568 instances, profiles/r05_final bench line)
constexpr double kRootEquivBytes = 3213.0;
}  // namespace

struct cmpc_multi {
  struct Part {
    int dev = 0;
    int comm = 0;                  // index into comms (the communicator's rank)
    cmpc_batch* h = nullptr;
    hipStream_t solve = nullptr;   // the handle's stream
    hipEvent_t ev_solved = nullptr, ev_recvd = nullptr;
    float* d_recs = nullptr;       // peers: their block of records / forces / status
    float* d_forces = nullptr;
    uint8_t* d_status = nullptr;
  };
  cmpc_params prm{};
  int G = 1;
  int max_batch = 0;
  int rec_words = 0;
  int out_cols = 0;
  float root_share = 1.f;
  bool loopback = false;
  std::vector<Part> parts;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> xfer;   // one transfer stream per communicator
  std::vector<hipEvent_t> ev_xfer; // recorded on xfer[c] after a transfer group
  hipEvent_t ev_in = nullptr;      // the caller's inputs are ready (root stream)
};

extern "C" float cmpc_multi_root_share(int record_bytes, int out_bytes, int pieces) {
  return 1.f + (float)((record_bytes + out_bytes) / (std::max(1, pieces) * kRootEquivBytes));
}

extern "C" const char* cmpc_multi_last_error(void) { return g_err.c_str(); }

extern "C" int cmpc_multi_rows(const cmpc_multi* m, int batch, int* rows) {
  if (!m || !rows || batch < 0) return fail("cmpc_multi_rows: bad arguments");
  const int G = m->G;
  if (G == 1 || m->root_share == 1.f) {  // contiguous, sizes differ by at most one
    for (int g = 0; g < G; g++) rows[g] = batch / G + (g < batch % G ? 1 : 0);
    return 0;
  }
  // the root about root_share times a peer's rows (parallel.rank_sizes)
  const int peer = (int)std::floor(batch / (G - 1 + (double)m->root_share));
  for (int g = 1; g < G; g++) rows[g] = peer;
  rows[0] = batch - peer * (G - 1);
  return 0;
}

extern "C" void cmpc_multi_destroy(cmpc_multi* m) {
  if (!m) return;
  for (auto& p : m->parts) {
    if (p.dev >= 0) (void)hipSetDevice(p.dev);
    if (p.h) {
      (void)hipStreamSynchronize(p.solve);
      cmpc_batch_destroy(p.h);
    }
    if (p.ev_solved) (void)hipEventDestroy(p.ev_solved);
    if (p.ev_recvd) (void)hipEventDestroy(p.ev_recvd);
    if (p.d_recs) (void)hipFree(p.d_recs);
    if (p.d_forces) (void)hipFree(p.d_forces);
    if (p.d_status) (void)hipFree(p.d_status);
  }
  for (size_t c = 0; c < m->comms.size(); c++) {
    (void)hipSetDevice(m->parts[c].dev);
    if (m->xfer[c]) {
      (void)hipStreamSynchronize(m->xfer[c]);
      (void)hipStreamDestroy(m->xfer[c]);
    }
    if (m->ev_xfer[c]) (void)hipEventDestroy(m->ev_xfer[c]);
    if (m->comms[c]) (void)ncclCommDestroy(m->comms[c]);
  }
  if (m->ev_in) {
    (void)hipSetDevice(m->parts[0].dev);
    (void)hipEventDestroy(m->ev_in);
  }
  delete m;
}

namespace {
int create_impl(cmpc_multi* m, const cmpc_params* prm, int ngpus, const int* devices, int max_batch,
                float root_share, int out_steps, int flags) {
  m->prm = *prm;
  m->G = ngpus;
  m->max_batch = max_batch;
  m->loopback = (flags & CMPC_MULTI_LOOPBACK) != 0;
  if (m->loopback && ngpus != 2) return fail("cmpc_multi_create: loopback needs ngpus == 2");
  m->rec_words = cmpc_record_words(prm->horizon);
  const int steps = (out_steps > 0 && out_steps < prm->horizon) ? out_steps : prm->horizon;
  m->out_cols = 12 * steps;
  m->root_share = (ngpus == 1) ? 1.f
                  : (root_share > 0.f ? root_share
                                      : cmpc_multi_root_share(4 * m->rec_words, 4 * m->out_cols + 1, 1));
  // communicators: one per distinct device (loopback: one, the root talks to itself)
  const int ncomm = m->loopback ? 1 : ngpus;
  m->parts.resize(ngpus);
  for (int g = 0; g < ngpus; g++) {
    m->parts[g].dev = m->loopback ? devices[0] : devices[g];
    m->parts[g].comm = m->loopback ? 0 : g;
  }
  m->comms.assign(ncomm, nullptr);
  m->xfer.assign(ncomm, nullptr);
  m->ev_xfer.assign(ncomm, nullptr);
  if (ngpus > 1) {
    std::vector<int> devs(ncomm);
    for (int c = 0; c < ncomm; c++) devs[c] = m->parts[c].dev;
    NCCLCHK(ncclCommInitAll(m->comms.data(), ncomm, devs.data()));
    for (int c = 0; c < ncomm; c++) {
      HIPCHK(hipSetDevice(devs[c]));
      HIPCHK(hipStreamCreateWithFlags(&m->xfer[c], hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&m->ev_xfer[c], hipEventDisableTiming));
    }
  }
  std::vector<int> rows(ngpus);
  cmpc_multi_rows(m, max_batch, rows.data());
  for (int g = 0; g < ngpus; g++) {
    auto& p = m->parts[g];
    HIPCHK(hipSetDevice(p.dev));
    // the root's block can be a little larger than rows[0] of max_batch for smaller batches
    // (rounding): size every handle for the largest block of any batch up to max_batch
    const int cap = std::max(1, g == 0 ? rows[0] + ngpus : rows[g] + 1);
    if (cmpc_batch_create(&p.h, prm, cap, nullptr) != 0)
      return fail(std::string("cmpc_batch_create: ") + cmpc_last_error());
    if (out_steps > 0 && cmpc_batch_set_output_steps(p.h, out_steps) != 0)
      return fail("cmpc_batch_set_output_steps failed");
    p.solve = (hipStream_t)cmpc_batch_stream(p.h);
    HIPCHK(hipEventCreateWithFlags(&p.ev_solved, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&p.ev_recvd, hipEventDisableTiming));
    if (g > 0) {
      HIPCHK(hipMalloc(&p.d_recs, sizeof(float) * (size_t)cap * m->rec_words));
      HIPCHK(hipMalloc(&p.d_forces, sizeof(float) * (size_t)cap * m->out_cols));
      HIPCHK(hipMalloc(&p.d_status, (size_t)cap));
    }
  }
  HIPCHK(hipSetDevice(m->parts[0].dev));
  HIPCHK(hipEventCreateWithFlags(&m->ev_in, hipEventDisableTiming));
  return 0;
}
}  // namespace

extern "C" int cmpc_multi_create(cmpc_multi** out, const cmpc_params* prm, int ngpus, const int* devices,
                                 int max_batch, float root_share, int out_steps, int flags) {
  if (!out || !prm || !devices || ngpus < 1 || max_batch < 1) return fail("cmpc_multi_create: bad arguments");
  if (prm->horizon < 1 || prm->horizon > CMPC_MAX_HORIZON) return fail("cmpc_multi_create: horizon out of range");
  *out = nullptr;
  auto* m = new cmpc_multi();
  const int rc = create_impl(m, prm, ngpus, devices, max_batch, root_share, out_steps, flags);
  if (rc != 0) {
    const std::string e = g_err;
    cmpc_multi_destroy(m);
    g_err = e;
    return rc;
  }
  *out = m;
  return 0;
}

extern "C" int cmpc_multi_solve(cmpc_multi* m, const float* d_records, int batch, float* d_forces,
                                uint8_t* d_status, void* root_stream) {
  if (!m || batch < 0 || batch > m->max_batch || (batch > 0 && (!d_records || !d_forces || !d_status)))
    return fail("cmpc_multi_solve: bad arguments");
  const int G = m->G;
  std::vector<int> rows(G), off(G);
  cmpc_multi_rows(m, batch, rows.data());
  for (int g = 0, a = 0; g < G; a += rows[g], g++) off[g] = a;
  auto& root = m->parts[0];
  hipStream_t rs = (hipStream_t)root_stream;
  HIPCHK(hipSetDevice(root.dev));
  HIPCHK(hipEventRecord(m->ev_in, rs));
  HIPCHK(hipStreamWaitEvent(root.solve, m->ev_in, 0));
  const size_t W = (size_t)m->rec_words, C = (size_t)m->out_cols;
  if (G > 1) {
    HIPCHK(hipStreamWaitEvent(m->xfer[root.comm], m->ev_in, 0));
    // 1. records root -> peers
    NCCLCHK(ncclGroupStart());
    for (int g = 1; g < G; g++) {
      if (rows[g] == 0) continue;
      const auto& p = m->parts[g];
      NCCLCHK(ncclSend(d_records + off[g] * W, rows[g] * W, ncclFloat32, p.comm, m->comms[root.comm],
                       m->xfer[root.comm]));
      NCCLCHK(ncclRecv(p.d_recs, rows[g] * W, ncclFloat32, root.comm, m->comms[p.comm], m->xfer[p.comm]));
    }
    NCCLCHK(ncclGroupEnd());
    // 2. every peer solves its block once its records are in
    for (int g = 1; g < G; g++) {
      auto& p = m->parts[g];
      if (rows[g] == 0) continue;
      HIPCHK(hipSetDevice(p.dev));
      HIPCHK(hipEventRecord(p.ev_recvd, m->xfer[p.comm]));
      HIPCHK(hipStreamWaitEvent(p.solve, p.ev_recvd, 0));
      if (cmpc_batch_solve(p.h, p.d_recs, rows[g], p.d_forces, p.d_status, nullptr) != 0)
        return fail(std::string("peer solve: ") + cmpc_last_error());
      HIPCHK(hipEventRecord(p.ev_solved, p.solve));
      HIPCHK(hipStreamWaitEvent(m->xfer[p.comm], p.ev_solved, 0));
    }
    HIPCHK(hipSetDevice(root.dev));
  }
  // the root's own block, where it lies, beside the transfers
  if (rows[0] > 0 && cmpc_batch_solve(root.h, d_records, rows[0], d_forces, d_status, nullptr) != 0)
    return fail(std::string("root solve: ") + cmpc_last_error());
  HIPCHK(hipEventRecord(root.ev_solved, root.solve));
  HIPCHK(hipStreamWaitEvent(rs, root.ev_solved, 0));
  if (G > 1) {
    // 3. forces and status peers -> root, into the root's rows
    NCCLCHK(ncclGroupStart());
    for (int g = 1; g < G; g++) {
      if (rows[g] == 0) continue;
      const auto& p = m->parts[g];
      NCCLCHK(ncclSend(p.d_forces, rows[g] * C, ncclFloat32, root.comm, m->comms[p.comm], m->xfer[p.comm]));
      NCCLCHK(ncclSend(p.d_status, rows[g], ncclUint8, root.comm, m->comms[p.comm], m->xfer[p.comm]));
      NCCLCHK(ncclRecv(d_forces + off[g] * C, rows[g] * C, ncclFloat32, p.comm, m->comms[root.comm],
                       m->xfer[root.comm]));
      NCCLCHK(ncclRecv(d_status + off[g], rows[g], ncclUint8, p.comm, m->comms[root.comm],
                       m->xfer[root.comm]));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipSetDevice(root.dev));
    HIPCHK(hipEventRecord(m->ev_xfer[root.comm], m->xfer[root.comm]));
    HIPCHK(hipStreamWaitEvent(rs, m->ev_xfer[root.comm], 0));
  }
  return 0;
}
