/*
 * cmpc_multi.h — multi-GPU sharding of a batched solve from C / C++ (libcmpc_multi.so).
 *
 * SURVEY.md §8(e) / BASELINE config 4: the records of the whole batch live on a root GPU; one
 * solve sends every other GPU its contiguous block of records over RCCL point-to-point transfers
 * (xGMI between the GPUs of a node), solves every block on its own GPU with the batched solver of
 * cmpc_solver.h, and receives the forces and status bytes back into the root's arrays. The root
 * solves its own, larger block where it lies while the transfers run (the same plan as the
 * Python path, quad-periodic-mpc_amd/parallel.py RootPipeline, for a caller without Python or
 * torch: the reference's callers are C++, ConvexMPCLocomotion.cpp:807-836).
 *
 * One process, one thread: the communicators come from ncclCommInitAll over the devices and every
 * transfer batch is one ncclGroupStart / ncclGroupEnd over all of them. The reference has no
 * multi-GPU path; this is a new API beside the batched one.
 *
 * No torch types cross this boundary: plain pointers and sizes only. Link: -lcmpc_multi
 * -lcmpc_hip -lrccl.
 */
#ifndef CMPC_MULTI_H
#define CMPC_MULTI_H

#include "cmpc_solver.h"

typedef struct cmpc_multi cmpc_multi;

/* ngpus devices, devices[0] the root (records and forces live there). root_share: the root's
 * rows over a peer's (it moves nothing, so it takes more); <= 0 picks cmpc_multi_root_share().
 * max_batch: the largest batch a solve will be given. out_steps as cmpc_batch_set_output_steps
 * (0 = every step). With CMPC_MULTI_LOOPBACK in flags and ngpus == 2, both "GPUs" are
 * devices[0] and the root's peer transfers go to itself over one communicator (a one-GPU test of
 * the whole transfer path). Returns 0 or a negative error (cmpc_multi_last_error()). */
#define CMPC_MULTI_LOOPBACK 1
CMPC_EXTERNC int cmpc_multi_create(cmpc_multi** out, const cmpc_params* prm, int ngpus,
                                   const int* devices, int max_batch, float root_share,
                                   int out_steps, int flags);
CMPC_EXTERNC void cmpc_multi_destroy(cmpc_multi* m);
/* d_records [batch * cmpc_record_words(N)] on the root device; d_forces [batch * out_cols] and
 * d_status [batch] on the root device, in instance order. Asynchronous on root_stream
 * (hipStream_t; NULL = the legacy default stream of the root device): the inputs are read after
 * the work already queued on it, and work queued on it afterwards sees the results. */
CMPC_EXTERNC int cmpc_multi_solve(cmpc_multi* m, const float* d_records, int batch, float* d_forces,
                                  uint8_t* d_status, void* root_stream);
/* Rows of each GPU for a batch (rows[ngpus]; the root first, contiguous blocks in order). */
CMPC_EXTERNC int cmpc_multi_rows(const cmpc_multi* m, int batch, int* rows);
/* The automatic root share: 1 + (bytes moved per instance) / (pieces x 3213 B), 3213 B being
 * what one xGMI link (153 GB/s per direction) carries in the marginal solve time of one instance
 * at N = 10 (21 ns, MI355X). bytes = record + forces (+ status). */
CMPC_EXTERNC float cmpc_multi_root_share(int record_bytes, int out_bytes, int pieces);
/* Last error of this library on this thread (diagnostics). */
CMPC_EXTERNC const char* cmpc_multi_last_error(void);

#endif /* CMPC_MULTI_H */
