#!/usr/bin/env python3
"""Benchmark: QP solves/s of the fused HIP convex-MPC solver (BASELINE.json metric).

One "step" = one pass of the hot path (ConvexMPCLocomotion::solveDenseMPC -> solve_mpc:
condensation + friction-cone QP + force scatter) over one batch of synthetic instances whose
records are already resident in HBM when the timed region starts.

Workloads (BASELINE.json configs; the default follows the GPU count):
  --config 3   (default at 1 GPU) batch 65536 per GPU, N = 10, fused condensation + QP.
  --config 4   (default at >1 GPU) batch 262144 in total, N = 10, strong-scaled over the
               ranks: the records live on rank 0's GPU, every step scatters them over RCCL
               (xGMI), solves each rank's contiguous shard and gathers the forces back to rank 0,
               software-pipelined over --chunks pieces (parallel.RootPipeline).
  --config 2   batch 4096 per GPU, N = 10.
  --config 5   batch 65536 per GPU, N = 20, one periodic-disturbance estimator step (LogData
               residual, Gaussian band-pass, DFT sine fit) fused ahead of every solve.
Instances come from the per-instance Philox generator (seed 0x5EED0000 + id), so any shard of
ids holds exactly the instances a 1-GPU run of the same global batch holds.

  python bench.py [--gpus N --steps K --warmup W] [--config C] [--batch B | --global-batch G]
  python bench.py --gpus 2 --dry-run     # CPU/gloo plumbing check of the config-4 path

With --gpus N > 1 and no torchrun environment the script relaunches itself under
torch.distributed.run (one process per GPU) before touching any GPU. Rank 0 prints ONE JSON
line.
"""
from __future__ import annotations

import argparse
import hashlib
import importlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "QP solves/sec (N=10, 13-state, 12-force) at batch=65536; 1/2/4/8 GPU"
METRIC_C2 = "QP solves/sec (N=10) at batch=4096, 1 GPU (config 2)"
METRIC_C5 = "QP solves/sec (N=20 + disturbance estimation, config 5) at batch=65536"
METRIC_N16 = "QP solves/sec (N=16 trot, the deployed horizon) at batch=65536"
FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (v_fma_f32 at 2 cyc/wave on SIMD-32)
HBM_PEAK_GBS = 8000.0
XGMI_LINK_GBS = 153.0      # one xGMI link, one direction (7 links per MI355X: SURVEY.md §5)


def algorithmic_flops(N: int) -> float:
    """F(N) = F_cond + F_chol (dense, reference algorithm)."""
    n = 12 * N
    f_cond = 4056 * (N - 1) + 338 * N + 3900 * N * (N + 1) * (N + 2) / 6 + 312 * N * (N + 1) / 2
    f_chol = n ** 3 / 3 + 2 * n ** 2
    return f_cond + f_chol


def algorithmic_bytes(N: int, config5: bool = False) -> int:
    """compulsory HBM bytes per QP (fp32 record in, forces out); config 5
    adds f_est (24 B), the 400-sample history window (1600 B) and the appended sample (4 B)."""
    b = 64 + 48 + 48 * N + 4 * N + 4 + 48 * N
    return b + (24 + 1600 + 4 if config5 else 0)


CPU_THREAD_CAP = 16   # the GPU box's CPU share per GPU (its nproc shows the whole machine)


def _host_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _threads():
    return max(1, min(CPU_THREAD_CAP, _host_cpus()))


def cpu_baseline(prm, N: int, config5: bool = False):
    """The reference pipeline on the host cores (rank 0, N=1 only), bounded sample: the fp32
    dense-S condensation restated from SolverMPC.cpp (oracle/cmpc_oracle.c) with its dense
    products register-tiled the way Eigen's GEMM kernels run them (impl 1: bit for bit the naive
    restatement's result, tests/test_oracle.py) + the reference's own qpOASES 3.2.0 compiled from
    its sources (oracle/_ref); at config 5 each instance also runs the residual + estimator step
    first (SolverMPC.cpp:688-811, restated in C). Throughput at the GPU's CPU share (16 threads)
    and at every visible CPU; latency of one call on one core."""
    try:
        from oracle import oracle as orc
    except Exception:
        return None
    if not orc.ref_available():
        return None
    cm = importlib.import_module("quad-periodic-mpc_amd")
    threads = _threads()
    visible = _host_cpus()
    sample = 2048 if N >= 16 else 8192
    recs = cm.make_instances(sample, N)
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    if config5:
        est, logs = _config5_state(cm, R, recs, sample)

    def run(nthreads, k=sample, impl=1):
        r = recs[:k].copy()
        if config5:
            e = est[:k].copy()
            t0 = time.perf_counter()
            orc.ref_pipeline_c5_batch(r, logs[:k], e, prm, 10.4, nthreads=nthreads, impl=impl)
        else:
            t0 = time.perf_counter()
            orc.ref_solve_batch(r, prm, nthreads=nthreads, impl=impl)
        return time.perf_counter() - t0

    run(threads, 64)  # warm
    dt = run(threads)
    dt_all = run(visible) if visible > threads else None
    # per-call latency of the reference pipeline on one core (what one solveDenseMPC costs)
    nlat = 256
    lat_us = run(1, nlat) / nlat * 1e6
    lat_naive_us = run(1, nlat, impl=0) / nlat * 1e6
    what = ("residual + band-pass/DFT estimator step (SolverMPC.cpp:688-811, restated in C) then "
            if config5 else "")
    out = {"value": round(sample / dt, 1), "unit": "QP solves/s", "cores": threads,
           "host_cpus_visible": visible,
           "cores_note": (f"{threads} threads: the GPU box's CPU share per GPU; "
                          f"value_all_visible_cpus: the same sample on {visible} threads"),
           "value_all_visible_cpus": round(sample / dt_all, 1) if dt_all else None,
           "latency_us_1core": round(lat_us, 1),
           "latency_us_1core_naive_loops": round(lat_naive_us, 1),
           "condensation_note": ("the dense-S products of SolverMPC.cpp:806-814 (B_qp^T S, (B_qp^T "
                                 "S) B_qp, (2 B_qp^T) S and its product with the state error) as "
                                 "dense register-tiled fp32 GEMMs (6 x 16 tiles, 8-wide FMA; "
                                 "oracle/cmpc_oracle.c condense_blocked), the full dense work Eigen "
                                 "does, summed in the same order as the naive loops (bit-identical "
                                 "results); latency_us_1core_naive_loops times the naive loops"),
           "kind": "reference",
           "sample": f"{sample} instances of the same synthetic workload (N={N}), per instance "
                     f"{what}the solve_mpc equivalent: fp32 dense-S condensation "
                     f"(SolverMPC.cpp:566-950 restated, oracle/cmpc_oracle.c) + reference "
                     f"qpOASES 3.2.0 (setToMPC, nWSR=100) built from /root/reference; "
                     f"{threads} std::threads; {dt:.2f} s wall"}
    try:
        out["cpu_model"] = next(l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo")
                                if l.startswith("model name"))
    except Exception:
        pass
    return out


def _config5_state(cm, R, recs_np, B):
    """Estimator histories pre-filled to 400 samples (so every timed step re-estimates,
    SolverMPC.cpp:704-707) and the previous step's LogData records."""
    f3, tt = cm.make_disturbance(B, R.EST_WINDOW)
    est = np.zeros((B, R.EST_WORDS), np.float32)
    est[:, R.EST_F:R.EST_F + R.EST_WINDOW] = f3
    est[:, R.EST_T:R.EST_T + R.EST_WINDOW] = tt[None, :]
    est.view(np.int32)[:, R.EST_COUNT] = R.EST_WINDOW
    est.view(np.int32)[:, R.EST_HEAD] = 0
    logs = cm.make_logs(recs_np)
    return est, logs


def load_pmc(N: int, batch: int, kernel_prefix: str):
    """HBM bytes per launch of the dominant kernel + its SQ counters from the committed
    rocprofv3 PMC summary (profiles/pmc_summary.json, scripts/pmc_collect.py)."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_summary.json")) as f:
            d = json.load(f)
    except Exception:
        return None, None
    for case in d.get("cases", [d]):
        if case.get("horizon") != N or case.get("batch") != batch:
            continue
        kernels = case.get("kernels", {})
        if kernel_prefix == "whole solve":
            # every launch of one solve (classify + class 1 + each wide class) summed, the unit
            # `achieved` is quoted on when the wide classes carry the batch
            parts = {n: k for n, k in kernels.items()
                     if "solve" in n or "classify" in n}
            if parts and all(k.get("hbm_bytes_per_launch") is not None for k in parts.values()):
                total = sum(k["hbm_bytes_per_launch"] for k in parts.values())
                return total, dict(kernels=sorted(parts), hbm_bytes_per_launch=total)
            continue
        for name, k in kernels.items():
            if kernel_prefix in name:
                return k.get("hbm_bytes_per_launch"), k
    return None, None


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def relaunch_distributed(nproc: int) -> int:
    """One process per GPU under torch.distributed.run; called before any GPU work."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def abi_latency():
    """Batch-1 latency of the drop-in single-instance ABI (setup_problem -> update_x_drag ->
    update_solver_settings -> update_problem_data_floats -> get_solution(0..11)), measured by a
    plain C++ caller (quad-periodic-mpc_amd/cmpc_abi_latency) in a child process."""
    exe = os.path.join(ROOT, "quad-periodic-mpc_amd", "cmpc_abi_latency")
    if not os.path.exists(exe):
        return None
    res = {}
    for N in (10, 16):
        try:
            r = subprocess.run([exe, str(N), "1000"], capture_output=True, text=True, timeout=120)
            res[f"N{N}"] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception as e:  # diagnostics only
            res[f"N{N}"] = repr(e)
    return res


def digest(t) -> str:
    return hashlib.sha256(np.ascontiguousarray(t.cpu().numpy()).tobytes()).hexdigest()[:16]


def plumbing_solve(N):
    """--dry-run stand-in for the device solve (CPU ranks, no GPU): a per-instance,
    order-sensitive function of the record, so the gathered rows show whether every instance
    reached its rank and came back to its slot. Not a solver and never timed as one."""
    def fn(recs, forces, status):
        forces.copy_(recs[:, 32:32 + 12 * N] * 2.0 + recs[:, 0:1])
        status.zero_()
    return fn


def local_leg(args, cm, prm, config, N, B, steps, warmup, dev, rank, barrier, sync, dist,
              frac=None):
    """Configs 2 / 3 / 5 on this rank: inputs resident in HBM, ``warmup`` untimed steps, then
    ``steps`` timed ones bracketed by barrier + synchronize, max over ranks. -> dict."""
    import torch
    frac = args.random_contact_frac if frac is None else frac
    world = int(os.environ.get("WORLD_SIZE", "1"))
    recs_np = cm.make_instances(B, N, random_contact_frac=frac, first_id=rank * B)
    recs = torch.from_numpy(recs_np).to(dev)
    forces = torch.empty((B, 12 * N), dtype=torch.float32, device=dev)
    status = torch.empty(B, dtype=torch.uint8, device=dev)
    iters = torch.empty(B, dtype=torch.int32, device=dev)
    solver = None
    est = est0 = None
    if args.dry_run:
        fn = plumbing_solve(N)

        def step():
            fn(recs, forces, status)
    else:
        solver_mod = importlib.import_module("quad-periodic-mpc_amd.solver")
        solver = solver_mod.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream(dev))
        if args.no_refine:  # A/B only: the refinement off (cmpc_batch_set_refine(0)); noted in config
            solver.set_refine(False)

        def step():
            solver.solve(recs, forces, status, iters)

        if config == 5:
            R = importlib.import_module("quad-periodic-mpc_amd.records")
            est_np, logs_np = _config5_state(cm, R, recs_np, B)
            est0 = torch.from_numpy(est_np).to(dev)
            est = est0.clone()
            logs = torch.from_numpy(logs_np).to(dev)
            t_next = [10.4]

            def step():  # noqa: F811  (config 5: estimator step, then the solve)
                solver.estimate(est, recs, logs=logs, sim_time=t_next[0])
                t_next[0] += prm.dt
                solver.solve(recs, forces, status, iters)

    sync()
    for _ in range(warmup):
        step()
    if config == 5 and est is not None:  # restart the histories at 400 samples for the timed steps
        sync()
        est.copy_(est0)
        t_next[0] = 10.4
    sync()
    if solver is not None and os.environ.get("CMPC_BENCH_NO_EVENTS") != "1":  # diagnostic: events off
        # HIP events on every TIMING_EVERY-th solve of the timed loop: each recorded solve adds
        # event packets between its launches (on every solve they cost config 3 1.9 %, r04_ev3)
        solver.enable_timing((steps + TIMING_EVERY - 1) // TIMING_EVERY, every=TIMING_EVERY)
    # ---- timed region: K steps, bracketed by barrier + synchronize on both sides ----------
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return dict(elapsed=elapsed, solver=solver, forces=forces, status=status, iters=iters,
                recs=recs, recs_np=recs_np, world=world)


TIMING_EVERY = 4   # the solves of a timed loop that record the roofline's HIP events
WIDE_CLASS_NV = (80, 96, 120, 128, 144, 192, 256)   # row widths of the wide classes (cmpc_wide.h)


def carrying_wide_kernel(N: int) -> str:
    """Kernel name of the wide class that holds the trot size n = 6 N (every instance of the
    trot workloads, the mode of any contact mix): launched one workgroup per list entry
    (cmpc_launch.hip one_per_entry), hence the `false` (not persistent) template argument."""
    nv = next(v for v in WIDE_CLASS_NV if v >= 6 * N)
    # the refining builds (fp64 refinement of the active set) serve N > 10
    return f"cmpc_solve_w_kernel<{nv}, false, {'true' if N > 10 else 'false'}>"


def make_roofline(launch_ms, ovf, units_per_launch, N, value, config):
    """roofline object of the dominant launch (see the module docstring / DESIGN.md §5)."""
    if not launch_ms.size:
        return None
    fl = algorithmic_flops(N)
    c1 = launch_ms[:, 0]
    c2 = launch_ms[:, 1]
    units1 = units_per_launch - ovf
    t1 = float(np.mean(c1)) * 1e-3
    wide = units1 < units_per_launch // 2   # at N >= 16 the wide classes carry the batch
    if wide:
        # whole solve (class 1 + the concurrently running wide classes) as one launch
        t1 = float(np.mean(c1 + c2)) * 1e-3
        units1 = units_per_launch
    achieved = fl * units1 / t1 / 1e12 if t1 > 0 else None
    # class 1 runs as the 60-wide build once the batch fills the GPU (>= 16384 instances at
    # N >= 6, cmpc_launch.hip), else as the 64-wide build
    c1w = 60 if (units_per_launch >= 16384 or N <= 5) else 64
    wide_k = carrying_wide_kernel(N)
    traffic, pmc = load_pmc(N, units_per_launch, f"cmpc_solve_c1_kernel<{c1w}>" if not wide
                            else "whole solve")
    _, pmc_wide = load_pmc(N, units_per_launch, wide_k) if wide else (None, None)
    roofline = {
        "bound": "valu",
        "achieved": round(achieved, 3) if achieved else None,
        "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP32_PEAK_TFLOPS, 5) if achieved else None,
        "traffic": traffic,
        "kernel": (f"cmpc_solve_c1_kernel<{c1w}> (class 1, {c1w}-wide rows, one wavefront per instance)" if not wide
                   else "whole solve: every size class, concurrent streams"),
        "units_per_launch": int(units1),
        "flops_per_unit": fl,
        "avg_launch_ms": round(t1 * 1e3, 4),
        "launches_timed": int(launch_ms.shape[0]),
        "class1_avg_launch_ms": round(float(np.mean(c1)), 4),
        "tail_avg_ms": round(float(np.mean(c2)), 4),
        "wide_class_units": int(ovf),
        "hbm_bytes_per_unit": algorithmic_bytes(N, config == 5),
        "hbm_gbs": round(algorithmic_bytes(N, config == 5) * value / 1e9, 3),
        "note": "FP32 VALU roof (the path is latency/VALU-bound, not HBM: ~1300 FLOP/B). "
                "achieved = SURVEY §8(d) F(N) (dense reference algorithm) x instances of "
                "the launch / its HIP-event time on the solver stream (events on every "
                f"{TIMING_EVERY}th solve of the timed loop, `launches_timed` of them); the kernels execute "
                "fewer flops (reduced n, structured condensation), so frac is speed against "
                "the reference's work. valu_pmc: counters of the same kernel (profiles/"
                "pmc_summary.json); valu_issue_util = VALU instructions x 2 cycles (wave64 on "
                "SIMD-32) / (1024 SIMDs x 2.4 GHz x launch time)",
    }
    if wide:
        if pmc:
            roofline["traffic_kernels"] = pmc["kernels"]
        pmc = pmc_wide
    if pmc:
        vp = {k: pmc[k] for k in ("valu_insts_per_wave", "lds_insts_per_wave", "waves",
                                   "lds_bank_conflict_frac", "wait_frac", "issue_stall_frac",
                                   "active_frac", "scratch", "pmc_tag") if k in pmc}
        if "vgpr" in pmc:
            # rocprofv3's kernel-trace VGPR_Count: on this image it reads half the compiler's
            # allocation (80 for class 1's 158 -> 160 registers in round 2); relabelled, not
            # converted
            vp["vgpr_count_rocprof_field"] = pmc["vgpr"]
        if "valu_insts_per_wave" in pmc and "waves" in pmc and t1 > 0:
            vp["valu_issue_util"] = round(pmc["valu_insts_per_wave"] * pmc["waves"] * 2.0 /
                                          (1024 * 2.4e9 * t1), 4)
        roofline["valu_pmc"] = vp
    return roofline


def scaling_model(args, cm, dev, sync):
    """Config 4 at G = 1, 2, 4, 8 GPUs predicted from ONE GPU (a labelled model, not a
    measurement): every rank of a G-GPU run solves its block of the 262144 records cut into
    parallel.auto_chunks pieces, which a world-1 RootPipeline over that many records reproduces
    exactly (the compact records expanded on the GPU, then solved), so the per-rank times are
    measured here. Rank 0 sends each piece's compact records (224 B at N = 10) to G - 1 peers (one
    xGMI link each, concurrently) and receives their forces back; only the first send and the last
    receive are exposed, the rest overlaps the solve of the neighbouring pieces unless it is longer
    than that solve. Root solves its own, larger share (parallel.root_share_auto: 1 + bytes moved /
    (pieces x 3213 B)) without waiting for a transfer. t_G = max(t_root, t_peer + t_first_scatter +
    t_last_gather + max(0, comm of the inner pieces - t_peer)); speedup = t_1 / t_G."""
    import torch
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    N, G_total = 10, 262144
    prm = cm.make_params(N)
    words = R.compact_words(N)
    rec_b = 4 * words
    out_b = 4 * 12 * N
    full_np = cm.make_instances(G_total, N, random_contact_frac=args.random_contact_frac)
    recs_all = torch.from_numpy(R.compact_records(full_np, N, prm.dt)).to(dev)
    del full_np
    rows = []

    def timed_pieces(local, chunks, out_steps=0):
        pipe = par.RootPipeline(prm, local, chunks=chunks, device=dev, out_steps=out_steps,
                                record_format="compact")
        recs = recs_all[:local]
        for _ in range(3):
            pipe.step(recs)
        steps = 20
        sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            pipe.step(recs)
        sync()
        t = (time.perf_counter() - t0) / steps
        sizes = pipe.sizes
        pipe.close()
        return t, sizes

    def model_t(t_peer_solve, t_root_solve, pieces, out_bytes, bw):
        """The peers' path (first scatter, solve, last gather, exposed inner transfers) against
        root's own solve, which waits for no transfer (parallel.RootPipeline)."""
        sc = [p * rec_b / (bw * 1e9) for p in pieces]   # per-peer bytes of a piece / link
        ga = [p * out_bytes / (bw * 1e9) for p in pieces]
        inner = sum(sc[1:]) + sum(ga[:-1])
        t_peer = t_peer_solve + sc[0] + ga[-1] + max(0.0, inner - t_peer_solve)
        return max(t_peer, t_root_solve)

    def plan(G, cols):
        chunks = par.auto_chunks(max(par.shard_sizes(G_total, G)), G)
        share = par.root_share_auto(words, cols, chunks) if G > 1 else 1.0
        return chunks, share, par.rank_sizes(G_total, G, 0, share)

    t1 = t1s = None
    for G in (1, 2, 4, 8):
        chunks, share, sizes_r = plan(G, 12 * N)
        local, root_local = sizes_r[-1], sizes_r[0]
        t_solve, pieces = timed_pieces(local, chunks)
        row = {"gpus": G, "per_rank_instances": local, "pieces": len(pieces),
               "piece_instances": pieces[0], "t_solve_ms_measured": round(t_solve * 1e3, 4)}
        if G > 1:
            t_root, _ = timed_pieces(root_local, chunks)
            row.update(root_instances=root_local, root_share=round(share, 3),
                       t_root_solve_ms_measured=round(t_root * 1e3, 4))
        if G == 1:
            t1 = t_solve
            row.update(t_model_ms=round(t_solve * 1e3, 4), speedup=1.0)
        else:
            for bw, key in ((XGMI_LINK_GBS, ""), (50.0, "_at_50GBs")):
                t = model_t(t_solve, t_root, pieces, out_b, bw)
                row["t_model_ms" + key] = round(t * 1e3, 4)
                row["speedup" + key] = round(t1 / t, 3)
            row["xgmi_mb_root_sends"] = round((G_total - root_local) * rec_b / 1e6, 2)
            row["xgmi_mb_root_receives"] = round((G_total - root_local) * out_b / 1e6, 2)
        # the same with the step-0 forces only (cmpc_batch_set_output_steps(1): what a caller of
        # get_solution(0..11) reads, ConvexMPCLocomotion.cpp:832-845): 48 B gathered per instance
        chunks0, share0, sizes0 = plan(G, 12)
        t0s, pieces0 = timed_pieces(sizes0[-1], chunks0, out_steps=1)
        row["step0_t_solve_ms_measured"] = round(t0s * 1e3, 4)
        if G == 1:
            t1s = t0s
            row["step0_speedup"] = 1.0
        else:
            t0r, _ = timed_pieces(sizes0[0], chunks0, out_steps=1)
            row.update(step0_root_instances=sizes0[0], step0_t_root_solve_ms_measured=round(t0r * 1e3, 4))
            t = model_t(t0s, t0r, pieces0, 48, XGMI_LINK_GBS)
            row["step0_t_model_ms"] = round(t * 1e3, 4)
            row["step0_speedup"] = round(t1s / t, 3)
        rows.append(row)
    del recs_all
    return {"kind": "model (not a measurement): per-rank solve times measured on this GPU, "
                    f"xGMI at {XGMI_LINK_GBS:.0f} GB/s per link and direction (and a pessimistic "
                    "50 GB/s), comm overlap per parallel.RootPipeline, compact records "
                    f"({rec_b} B per instance) expanded on every rank",
            "global_batch": G_total, "horizon": N, "record_bytes_sent": rec_b, "rows": rows}


def other_configs(args, cm, dev, rank, barrier, sync, dist):
    """BASELINE configs 2 and 5, and the deployed horizon N = 16 (ros_config.yaml:93, trot), measured
    in the same (default, 1-GPU) run after config 3, with the same protocol: resident inputs,
    warmup, barrier + synchronize, HIP-event roofline."""
    out = {}
    legs = ((2, 10, 4096, 200, 20, None), ("n16_trot", 16, 65536, 20, 3, 0.0), (5, 20, 65536, 5, 2, None))
    for config, N, B, steps, warmup, frac in legs:
        prm = cm.make_params(N)
        leg = local_leg(args, cm, prm, config, N, B, steps, warmup, dev, rank, barrier, sync, dist,
                        frac=frac)
        launch_ms, ovf = leg["solver"].read_timing()
        value = B * steps / leg["elapsed"]
        st = np.bincount(leg["status"].cpu().numpy(), minlength=5)
        metric = {2: METRIC_C2, 5: METRIC_C5}.get(config, METRIC_N16)
        d = {"metric": metric, "value": round(value, 1),
             "unit": "QP solves/s", "ms_per_step": round(leg["elapsed"] / steps * 1e3, 4),
             "steps": steps, "warmup": warmup, "batch": B, "horizon": N,
             "roofline": make_roofline(launch_ms, ovf, B, N, value, config),
             "status_counts": {cm.STATUS_NAMES[i]: int(c) for i, c in enumerate(st) if c},
             "forces_digest": digest(leg["forces"])}
        if config == 5:
            d["workload"] = ("N=20, per step one batched periodic-disturbance estimator step "
                             "(LogData residual, Gaussian band-pass, DFT sine fit) fused ahead of "
                             "the solve, histories at 400..405 samples")
            if not args.no_cpu_baseline:
                d["cpu_baseline"] = cpu_baseline(prm, N, config5=True)
        elif config == 2:
            d["workload"] = "N=10, batch 4096 (same instance mix as config 3)"
            d["cpu_baseline"] = "same per-instance workload as config 3: see cpu_baseline"
        else:
            d["workload"] = ("N=16, batch 65536, A1 trot at random phase (every instance n = 96 "
                             "reduced variables): the reference's deployed operating point "
                             "(ros_config.yaml:93), not a BASELINE config")
        leg["solver"].close()
        out[f"config{config}" if isinstance(config, int) else config] = d
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, choices=(2, 3, 4, 5), default=None)
    ap.add_argument("--config5", action="store_true", help="alias of --config 5")
    ap.add_argument("--batch", type=int, default=None, help="instances per GPU (configs 2, 3, 5)")
    ap.add_argument("--global-batch", type=int, default=None, help="total instances (config 4)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="config-4 pipeline pieces per rank (default: parallel.auto_chunks)")
    ap.add_argument("--horizon", type=int, default=None)
    ap.add_argument("--random-contact-frac", type=float, default=0.25)
    ap.add_argument("--record-format", choices=("compact", "full"), default="compact",
                    help="config 4: the records root holds and sends (compact: trajAll's step-0 row, "
                         "expanded on every rank by cmpc_batch_expand)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip end-to-end / solve-only legs")
    ap.add_argument("--no-refine", action="store_true",
                    help="A/B only: the wide classes' fp64 refinement off (cmpc_batch_set_refine)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU ranks over gloo with a plumbing stand-in for the solve (no GPU)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args.gpus))

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    config = 5 if args.config5 else (args.config or (4 if world > 1 else 3))
    N = args.horizon or (20 if config == 5 else 10)

    dist = None
    if args.dry_run:
        dev = torch.device("cpu")
        if world > 1:
            import torch.distributed as tdist
            tdist.init_process_group("gloo")
            dist = tdist
    else:
        torch.cuda.set_device(local_rank)
        dev = torch.device("cuda", local_rank)
        # one non-default stream carries everything of this rank (copies, collectives' stream
        # joins, the solver's launches), so the library's launches order with torch's work
        torch.cuda.set_stream(torch.cuda.Stream(dev))
        if world > 1:
            import torch.distributed as tdist
            tdist.init_process_group("nccl", device_id=dev)
            dist = tdist

    cm = importlib.import_module("quad-periodic-mpc_amd")
    prm = cm.make_params(N)

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync():
        if not args.dry_run:
            torch.cuda.synchronize()

    extras = {}
    solver = None
    if config == 4:
        par = importlib.import_module("quad-periodic-mpc_amd.parallel")
        G = args.global_batch or 262144
        R = importlib.import_module("quad-periodic-mpc_amd.records")
        pipe = par.RootPipeline(prm, G, chunks=args.chunks, device=dev,
                                solve_fn=plumbing_solve(N) if args.dry_run else None,
                                record_format=args.record_format)
        recs_root = None
        if rank == 0:
            full_np = cm.make_instances(G, N, random_contact_frac=args.random_contact_frac)
            if args.record_format == "compact":   # trajAll's step-0 row, expanded on every rank
                full_np = R.compact_records(full_np, N, prm.dt)
            recs_root = torch.from_numpy(full_np).to(dev)
        B_total, B_local = G, pipe.local_batch

        def step():
            pipe.step(recs_root)

        sync()
        for _ in range(args.warmup):
            step()
        sync()
        timed = None if args.dry_run else pipe   # per-launch events on every lane's handle
        units_per_launch = max(pipe.sizes)
        if timed is not None:
            timed.enable_timing(args.steps * pipe.chunks)
        # ---- timed region: K steps, bracketed by barrier + synchronize on both sides ------
        barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        barrier()
        elapsed = time.perf_counter() - t0
        if dist is not None:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
    else:
        B = args.batch or (4096 if config == 2 else 65536)
        leg = local_leg(args, cm, prm, config, N, B, args.steps, args.warmup, dev, rank, barrier,
                        sync, dist)
        elapsed, timed, units_per_launch = leg["elapsed"], leg["solver"], B
        forces, status, recs_np, solver = leg["forces"], leg["status"], leg["recs_np"], leg["solver"]
        iters = leg["iters"]
        recs = leg["recs"]
        B_total, B_local = B * world, B

    # ---- untimed extras -------------------------------------------------------------------
    launch_ms, ovf = (timed.read_timing() if timed is not None else (np.zeros((0, 2)), 0))
    if config == 4:
        out_forces = pipe.forces if rank == 0 else None
        st_local = pipe.local_status
        if not args.no_extras:
            barrier()
            sync()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                pipe.solve_only()
            sync()
            so = time.perf_counter() - t1
            if dist is not None:
                t = torch.tensor([so], dtype=torch.float64, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                so = float(t.item())
            extras["solve_only"] = {
                "value": round(B_total * args.steps / so, 1), "ms_per_step": round(so / args.steps * 1e3, 4),
                "what": "the same per-rank pieces solved with no collective (max over ranks)"}
    else:
        out_forces, st_local = forces, status
        if config == 3 and not args.dry_run and not args.no_extras and world == 1:
            # end to end: records from pinned host memory, H2D + solve + D2H per step
            h_recs = torch.from_numpy(recs_np).pin_memory()
            h_forces = torch.empty((B, 12 * N), dtype=torch.float32).pin_memory()
            solver.enable_timing(0)
            sync()
            t1 = time.perf_counter()
            for _ in range(args.steps):
                recs.copy_(h_recs, non_blocking=True)
                solver.solve(recs, forces, status, iters)
                h_forces.copy_(forces, non_blocking=True)
            sync()
            e2e = time.perf_counter() - t1
            extras["end_to_end"] = {
                "value": round(B * args.steps / e2e, 1), "ms_per_step": round(e2e / args.steps * 1e3, 4),
                "what": "H2D of the records from pinned host memory + solve + D2H of the forces "
                        "per step (PCIe-inclusive; not `value`)"}
    if config == 3 and not args.dry_run and not args.no_extras and world == 1:
        extras["abi_latency"] = abi_latency()
        if solver is not None:
            solver.close()
            solver = None
        extras["other_configs"] = other_configs(args, cm, dev, rank, barrier, sync, dist)
        extras["scaling_model"] = scaling_model(args, cm, dev, sync)
    status_counts = None
    if st_local is not None:
        sc = np.bincount(st_local.cpu().numpy(), minlength=5)
        if dist is not None:
            t = torch.tensor(sc.astype(np.int64), device=dev)
            dist.all_reduce(t)
            sc = t.cpu().numpy()
        status_counts = {cm.STATUS_NAMES[i]: int(c) for i, c in enumerate(sc) if c}

    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    value = B_total * args.steps / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    roofline = make_roofline(launch_ms, ovf, units_per_launch, N, value, config)

    cpu = None
    if not args.no_cpu_baseline and world == 1 and not args.dry_run:
        cpu = cpu_baseline(prm, N, config5=(config == 5))

    pct = int(args.random_contact_frac * 100)
    mix = f"A1 trot at random phase + {pct}% Bernoulli(0.5) contact tables"
    if config == 4:
        peer = (B_total - B_local) // max(1, world - 1) if world > 1 else 0
        workload = (f"BASELINE config 4: {B_total} instances in total (N={N}, {mix}) on rank 0's "
                    f"GPU as {args.record_format} records ({4 * pipe.words} B each); per step RCCL "
                    f"point-to-point sends over xGMI -> per-rank expansion + solve of its "
                    f"contiguous shard (rank 0 {B_local}, solved where it lies"
                    + (f"; each peer {peer}" if world > 1 else "") +
                    f") -> the forces back to rank 0, pipelined over {pipe.chunks} pieces per rank")
        metric, scaling = METRIC, "strong"
        par_s = f"dp{world} (contiguous instance shards; RCCL send/recv)"
    elif config == 5:
        workload = (f"BASELINE config 5: horizon N={N}, per step one batched periodic-disturbance "
                    f"estimator step (LogData residual, Gaussian band-pass, DFT sine fit; "
                    f"histories at 400..{400 + args.steps} samples) fused ahead of the solve, "
                    f"batch={B_local} per GPU ({mix})")
        metric, scaling = METRIC_C5, "weak"
        par_s = f"dp{world} (independent instance shards, no data-path collective)"
    else:
        workload = (f"BASELINE config {config}: fused condensation + friction-cone QP, horizon "
                    f"N={N}, batch={B_local} per GPU ({mix}), inputs resident in HBM")
        metric, scaling = (METRIC_C2 if config == 2 else METRIC), "weak"
        par_s = f"dp{world} (independent instance shards, no data-path collective)"
    out = {
        "metric": metric,
        "value": round(value, 1),
        "unit": "QP solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (per-instance Philox, seed 0x5EED0000 + id)",
        "config": {
            "workload": workload,
            "config": config,
            "global_batch": B_total,
            "batch_per_gpu": B_local,
            "horizon": N,
            "parallelism": par_s,
        },
        "roofline": roofline,
        "cpu_baseline": cpu,
        "status_counts": status_counts,
        "forces_digest": digest(out_forces) if out_forces is not None else None,
    }
    if getattr(args, "no_refine", False):
        out["config"]["refine"] = "off (A/B run, cmpc_batch_set_refine(0): not the product setting)"
    if args.dry_run:
        out["dry_run"] = "gloo CPU ranks, plumbing stand-in for the solve (not a measurement)"
    out.update(extras)
    print(json.dumps(out), flush=True)
    if solver is not None:
        solver.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
