"""Throughput vs batch size for one size class: instances of a fixed reduced size (trot tables,
n = 60 at N = 10, 96 at N = 16, 120 at N = 20) solved in batches from a few hundred to the full
bench batch. Separates the per-wave latency (small batches: one round of waves) from the steady
state (many rounds), and shows where the GPU fills.

  python scripts/occupancy_sweep.py [--horizon 10] [--batches 256,1024,4096,16384,65536]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--batches", default="256,1024,2048,4096,8192,16384,32768,65536")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--random-contact-frac", type=float, default=0.0)
    a = ap.parse_args()
    import torch
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    N = a.horizon
    batches = [int(x) for x in a.batches.split(",")]
    B = max(batches)
    recs_np = cm.make_instances(B, N, random_contact_frac=a.random_contact_frac)
    n = 3 * (cm.unpack_gait(recs_np, N) != 0).sum(1)
    prm = cm.make_params(N)
    torch.cuda.set_stream(torch.cuda.Stream())
    s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())
    recs = torch.from_numpy(recs_np).cuda()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    it = torch.empty(B, dtype=torch.int32, device="cuda")
    for b in batches:
        r = recs[:b]
        s.solve(r, f[:b], st[:b], it[:b])
        torch.cuda.synchronize()
        s.enable_timing(a.reps)
        t0 = time.perf_counter()
        for _ in range(a.reps):
            s.solve(r, f[:b], st[:b], it[:b])
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps * 1e3
        ms, _ = s.read_timing()
        whole = ms[:, 0].mean() + ms[:, 1].mean()
        print(f"N={N} batch {b:6d}: {dt:8.3f} ms/solve  {b / dt / 1e3:7.2f} M QP/s  class1 "
              f"{ms[:, 0].mean():7.3f} ms  tail {ms[:, 1].mean():7.3f}  per-round-of-16/CU "
              f"{whole / max(1.0, b / 4096):7.4f} ms  n {np.unique(n[:b]).tolist()[:6]}  "
              f"ok {(st[:b].cpu().numpy() == 0).mean():.4f}  iters {it[:b].float().mean().item():.2f}",
              flush=True)
    s.close()


if __name__ == "__main__":
    main()
