"""Is a small batch host-bound? (diagnostic, not part of the product path.) Enqueues K solves of
config 2 (4096 instances, N = 10) without synchronising and prints the host time per enqueue
next to the device time per solve: equal times mean the GPU waits for the host.

usage (GPU box): python scripts/host_rate_probe.py [--batch 4096] [--steps 400]
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=400)
    a = ap.parse_args()
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    torch.cuda.set_stream(torch.cuda.Stream())
    N, B = 10, a.batch
    prm = cm.make_params(N)
    recs = torch.from_numpy(cm.make_instances(B, N)).cuda()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())
    for _ in range(20):
        s.solve(recs, f, st)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        s.solve(recs, f, st)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"batch {B}: host {1e6 * (t1 - t0) / a.steps:.1f} us per enqueued solve, "
          f"device {1e6 * (t2 - t0) / a.steps:.1f} us per solve (wall incl. drain)")
    # the same with a sleep-free host already far ahead: enqueue then measure the GPU alone
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    ev0.record()
    for _ in range(a.steps):
        s.solve(recs, f, st)
    ev1.record()
    torch.cuda.synchronize()
    print(f"batch {B}: stream time {1e3 * ev0.elapsed_time(ev1) / a.steps:.1f} us per solve")
    s.close()


if __name__ == "__main__":
    main()
