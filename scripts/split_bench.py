"""Where the config-3 step goes: the bench batch solved whole, then split into its class-1
instances (n <= 64) and its wide instances (n > 64) solved alone, and the latency of a single
wide / class-1 instance. Prints one line per case (ms per solve, HIP-event class timings).

  python scripts/split_bench.py [--batch 65536 --horizon 10 --reps 20]
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
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--random-contact-frac", type=float, default=0.25)
    a = ap.parse_args()
    import torch
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    N, B = a.horizon, a.batch
    recs_np = cm.make_instances(B, N, random_contact_frac=a.random_contact_frac)
    n = 3 * (cm.unpack_gait(recs_np, N) != 0).sum(1)
    prm = cm.make_params(N)
    torch.cuda.set_stream(torch.cuda.Stream())
    s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())

    def run(sel, name, reps=a.reps):
        r = torch.from_numpy(np.ascontiguousarray(recs_np[sel])).cuda()
        b = r.shape[0]
        f = torch.empty((b, 12 * N), device="cuda")
        st = torch.empty(b, dtype=torch.uint8, device="cuda")
        it = torch.empty(b, dtype=torch.int32, device="cuda")
        s.solve(r, f, st, it)
        torch.cuda.synchronize()
        s.enable_timing(reps)
        t0 = time.perf_counter()
        for _ in range(reps):
            s.solve(r, f, st, it)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps * 1e3
        ms, ovf = s.read_timing()
        hist = np.bincount(np.minimum(n[sel] // 16, 8), minlength=9)
        print(f"{name:28s} batch {b:6d}: {dt:8.3f} ms/solve  class1 {ms[:, 0].mean():7.3f}  "
              f"tail {ms[:, 1].mean():7.3f}  wide {ovf:5d}  ok {(st.cpu().numpy() == 0).mean():.4f}"
              f"  n/16 hist {hist.tolist()}", flush=True)

    allm = np.ones(B, bool)
    run(allm, "whole batch")
    run(n <= 64, "class-1 instances only")
    run(n > 64, "wide instances only")
    for lo, hi in ((65, 80), (81, 96), (97, 128)):
        m = (n >= lo) & (n <= hi)
        if m.any():
            run(m, f"wide n in [{lo},{hi}]")
    i1 = np.nonzero(n <= 64)[0][:1]
    iw = np.nonzero((n > 64) & (n <= 80))[0][:1]
    run(i1, "single class-1 instance", reps=50)
    if iw.size:
        run(iw, "single n<=80 instance", reps=50)
    s.close()


if __name__ == "__main__":
    main()
