"""Small-batch solve anatomy (the per-rank batch of config 4 at 8 GPUs, config 2): solves of B
instances back to back on one handle (for a kernel trace), then the active-set trip distribution
and the size-class counts of the batch. Run under rocprofv3 --kernel-trace and read the steps with
scripts/trace_timeline.py.

  python scripts/small_batch_probe.py [B ...]
"""
import importlib
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    torch.cuda.set_stream(torch.cuda.Stream())
    N = 10
    prm = cm.make_params(N)
    for B in [int(x) for x in sys.argv[1:]] or [4096, 32768]:
        rn = cm.make_instances(B, N)
        recs = torch.from_numpy(rn).cuda()
        f = torch.empty((B, 12 * N), device="cuda")
        st = torch.empty(B, dtype=torch.uint8, device="cuda")
        it = torch.empty(B, dtype=torch.int32, device="cuda")
        s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())
        for _ in range(3):
            s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / reps * 1e3
        s.close()
        n = 3 * (cm.unpack_gait(rn, N) != 0).sum(1)
        its = it.cpu().numpy()
        cls = {"<=60": (n <= 60).sum(), "61-64": ((n > 60) & (n <= 64)).sum(),
               "65-72": ((n > 64) & (n <= 72)).sum(), "73-80": ((n > 72) & (n <= 80)).sum(),
               "81-96": ((n > 80) & (n <= 96)).sum(), ">96": (n > 96).sum()}
        q = np.percentile(its, [50, 90, 99, 99.9, 100])
        print(f"B={B}: {ms:.4f} ms/solve ({B / ms / 1e3:.2f} M QP/s); classes "
              + " ".join(f"{k}:{v}" for k, v in cls.items())
              + f"; active-set trips p50/p90/p99/p99.9/max {q.round(1).tolist()}; "
              f"trips of n<=64 max {its[n <= 64].max()}, n>64 max {its[n > 64].max() if (n > 64).any() else 0}",
              flush=True)


if __name__ == "__main__":
    main()
