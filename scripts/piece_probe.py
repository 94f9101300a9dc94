"""Unequal pieces for config 4's per-rank load at 8 ranks (32768 instances on one GPU): one solve
of all of them against a small first piece and the rest solved concurrently on two solver handles
(two lanes, each with its own streams), so a pipeline could start on the first piece while the
second is still in flight over xGMI. ms per step, 20 steps after 3 warm-ups; diagnostic only."""
import importlib
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    N, B = 10, 32768
    prm = cm.make_params(N)
    recs = torch.from_numpy(cm.make_instances(B, N)).cuda()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    lanes = [sm.BatchSolver(prm, max_batch=B, stream=s) for s in streams]

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    print(f"B={B}: one solve {timeit(lambda: lanes[0].solve(recs, f, st)):.3f} ms", flush=True)
    for first in (2048, 4096, 8192, 16384):
        def two():
            lanes[0].solve(recs[:first], f[:first], st[:first])
            lanes[1].solve(recs[first:], f[first:], st[first:])
        def seq():
            lanes[0].solve(recs[:first], f[:first], st[:first])
            lanes[0].solve(recs[first:], f[first:], st[first:])
        print(f"  pieces {first} + {B - first}: two lanes {timeit(two):.3f} ms, one lane {timeit(seq):.3f} ms",
              flush=True)
    for s in lanes:
        s.close()


if __name__ == "__main__":
    main()
