"""Does a solve's time depend on what the process created before it? (diagnostic, not part of the
product path). Times B instances (N = 10, config-3 mix) on a fresh handle, again after several
handles were created and destroyed (as bench.py does before its scaling model), and through a
world-1 parallel.RootPipeline, in one process. ms per solve, 20 solves after 3 warm-ups.

usage (GPU box): python scripts/stream_probe.py [--batch 32768]
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
    ap.add_argument("--batch", type=int, default=32768)
    a = ap.parse_args()
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    torch.cuda.set_stream(torch.cuda.Stream())
    N, B = 10, a.batch
    prm = cm.make_params(N)
    recs = torch.from_numpy(cm.make_instances(B, N)).cuda()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")

    def timeit(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e3

    def fresh(label):
        s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())
        t = timeit(lambda: s.solve(recs, f, st))
        s.enable_timing(10)
        for _ in range(10):
            s.solve(recs, f, st)
        ms, _ = s.read_timing()
        s.close()
        print(f"{label:40s} {t:.4f} ms  (class 1 {ms[:, 0].mean():.4f}, beyond it {ms[:, 1].mean():.4f})",
              flush=True)

    def piped(label):
        pipe = par.RootPipeline(prm, B, chunks=1, device="cuda")
        t = timeit(lambda: pipe.step(recs))
        pipe.close()
        print(f"{label:40s} {t:.4f} ms", flush=True)

    if os.environ.get("PROBE_ORDER") == "model":  # the scaling model's pieces, twice
        recs_all = torch.from_numpy(cm.make_instances(262144, N)).cuda()
        for rep in range(2):
            for G in (1, 2, 4, 8):
                local = 262144 // G
                pipe = par.RootPipeline(prm, local, chunks=par.auto_chunks(local, G), device="cuda")
                t = timeit(lambda: pipe.step(recs_all[:local]))
                pipe.close()
                print(f"rep {rep} G={G}: {local} in {len(pipe.sizes)} pieces {t:.4f} ms", flush=True)
        return
    if os.environ.get("PROBE_ORDER") == "pipe_first":
        piped("RootPipeline first")
        fresh("fresh after it")
        time.sleep(5)
        fresh("fresh after 5 s idle")
        piped("RootPipeline again")
        fresh("fresh again")
        return
    fresh("fresh handle")
    for k in range(6):  # handles of other sizes, created and destroyed
        s = sm.BatchSolver(prm, max_batch=4096 * (k + 1))
        s.solve(recs[:4096], f[:4096], st[:4096])
        torch.cuda.synchronize()
        s.close()
    fresh("after 6 handles created / destroyed")
    keep = [sm.BatchSolver(prm, max_batch=4096) for _ in range(3)]
    fresh("with 3 other live handles")
    for s in keep:
        s.close()
    pipe = par.RootPipeline(prm, B, chunks=1, device="cuda")
    t = timeit(lambda: pipe.step(recs))
    pipe.close()
    print(f"{'RootPipeline world 1, one piece':40s} {t:.4f} ms", flush=True)
    fresh("fresh handle again")


if __name__ == "__main__":
    main()
