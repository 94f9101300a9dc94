"""Where the small-batch / pipeline time goes (config 4's per-rank loads on one GPU): a direct
cmpc_batch_solve of B instances vs parallel.RootPipeline (world 1) over the same records in 1, 2
and 4 pieces, with one and two solver lanes. ms per step, 20 steps after 3 warm-ups."""
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
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    torch.cuda.set_stream(torch.cuda.Stream())
    N = 10
    prm = cm.make_params(N)
    for B in (16384, 32768, 65536):
        recs = torch.from_numpy(cm.make_instances(B, N)).cuda()
        f = torch.empty((B, 12 * N), device="cuda")
        st = torch.empty(B, dtype=torch.uint8, device="cuda")
        s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())

        def timeit(fn, reps=20):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / reps * 1e3

        t_direct = timeit(lambda: s.solve(recs, f, st))
        s.close()
        row = [f"B={B}: direct {t_direct:.3f}"]
        for chunks in (1, 2, 4):
            for lanes in (1, 2):
                if lanes > chunks:
                    continue
                pipe = par.RootPipeline(prm, B, chunks=chunks, device="cuda", lanes=lanes)
                t = timeit(lambda: pipe.step(recs))
                pipe.close()
                row.append(f"pieces {chunks} lanes {lanes}: {t:.3f}")
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
