"""GPU cost per instance of each size class in isolation (diagnostic, not part of the product
path): 65536 instances at N = 10 whose contact tables all give the same reduced size n (n / 3
random stance foot-steps of the 40), solved alone, against the trot batch (n = 60, class 1) and
the config-3 mix. Prints ms per solve and ns of GPU per instance.

usage (GPU box): python scripts/class_cost_probe.py [--batch 65536] [--sizes 60,63,66,...]
"""
from __future__ import annotations

import argparse
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def records_with_size(cm, B, N, n, seed):
    """Trot records whose gait tables are replaced by n / 3 random stance foot-steps."""
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    recs = cm.make_instances(B, N, seed=seed, random_contact_frac=0.0)
    rng = np.random.default_rng(seed)
    k = n // 3
    keys = rng.random((B, 4 * N))
    order = np.argsort(keys, axis=1)
    gait = np.zeros((B, 4 * N), np.uint8)
    np.put_along_axis(gait, order[:, :k], 1, axis=1)
    off = R.gait_offset(N)
    recs[:, off:off + N].view(np.uint8)[:, :] = gait
    return recs


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--sizes", default="60,63,66,69,72,75,78,81,84,90,96")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    N, B = a.horizon, a.batch
    prm = cm.make_params(N)
    s = sm.BatchSolver(prm, max_batch=B)
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    it = torch.empty(B, dtype=torch.int32, device="cuda")

    def run(label, recs_np):
        recs = torch.from_numpy(recs_np).cuda()
        for _ in range(3):
            s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        stc = np.bincount(st.cpu().numpy(), minlength=4)
        itm = it.float().mean().item()
        print(f"{label:>12}: {ms:8.3f} ms  {ms * 1e6 / B:7.2f} ns/instance  mean iters {itm:5.2f}  "
              f"status {stc.tolist()}", flush=True)

    run("config3", cm.make_instances(B, N))
    for n in [int(x) for x in a.sizes.split(",")]:
        run(f"n={n}", records_with_size(cm, B, N, n, seed=500 + n))
    s.close()


if __name__ == "__main__":
    main()
