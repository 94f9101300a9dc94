"""Parity margin against the reference pipeline (oracle/_ref: restated fp32 condensation + the
reference's qpOASES) on large seeded samples, per horizon and contact mix: max / p99.9 of the
per-instance force error |f - q|_inf / max(|q|_inf, 1 N) and how many instances exceed 5e-5 and
1e-4. Solves through whichever library CMPC_LIB names (default: the in-tree build), so two runs
compare two builds (e.g. the refinement on and off at a horizon).

usage: python scripts/parity_margin.py [B] [N ...]
"""
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    from oracle import oracle as orc
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    horizons = [int(a) for a in sys.argv[2:]] or [11, 12, 13, 14, 15, 16]
    mixes = [(0.0, "trotting", False), (0.25, "trotting", False), (1.0, "trotting", False),
             (0.0, "standing", False), (0.0, "walking", False), (1.0, "trotting", True)]
    print(f"lib: {os.environ.get('CMPC_LIB', 'in-tree')}", flush=True)
    for N in horizons:
        prm = cm.make_params(N)
        s = sm.BatchSolver(prm, max_batch=B)
        for frac, gait, stress in mixes:
            t0 = time.time()
            recs = cm.make_instances(B, N, seed=91000 + 10 * N + int(4 * frac), stress=stress,
                                     random_contact_frac=frac, gait=gait)
            f, st, _ = s.solve_host(recs)
            q, st_ref, _ = orc.ref_solve_batch(recs, prm, nthreads=16)
            ok = st_ref == 0
            fr = np.asarray(f, np.float64)[ok]
            qr = q[ok]
            err = np.abs(fr - qr).max(axis=1) / np.maximum(np.abs(qr).max(axis=1), 1.0)
            print(f"N={N:2d} {gait:9s} frac={frac:4.2f} stress={int(stress)}: {ok.sum()} solved, "
                  f"unsolved ours {(st[ok] != 0).sum()}, max {err.max():.2e} p99.9 "
                  f"{np.quantile(err, 0.999):.2e} >5e-5 {(err > 5e-5).sum()} >1e-4 {(err > 1e-4).sum()} "
                  f"({time.time() - t0:.1f} s)", flush=True)
        s.close()


if __name__ == "__main__":
    main()
