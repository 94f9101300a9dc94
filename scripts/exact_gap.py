"""How far is the reference's fp32 pipeline from the exact (fp64) optimum?

For a seeded batch: (1) the reference pipeline (fp32 condensation as SolverMPC.cpp + the
reference's qpOASES), (2) an fp64 pipeline (scipy expm discretisation, dense fp64 condensation,
the same swing elimination and qpOASES on the fp64 reduced QP). Prints the distribution of the
reference's relative force gap to the fp64 optimum, the quantity that bounds any parity tolerance
between two correct fp32 implementations. CPU only (test infrastructure: uses oracle/).

usage: python scripts/exact_gap.py [--horizon 20] [--batch 512] [--seed 7020] [--frac 1.0]
"""
import argparse
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from oracle import oracle as orc  # noqa: E402

cm = importlib.import_module("quad-periodic-mpc_amd")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--seed", type=int, default=7020)
    ap.add_argument("--frac", type=float, default=1.0)
    ap.add_argument("--stress", action="store_true")
    a = ap.parse_args()
    prm = cm.make_params(a.horizon)
    recs = cm.make_instances(a.batch, a.horizon, seed=a.seed, stress=a.stress,
                             random_contact_frac=a.frac)
    q, st, _ = orc.ref_solve_batch(recs, prm, nthreads=8)
    gaps = []
    for i in range(a.batch):
        if st[i] != 0:
            continue
        xe, ri = orc.fp64_solve(recs[i], prm)
        if ri != 0:
            continue
        gaps.append(np.abs(q[i] - xe).max() / max(np.abs(xe).max(), 1.0))
    g = np.array(gaps)
    print(f"N={a.horizon} frac={a.frac} seed={a.seed}: {len(g)} instances; ref-vs-fp64 gap "
          f"max {g.max():.3e} p99 {np.quantile(g, .99):.3e} median {np.median(g):.3e} "
          f"argmax {int(np.argmax(g))}")


if __name__ == "__main__":
    main()
