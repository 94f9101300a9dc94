"""Stage-level cycle breakdown of the tail-class kernel (diagnostic, not part of the product path),
beside class 1's at the same batch.

Build (here, CPU):  python scripts/tail_phase_prof.py --build
Run (GPU box):      python scripts/tail_phase_prof.py [--batch 256 --sizes 66,72,78]

The diagnostic library is the product kernels compiled with -DCMPC_PHASE_PROF: lane 0 of every
instance adds the s_memtime cycles of each stage to a device counter. At a small batch every wave
is alone on its SIMD, so the numbers are per-wave latencies.
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
PROF_LIB = os.path.join(ROOT, "variants", "libcmpc_tprof.so")
STAGES = ["condensation (both passes)", "H rows + tail block load", "Cholesky, 64 main pivots",
          "Cholesky, tail pivots", "J = L^-T (+ J22)", "x = -J y", "active set", "scatter"]
C1_STAGES = ["prep", "condensation H", "Cholesky", "J = L^-T", "active set", "scatter"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--sizes", default="60,66,72,78")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    if a.build:
        os.makedirs(os.path.dirname(PROF_LIB), exist_ok=True)
        b = importlib.import_module("quad-periodic-mpc_amd.build")
        print(b.build(out=PROF_LIB, defines=("CMPC_PHASE_PROF",)))
        return
    import numpy as np
    import torch
    from class_cost_probe import records_with_size

    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    lib = sm.load_library(PROF_LIB)
    cm = importlib.import_module("quad-periodic-mpc_amd")
    N, B = 10, a.batch
    s = sm.BatchSolver(cm.make_params(N), max_batch=B)
    out = (ctypes.c_ulonglong * 16)()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    it = torch.empty(B, dtype=torch.int32, device="cuda")
    for n in [int(x) for x in a.sizes.split(",")]:
        recs = torch.from_numpy(records_with_size(cm, B, N, n, seed=700 + n)).cuda()
        s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        lib.cmpc_debug_tphase_read(out)
        lib.cmpc_debug_phase_read(out)
        for _ in range(a.reps):
            s.solve(recs, f, st, it)
        torch.cuda.synchronize()
        if n <= 64:
            lib.cmpc_debug_phase_read(out)
            v = np.array(list(out), dtype=np.float64)
            inst, iters, names, k = max(v[6], 1.0), v[7], C1_STAGES, 6
        else:
            lib.cmpc_debug_tphase_read(out)
            v = np.array(list(out), dtype=np.float64)
            inst, iters, names, k = max(v[8], 1.0), v[9], STAGES, 8
        tot = v[:k].sum()
        print(f"n = {n}: {int(inst)} instances, mean active-set iterations {iters / inst:.2f}, "
              f"mean {tot / inst:.0f} cycles / instance ({tot / inst / 2.4e3:.1f} us at 2.4 GHz)")
        for i, name in enumerate(names):
            print(f"    {name:36s} {v[i] / inst:10.0f} cyc  {100 * v[i] / max(tot, 1):5.1f} %")
    s.close()


if __name__ == "__main__":
    main()
