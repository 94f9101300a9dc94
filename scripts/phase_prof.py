"""Stage-level cycle breakdown of the class-1 kernel (diagnostic, not part of the product path).

Build (here, CPU):  python scripts/phase_prof.py --build
Run (GPU box):      python scripts/phase_prof.py [--batch 65536 --horizon 10]

The diagnostic library is the product kernels compiled with -DCMPC_PHASE_PROF: lane 0 of every
class-1 instance adds the s_memtime cycles of each stage to a device counter. The numbers are
per-wave latencies (waves on a SIMD interleave), so they rank the stages; the kernel time
itself comes from bench.py / rocprofv3.
"""
from __future__ import annotations

import argparse
import ctypes
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PROF_LIB = os.path.join(ROOT, "quad-periodic-mpc_amd", "libcmpc_prof.so")
STAGES = ["prep (stance, model, gradient recursion)", "condensation H", "Cholesky [H|g]",
          "J = L^-T", "active set (x = -Jy, GI loop)", "scatter"]
GI_SEGS = ["select the most violated constraint", "export J rows, d, z = J d, |d|^2",
           "back substitution, step lengths", "add / drop: R update", "J reflection (every trip)",
           "J Givens chain (drops)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default=PROF_LIB)
    a = ap.parse_args()
    if a.build:
        b = importlib.import_module("quad-periodic-mpc_amd.build")
        print(b.build(out=PROF_LIB, defines=("CMPC_PHASE_PROF",)))
        return
    import numpy as np
    import torch

    solver_mod = importlib.import_module("quad-periodic-mpc_amd.solver")
    lib = solver_mod.load_library(a.lib)
    cm = importlib.import_module("quad-periodic-mpc_amd")
    N, B = a.horizon, a.batch
    recs = torch.from_numpy(cm.make_instances(B, N)).cuda()
    forces = torch.empty((B, 12 * N), dtype=torch.float32, device="cuda")
    status = torch.empty(B, dtype=torch.uint8, device="cuda")
    iters = torch.empty(B, dtype=torch.int32, device="cuda")
    s = solver_mod.BatchSolver(cm.make_params(N), max_batch=B)
    out = (ctypes.c_ulonglong * 16)()
    s.solve(recs, forces, status, iters)
    torch.cuda.synchronize()
    lib.cmpc_debug_phase_read(out)  # reset after the warm-up solve
    for _ in range(a.reps):
        s.solve(recs, forces, status, iters)
    torch.cuda.synchronize()
    if lib.cmpc_debug_phase_read(out) != 0:
        raise RuntimeError("cmpc_debug_phase_read failed")
    v = np.array(list(out), dtype=np.float64)
    inst = max(v[6], 1.0)
    tot = v[:6].sum()
    print(f"class-1 instances {int(v[6])} over {a.reps} solves, mean active-set iterations "
          f"{v[7] / inst:.2f}, mean {tot / inst:.0f} cycles / instance")
    for i, name in enumerate(STAGES):
        print(f"  {name:45s} {v[i] / inst:10.0f} cyc  {100 * v[i] / tot:5.1f} %")
    trips = max(v[7], 1.0)
    print(f"  active-set trips {int(v[7])}, drops {int(v[14])}; per trip:")
    for i, name in enumerate(GI_SEGS):
        print(f"    {name:43s} {v[8 + i] / trips:10.0f} cyc")
    s.close()


if __name__ == "__main__":
    main()
