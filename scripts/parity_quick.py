"""Quick parity check of the loaded library against every golden set (prints max errors)."""
import importlib, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import GOLDEN_SETS, golden_params, load_golden, rel_force_err
cm = importlib.import_module("quad-periodic-mpc_amd")
sm = importlib.import_module("quad-periodic-mpc_amd.solver")
worst = 0.0
for name in GOLDEN_SETS:
    g = load_golden(name)
    prm = golden_params(cm, g)
    s = sm.BatchSolver(prm, max_batch=g["records"].shape[0])
    f, st, it = s.solve_host(g["records"])
    e = rel_force_err(f, g["q_ref"]).max()
    worst = max(worst, e)
    print(f"{name:14s} status={np.bincount(st, minlength=5).tolist()} max_rel_err={e:.2e} iters={it.mean():.1f}")
print("WORST", worst)
sys.exit(0 if worst <= 2e-4 else 3)
