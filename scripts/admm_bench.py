"""use_jcqp == 1 throughput: condense + batched JCQP ADMM (cmpc_batch_admm) at N = 10, deployed
settings (ros_config.yaml:73-77) and tight ones; prints one JSON line per setting."""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
cm = importlib.import_module("quad-periodic-mpc_amd")
sm = importlib.import_module("quad-periodic-mpc_amd.solver")
sm.load_library()

B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
REDUCED = len(sys.argv) > 3 and sys.argv[3] == "reduced"
prm = cm.make_params(N)
recs_np = cm.make_instances(B, N, random_contact_frac=0.0) if REDUCED else cm.make_instances(B, N)
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    s = sm.BatchSolver(prm, max_batch=B, stream=st)
    recs = torch.from_numpy(recs_np).cuda()
    H = torch.empty((B, 12 * N, 12 * N), dtype=torch.float32, device="cuda")
    g = torch.empty((B, 12 * N), dtype=torch.float32, device="cuda")
    f = torch.empty((B, 12 * N), dtype=torch.float32, device="cuda")
    status = torch.empty(B, dtype=torch.uint8, device="cuda")
    iters = torch.empty(B, dtype=torch.int32, device="cuda")
    for name, kw in [("deployed", dict()), ("tight", dict(rho=1e-3, terminate=1e-4))]:
        cfg = sm.admm_settings(reduced=REDUCED, **kw)
        s.condense(recs, H, g)
        s.admm(recs, H, g, f, status, iters, settings=cfg)
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            s.condense(recs, H, g)
            s.admm(recs, H, g, f, status, iters, settings=cfg)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        it = iters.cpu().numpy()
        print(json.dumps({"mode": "use_jcqp=2" if REDUCED else "use_jcqp=1", "settings": name, "batch": B, "horizon": N,
                          "qp_per_s": B / dt, "ms": dt * 1e3, "iters_mean": float(it.mean()),
                          "iters_max": int(it.max()),
                          "converged_frac": float((status.cpu().numpy() == 0).mean())}),
              flush=True)
    s.close()
