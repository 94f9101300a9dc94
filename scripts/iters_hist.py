"""Active-set iteration histogram of the bench workloads (how many instances would skip the
J = L^-T build if the unconstrained minimiser were checked first)."""
import importlib, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
cm = importlib.import_module("quad-periodic-mpc_amd")
sm = importlib.import_module("quad-periodic-mpc_amd.solver")
torch.cuda.set_stream(torch.cuda.Stream())
for N, frac in ((10, 0.25), (16, 0.0), (20, 0.0), (20, 0.25)):
    B = 65536
    recs_np = cm.make_instances(B, N, random_contact_frac=frac)
    n = 3 * (cm.unpack_gait(recs_np, N) != 0).sum(1)
    recs = torch.from_numpy(recs_np).cuda()
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    it = torch.empty(B, dtype=torch.int32, device="cuda")
    s = sm.BatchSolver(cm.make_params(N), max_batch=B, stream=torch.cuda.current_stream())
    s.solve(recs, f, st, it)
    torch.cuda.synchronize()
    itn = it.cpu().numpy()
    h = np.bincount(np.minimum(itn, 20), minlength=21)
    print(f"N={N} frac={frac}: mean iters {itn.mean():.2f}, zero {np.mean(itn == 0):.3f}, "
          f"hist(0..20+) {h.tolist()}; n>64 zero-frac {np.mean(itn[n > 64] == 0) if (n > 64).any() else 0:.3f}",
          flush=True)
    s.close()
