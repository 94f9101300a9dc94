"""Generate the committed golden fixtures (tests/golden/*.npz) with the oracle.

Outputs of the reference pipeline run here: the fp32 condensation restatement
(oracle/cmpc_oracle.c, SolverMPC.cpp:566-950) chained with the reference's own vendored
qpOASES 3.2.0 compiled from /root/reference (oracle/_ref, SolverMPC.cpp:952-982).
Run from the repo root:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
cm = importlib.import_module("quad-periodic-mpc_amd")
from oracle import oracle as orc  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def edge_records(N: int) -> np.ndarray:
    """All-swing, one stance foot, all-stance, x_drag extremes, upside-down-ish orientation."""
    base = cm.make_instances(6, N, seed=99, random_contact_frac=0.0)
    gait = cm.unpack_gait(base, N).astype(np.int32)
    gait[0, :] = 0                       # all swing: n = 0
    gait[1, :] = 0
    gait[1, 0::4] = 1                    # one foot in stance every step
    gait[2, :] = 1                       # all stance: n = 12 N
    gait[3, :] = 0
    gait[3, :4] = 1                      # stance only at the first step
    recs = base.copy()
    off = cm.records.gait_offset(N)
    recs[:, off:off + N] = np.ascontiguousarray(gait.astype(np.uint8)).view(np.float32).reshape(6, N)
    recs[4, cm.records.REC_XDRAG] = 0.5
    recs[5, cm.records.REC_XDRAG] = -0.5
    return recs


def allstance_records(N: int, count: int) -> np.ndarray:
    """Every leg in stance at every step: n = 12 N (the largest reduced QP of a horizon)."""
    recs = cm.make_instances(count, N, seed=1007, random_contact_frac=0.0)
    off = cm.records.gait_offset(N)
    ones = np.ones((count, 4 * N), np.uint8)
    recs[:, off:off + N] = ones.view(np.float32).reshape(count, N)
    return recs


def build_set(name, records, prm, cond_count=0):
    q, st, nw = orc.ref_solve_batch(records, prm, nthreads=8)
    out = dict(records=records, horizon=prm.horizon, dt=prm.dt, mu=prm.mu, f_max=prm.f_max,
               weights=np.array(prm.weights, np.float32), alpha=prm.alpha, q_ref=q, status=st,
               nwsr=nw)
    if cond_count:
        qH, qg, Adt, Bdt, Qdt, x0 = [], [], [], [], [], []
        for i in range(cond_count):
            c = orc.condense(records[i], prm)
            qH.append(c["qH"]); qg.append(c["qg"]); Adt.append(c["Adt"]); Bdt.append(c["Bdt"])
            Qdt.append(c["Qdt"]); x0.append(c["x0"])
        out.update(qH=np.stack(qH), qg=np.stack(qg), Adt=np.stack(Adt), Bdt=np.stack(Bdt),
                   Qdt=np.stack(Qdt), x0=np.stack(x0))
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(name, records.shape, "status", np.bincount(st), "nWSR mean", nw.mean())


def gait_set(count, N, seed, gait):
    return cm.make_instances(count, N, seed=seed, random_contact_frac=0.0, gait=gait)


# name -> (records, params, cond_count)
SETS = {
    "n10_mixed": lambda: (cm.make_instances(48, 10, seed=1001), cm.make_params(10), 4),
    "n10_stress": lambda: (cm.make_instances(16, 10, seed=1002, stress=True), cm.make_params(10), 0),
    "n10_edge": lambda: (edge_records(10), cm.make_params(10), 1),
    "n16_trot": lambda: (cm.make_instances(8, 16, seed=1003, random_contact_frac=0.0), cm.make_params(16), 0),
    "n19_mixed": lambda: (cm.make_instances(8, 19, seed=1004), cm.make_params(19), 0),
    "n20_trot": lambda: (cm.make_instances(8, 20, seed=1005, random_contact_frac=0.0), cm.make_params(20), 1),
    # general size class (n > 128): random contacts at N = 20 and all-stance at N = 12
    "n20_mixed": lambda: (cm.make_instances(16, 20, seed=1006, random_contact_frac=1.0), cm.make_params(20), 0),
    "n12_allstance": lambda: (allstance_records(12, 4), cm.make_params(12), 1),
    # the controller's other gaits (ConvexMPCLocomotion.cpp:46, :48) at the deployed horizon
    # N = 16 (ros_config.yaml:93) and at N = 20: standing n = 12 N (192 / 240: the 192- and
    # 256-column classes), walking n = 138..141 at N = 16 (144 class) and 180 at N = 20 (192)
    "n16_standing": lambda: (gait_set(8, 16, 1010, "standing"), cm.make_params(16), 1),
    "n20_standing": lambda: (gait_set(8, 20, 1011, "standing"), cm.make_params(20), 0),
    "n16_walking": lambda: (gait_set(8, 16, 1012, "walking"), cm.make_params(16), 0),
    "n20_walking": lambda: (gait_set(8, 20, 1013, "walking"), cm.make_params(20), 0),
}


def main(names):
    orc.build()
    for name in names:
        recs, prm, cond = SETS[name]()
        build_set(name, recs, prm, cond_count=cond)


if __name__ == "__main__" and (len(sys.argv) == 1 or sys.argv[1] != "config5"):
    # no arguments: every set; otherwise the named ones (the others stay byte-identical)
    main(sys.argv[1:] or list(SETS))


def build_config5_set(name="n20_config5", batch=32, steps=520, N=20):
    """Config 5: the estimator sequence of every instance (oracle/cmpc_oracle.c restatement of
    SolverMPC.cpp:404-553, 688-798, DFT pinned against numpy's FFT in tests/test_oracle.py),
    then the final step's solve by the reference pipeline with f_est in qg (count > 500)."""
    prm = cm.make_params(N)
    recs = cm.make_instances(batch, N, seed=1008, random_contact_frac=0.0)
    f3, t = cm.make_disturbance(batch, steps, seed=1009)
    fest = np.zeros((batch, steps), np.float32)
    flag = np.zeros((batch, steps), bool)
    for i in range(batch):
        st = np.zeros(orc.EST_WORDS, np.float32)
        for k in range(steps):
            fest[i, k], flag[i, k] = orc.est_step(st, f3[i, k], t[k])
    final = recs.copy()
    final[:, cm.records.REC_FEST3] = fest[:, -1]
    final[:, cm.records.REC_FLAGS] = flag[:, -1].astype(np.uint32).view(np.float32)
    q, status, nw = orc.ref_solve_batch(final, prm, nthreads=8)
    logs = cm.make_logs(recs)
    fext6 = np.stack([orc.residual(logs[i], recs[i]) for i in range(batch)])
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), records=recs, f3=f3, t=t, fest_ref=fest,
                        flag_ref=flag, final_records=final, q_ref=q, status=status, nwsr=nw,
                        logs=logs, fext6_ref=fext6, horizon=N, dt=prm.dt, mu=prm.mu,
                        f_max=prm.f_max, weights=np.array(prm.weights, np.float32),
                        alpha=prm.alpha)
    print(name, "status", np.bincount(status), "f_est3 range", fest[:, -1].min(), fest[:, -1].max())


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "config5":
    build_config5_set()
