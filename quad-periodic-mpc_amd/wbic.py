"""Host side of the whole-body-impulse-control QP (second half).

``WBIC::MakeTorque`` (be2r_cmpc_unitree/src/controllers/WBC/WBIC/WBIC.cpp:17-142) builds one
small QP per control tick and hands it to QuadProg++'s ``solve_quadprog`` (:91). This module
builds that QP for a batch of robots, exactly as WBIC does, in the dense QuadProg++ layout that
``BatchSolver.quadprog`` / ``cmpc_batch_quadprog`` (include/cmpc_quadprog.h) solves on the GPU:

* variables z = [delta floating-base acceleration (6), delta reaction forces (3 per contact)]
  (``_SetOptimizationSize``, :326-364);
* cost 0.5 z' diag(W_floating, W_rf) z (``_SetCost``, :281-301; WBC_Ctrl.cpp:20-23: 0.1, 1.0);
* 6 equalities, the floating-base rows of the dynamics (``_SetEqualityConstraint``, :144-170):
  [A_fb | -Jc_fb'] z = -(b_fb - Jc_fb' Fr_des), with b_fb = Sv (A qddot + cori + grav);
* 6 inequalities per contact, the friction pyramid and normal-force bounds of SingleContact
  (``_SetInEqualityConstraint``, :172-190; SingleContact.cpp:7-30, 62-66):
  Uf (Fr_des + delta_f) >= ieq.

The reaction forces WBIC passes on are Fr = z[6:] + Fr_des (``_GetSolution``, :244-275).
"""
from __future__ import annotations

import numpy as np

N_MAX, P_MAX, M_MAX = 18, 6, 24      # 4 contacts: n = 6 + 12, 6 equalities, 24 inequalities
W_FLOATING, W_RF = 0.1, 1.0           # WBC_Ctrl.cpp:20, :23
MU, MAX_FZ = 0.4, 1500.0              # SingleContact.cpp:7, :14


def single_contact_uf(mu: float = MU) -> np.ndarray:
    """Uf of SingleContact (SingleContact.cpp:12-29): rows fz, fx + mu fz, -fx + mu fz,
    fy + mu fz, -fy + mu fz, -fz."""
    uf = np.zeros((6, 3))
    uf[0, 2] = 1.0
    uf[1, 0], uf[1, 2] = 1.0, mu
    uf[2, 0], uf[2, 2] = -1.0, mu
    uf[3, 1], uf[3, 2] = 1.0, mu
    uf[4, 1], uf[4, 2] = -1.0, mu
    uf[5, 2] = -1.0
    return uf


def single_contact_ieq(max_fz: float = MAX_FZ) -> np.ndarray:
    """SingleContact::_UpdateInequalityVector (SingleContact.cpp:62-66)."""
    v = np.zeros(6)
    v[5] = -max_fz
    return v


def wbic_qp(A_fb, b_fb, Jc_fb, Fr_des, contact, W_floating=W_FLOATING, W_rf=W_RF, mu=MU,
            max_fz=MAX_FZ):
    """Batched WBIC QPs in QuadProg++ layout.

    A_fb [B,6,6] = A[:6,:6]; b_fb [B,6] = Sv (A qddot_pre + cori + grav); Jc_fb [B,4,3,6] the
    floating-base columns of each foot's contact Jacobian; Fr_des [B,4,3] the MPC forces;
    contact [B,4] bool (the contact list holds the stance feet in leg order).
    -> dict of fp64 blocks G, g0, CE, ce0, CI, ci0 (strides N_MAX, P_MAX, M_MAX) and dims [B,3].
    """
    A_fb = np.asarray(A_fb, np.float64)
    B = A_fb.shape[0]
    G = np.zeros((B, N_MAX, N_MAX))
    g0 = np.zeros((B, N_MAX))
    CE = np.zeros((B, N_MAX, P_MAX))
    ce0 = np.zeros((B, P_MAX))
    CI = np.zeros((B, N_MAX, M_MAX))
    ci0 = np.zeros((B, M_MAX))
    dims = np.zeros((B, 3), np.int32)
    uf1, ieq1 = single_contact_uf(mu), single_contact_ieq(max_fz)
    for b in range(B):
        legs = [l for l in range(4) if contact[b][l]]
        nc = len(legs)
        n = 6 + 3 * nc
        m = 6 * nc if nc else 1      # CI.resize(0., n, 1) without contacts (WBIC.cpp:360-363)
        dims[b] = (n, 6, m)
        G[b, np.arange(6), np.arange(6)] = W_floating                 # _SetCost
        G[b, np.arange(6, n), np.arange(6, n)] = W_rf
        jc = np.concatenate([Jc_fb[b][l] for l in legs], 0) if nc else np.zeros((0, 6))  # [3nc,6]
        fr = np.concatenate([Fr_des[b][l] for l in legs]) if nc else np.zeros(0)
        dyn_CE = np.zeros((6, n))
        dyn_CE[:, :6] = A_fb[b]
        dyn_CE[:, 6:] = -jc.T                                          # -Sv Jc'
        dyn_ce0 = -(np.asarray(b_fb[b], np.float64) - jc.T @ fr)
        CE[b, :n, :] = dyn_CE.T                                        # CE[j][i] = dyn_CE(i, j)
        ce0[b] = -dyn_ce0
        if nc:
            Uf = np.zeros((6 * nc, 3 * nc))
            ieq = np.zeros(6 * nc)
            for c in range(nc):
                Uf[6 * c:6 * c + 6, 3 * c:3 * c + 3] = uf1
                ieq[6 * c:6 * c + 6] = ieq1
            dyn_CI = np.zeros((6 * nc, n))
            dyn_CI[:, 6:] = Uf
            dyn_ci0 = ieq - Uf @ fr
            CI[b, :n, :m] = dyn_CI.T
            ci0[b, :m] = -dyn_ci0
    return dict(G=G, g0=g0, CE=CE, ce0=ce0, CI=CI, ci0=ci0, dims=dims)


def reaction_forces(z, Fr_des, contact):
    """Fr = z[6:] + Fr_des for the stance feet (WBIC.cpp:253-257), as [B,4,3] (0 in swing)."""
    B = z.shape[0]
    out = np.zeros((B, 4, 3))
    for b in range(B):
        k = 6
        for l in range(4):
            if contact[b][l]:
                out[b, l] = z[b, k:k + 3] + Fr_des[b][l]
                k += 3
    return out


def _skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def make_wbic_problems(batch: int, seed: int = 0x5EED0100, contact_probs=(0.05, 0.05, 0.6, 0.1, 0.2)):
    """Synthetic WBIC inputs for an A1-sized robot: composite floating-base inertia (12 kg,
    body inertia of MiniCheetah.h's A1 scaled to the whole robot), foot Jacobians
    R [-skew(p_foot) | I] at the hips (+- 0.18, +- 0.13, -0.28 m), the floating-base dynamics
    b_fb ~ gravity + disturbance, and MPC forces that share the weight over the stance feet with
    random tangential parts (some outside the friction pyramid, so constraints activate).
    contact_probs: P(number of stance feet = 0..4)."""
    g = np.random.Generator(np.random.Philox(seed))
    B = batch
    mass = 12.0
    A_fb = np.zeros((B, 6, 6))
    b_fb = np.zeros((B, 6))
    Jc = np.zeros((B, 4, 3, 6))
    Fr = np.zeros((B, 4, 3))
    contact = np.zeros((B, 4), bool)
    hips = np.array([[0.18, -0.13], [0.18, 0.13], [-0.18, -0.13], [-0.18, 0.13]])
    counts = g.choice(5, size=B, p=np.asarray(contact_probs) / np.sum(contact_probs))
    for b in range(B):
        Ib = np.diag([0.07, 0.26, 0.24]) * g.uniform(0.8, 1.2, 3)
        c = g.normal(0, 0.01, 3)                                 # CoM offset from the base
        A = np.zeros((6, 6))
        A[:3, :3] = Ib + mass * _skew(c) @ _skew(c).T
        A[:3, 3:] = mass * _skew(c)
        A[3:, :3] = mass * _skew(c).T
        A[3:, 3:] = mass * np.eye(3)
        A_fb[b] = A
        rpy = g.normal(0, 0.05, 3)
        cr, sr, cp, sp, cy, sy = (np.cos(rpy[0]), np.sin(rpy[0]), np.cos(rpy[1]), np.sin(rpy[1]),
                                  np.cos(rpy[2]), np.sin(rpy[2]))
        Rm = (np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]]) @
              np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]]) @
              np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]]))
        legs = g.permutation(4)[:counts[b]]
        contact[b, legs] = True
        grav_body = Rm.T @ np.array([0, 0, mass * 9.81])
        b_fb[b, :3] = g.normal(0, 0.5, 3)
        b_fb[b, 3:] = grav_body + g.normal(0, 5.0, 3)
        nc = max(1, counts[b])
        for l in range(4):
            pf = np.array([hips[l, 0], hips[l, 1], -0.28]) + g.normal(0, 0.03, 3)
            Jc[b, l, :, :3] = -Rm @ _skew(pf)
            Jc[b, l, :, 3:] = Rm
            fz = mass * 9.81 / nc * g.uniform(0.6, 1.4)
            Fr[b, l] = (g.normal(0, 0.35 * fz), g.normal(0, 0.35 * fz), fz)
    return dict(A_fb=A_fb, b_fb=b_fb, Jc_fb=Jc, Fr_des=Fr, contact=contact)
