"""CPU tests of the oracle itself (test infrastructure): closed-form discretisation against
scipy's expm, the condensed prediction against a forward simulation, and the oracle pipeline
against the committed qpOASES golden fixtures."""
import numpy as np
import pytest
from scipy.linalg import expm

from conftest import GOLDEN_SETS, golden_params, load_golden, rel_force_err


def _ct_mats(rec, x0_rpy=None):
    """Independent numpy restatement of ct_ss_mats (SolverMPC.cpp:260-279), float64."""
    q = rec[6:10].astype(np.float64)
    w_, x, y, z = q
    R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w_ * z), 2 * (x * z + w_ * y)],
                  [2 * (x * y + w_ * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w_ * x)],
                  [2 * (x * z - w_ * y), 2 * (y * z + w_ * x), 1 - 2 * (x * x + y * y)]])
    Iw = R @ np.diag([.07, .26, .242]) @ R.T
    Ii = np.linalg.inv(Iw)
    r = rec[13:25].reshape(3, 4).astype(np.float64)
    A = np.zeros((13, 13)); B = np.zeros((13, 12))
    A[3, 9] = A[4, 10] = A[5, 11] = A[11, 12] = 1.0
    A[11, 9] = rec[28]
    A[0:3, 6:9] = R.T
    for b in range(4):
        rx = np.array([[0, -r[2, b], r[1, b]], [r[2, b], 0, -r[0, b]], [-r[1, b], r[0, b], 0]])
        B[6:9, 3 * b:3 * b + 3] = Ii @ rx
        B[9:12, 3 * b:3 * b + 3] = np.eye(3) / 12.0
    Q = np.zeros((13, 6)); Q[6:12] = np.eye(6)
    return A, B, Q


def test_discretisation_matches_expm(cm, orc):
    prm = cm.make_params(10)
    recs = cm.make_instances(16, 10, seed=5)
    for rec in recs:
        c = orc.condense(rec, prm, full=False)
        A, B, Q = _ct_mats(rec)
        M = np.zeros((31, 31))
        M[:13, :13] = A; M[:13, 13:25] = B; M[:13, 25:31] = Q
        E = expm(prm.dt * M)
        np.testing.assert_allclose(c["Adt"], E[:13, :13], rtol=0, atol=2e-7)
        np.testing.assert_allclose(c["Bdt"], E[:13, 13:25], rtol=0, atol=2e-7)
        np.testing.assert_allclose(c["Qdt"], E[:13, 25:31], rtol=0, atol=2e-7)


def test_nilpotent_generator(cm):
    """A_c^3 = 0 for every state (the closed-form discretisation relies on it)."""
    for rec in cm.make_instances(8, 10, seed=6):
        A, _, _ = _ct_mats(rec)
        assert np.abs(np.linalg.matrix_power(A, 3)).max() == 0.0


def test_condensation_matches_forward_simulation(cm, orc):
    """qH/qg define 1/2 U'qH U + qg'U = sum |x_k - xd_k|_S^2 + alpha|U|^2 (up to a constant):
    check the gradient at random U against a forward rollout with the discrete model."""
    N = 10
    prm = cm.make_params(N)
    rng = np.random.default_rng(0)
    for rec in cm.make_instances(4, N, seed=7):
        c = orc.condense(rec, prm)
        A = c["Adt"].astype(np.float64); B = c["Bdt"].astype(np.float64)
        x0 = c["x0"].astype(np.float64)
        traj = rec[32:32 + 12 * N].reshape(N, 12).astype(np.float64)
        w = np.array(list(prm.weights) + [0.0])
        U = rng.normal(0, 30, 12 * N)

        def cost(U):
            x = x0.copy(); J = 0.0
            for k in range(N):
                x = A @ x + B @ U[12 * k:12 * k + 12]
                e = x.copy(); e[:12] -= traj[k]
                J += e @ (w * e)
            return J + prm.alpha * U @ U
        grad_model = c["qH"].astype(np.float64) @ U + c["qg"].astype(np.float64)
        eps = 1e-3
        for idx in rng.choice(12 * N, 6, replace=False):
            dU = np.zeros_like(U); dU[idx] = eps
            fd = (cost(U + dU) - cost(U - dU)) / (2 * eps)
            assert abs(fd - grad_model[idx]) <= 2e-3 * max(1.0, abs(fd)), (idx, fd, grad_model[idx])


@pytest.mark.parametrize("name", GOLDEN_SETS)
def test_oracle_pipeline_reproduces_golden(cm, orc, name):
    if not orc.ref_available():
        pytest.skip("oracle/_ref (qpOASES from /root/reference) not built")
    g = load_golden(name)
    prm = golden_params(cm, g)
    q, st, nw = orc.ref_solve_batch(g["records"], prm, nthreads=4)
    assert (st == g["status"]).all()
    assert rel_force_err(q, g["q_ref"]).max() <= 1e-9


@pytest.mark.parametrize("name", ["n10_mixed", "n10_edge", "n20_trot"])
def test_oracle_condensation_reproduces_golden(cm, orc, name):
    g = load_golden(name)
    prm = golden_params(cm, g)
    for i in range(g["qH"].shape[0]):
        c = orc.condense(g["records"][i], prm)
        np.testing.assert_array_equal(c["qH"], g["qH"][i])
        np.testing.assert_array_equal(c["qg"], g["qg"][i])


def test_golden_solutions_satisfy_kkt(cm):
    """qpOASES solutions in the fixtures are feasible for the friction pyramid (sanity)."""
    for name in GOLDEN_SETS:
        g = load_golden(name)
        N = int(g["horizon"])
        mu = float(g["mu"])
        q = g["q_ref"].reshape(-1, N, 4, 3)
        fx, fy, fz = q[..., 0], q[..., 1], q[..., 2]
        tol = 1e-6 * max(1.0, np.abs(q).max())
        assert (fz >= -tol).all()
        assert (np.abs(fx) <= mu * fz + tol).all() and (np.abs(fy) <= mu * fz + tol).all()
        assert (fz <= float(g["f_max"]) + tol).all()
