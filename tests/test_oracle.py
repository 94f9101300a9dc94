"""CPU tests of the oracle itself (test infrastructure): closed-form discretisation against
scipy's expm, the condensed prediction against a forward simulation, and the oracle pipeline
against the committed qpOASES golden fixtures."""
import numpy as np
import pytest
from scipy.linalg import expm

from conftest import GOLDEN_SETS, golden_params, load_golden, rel_force_err


def test_discretisation_matches_expm(cm, orc):
    prm = cm.make_params(10)
    recs = cm.make_instances(16, 10, seed=5)
    for rec in recs:
        c = orc.condense(rec, prm, full=False)
        A, B, Q = orc.ct_mats64(rec)
        M = np.zeros((31, 31))
        M[:13, :13] = A; M[:13, 13:25] = B; M[:13, 25:31] = Q
        E = expm(prm.dt * M)
        np.testing.assert_allclose(c["Adt"], E[:13, :13], rtol=0, atol=2e-7)
        np.testing.assert_allclose(c["Bdt"], E[:13, 13:25], rtol=0, atol=2e-7)
        np.testing.assert_allclose(c["Qdt"], E[:13, 25:31], rtol=0, atol=2e-7)


def test_nilpotent_generator(cm, orc):
    """A_c^3 = 0 for every state (the closed-form discretisation relies on it)."""
    for rec in cm.make_instances(8, 10, seed=6):
        A, _, _ = orc.ct_mats64(rec)
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


# ---- config 5: periodic-disturbance estimation (parity anchor: numpy, since FFTW is absent) --
def _np_gaussian(data, sigma):
    """Independent numpy restatement of gaussian_filter (SolverMPC.cpp:404-437)."""
    r = int(np.ceil(3 * sigma))
    i = np.arange(-r, r + 1)
    k = np.exp(-0.5 * (i * i) / np.float64(np.float32(sigma) * np.float32(sigma))).astype(np.float32)
    s = np.float32(0)
    for x in k:
        s = np.float32(s + x)
    k = (k / s).astype(np.float32)
    idx = np.clip(np.arange(data.size)[:, None] + i[None, :], 0, data.size - 1)
    return (data[idx] * k.astype(np.float64)[None, :]).sum(1)


def test_gaussian_filter_matches_numpy(orc):
    rng = np.random.default_rng(5)
    x = rng.normal(0, 3, 400)
    for sigma in (7.0, 27.0):
        np.testing.assert_allclose(orc.gaussian_filter(x, sigma), _np_gaussian(x, sigma),
                                   rtol=1e-12, atol=1e-12)


def test_fit_sin_peak_matches_numpy_fft(cm, orc):
    """The DFT-peak search (FFTW r2c in the reference, SolverMPC.cpp:489-510) against numpy's
    FFT on band-passed config-5 windows: same peak bin, same frequency, amp = sqrt(2) std."""
    f3, t = cm.make_disturbance(24, 400, seed=77)
    for i in range(f3.shape[0]):
        d = f3[i].astype(np.float64)
        band = orc.gaussian_filter(d, 7.0) - orc.gaussian_filter(d, 27.0)
        amp, freq, phase, offset, k = orc.fit_sin(t.astype(np.float64), band)
        mags = np.abs(np.fft.rfft(band))
        assert k == 1 + int(np.argmax(mags[1:]))
        dt = float(t[1]) - float(t[0])
        assert freq == pytest.approx(k / (400 * dt), rel=1e-12)
        assert amp == pytest.approx(np.sqrt(2) * band.std(), rel=1e-10)
        assert offset == pytest.approx(band.mean(), abs=1e-10)
        assert phase == 0.0
        assert abs(freq - 0.33) < 1.0 / (400 * dt)  # the injected 0.33 Hz disturbance


def test_estimator_step_semantics(cm, orc):
    """SolverMPC.cpp:688-811: no compensation before 400 samples, re-estimation while the
    history holds 400..500 samples, f_est in qg only above 500, frozen estimate afterwards."""
    f3, t = cm.make_disturbance(1, 560, seed=78)
    st = np.zeros(orc.EST_WORDS, np.float32)
    out = [orc.est_step(st, f3[0, k], t[k]) for k in range(560)]
    fest = np.array([o[0] for o in out])
    use = np.array([o[1] for o in out])
    assert (fest[:399] == 0).all() and fest[399] != 0
    assert not use[:500].any() and use[500:].all()
    prm = st[804:812].view(np.float64)
    amp, freq = prm[1], prm[2]
    # after 500 samples the estimate is frozen: f_est3 = amp + sin(2 pi t f)
    k = 555
    assert fest[k] == np.float32(amp + np.sin(2 * np.pi * np.float64(t[k]) * freq))


def test_residual_matches_numpy(cm, orc):
    """ConvexMPCLocomotion.cpp:639-771 restated independently in numpy."""
    recs = cm.make_instances(8, 10, seed=79)
    logs = cm.make_logs(recs)
    r = cm.records
    for i in range(8):
        lg, rec = logs[i].astype(np.float64), recs[i].astype(np.float64)
        R = lg[r.LOG_ROT:r.LOG_ROT + 9].reshape(3, 3)
        A = np.zeros((13, 13)); A[3, 9] = A[4, 10] = A[5, 11] = A[11, 12] = 1
        A[11, 9] = lg[r.LOG_XDRAG]; A[0:3, 6:9] = R.T
        Iinv = np.linalg.inv(R @ np.diag([0.07, 0.26, 0.242]) @ R.T)
        B = np.zeros((13, 12))
        for b in range(4):
            rv = lg[r.LOG_R + np.array([0, 4, 8]) + b]
            cmx = np.array([[0, -rv[2], rv[1]], [rv[2], 0, -rv[0]], [-rv[1], rv[0], 0]])
            B[6:9, 3 * b:3 * b + 3] = Iinv @ cmx
            B[9:12, 3 * b:3 * b + 3] = np.eye(3) / 12
        xk = np.concatenate([rec[r.REC_RPY:r.REC_RPY + 3], rec[r.REC_P:r.REC_P + 3],
                             rec[r.REC_W:r.REC_W + 3], rec[r.REC_V:r.REC_V + 3], [-9.81]])
        xp = np.concatenate([lg[r.LOG_EUL:r.LOG_EUL + 3], lg[r.LOG_POS:r.LOG_POS + 3],
                             lg[r.LOG_ANG:r.LOG_ANG + 3], lg[r.LOG_LIN:r.LOG_LIN + 3], [-9.81]])
        e = xk - A @ xp - B @ (-lg[r.LOG_FORCE:r.LOG_FORCE + 12])
        ref = np.array([-e[6], -e[7], e[8], e[9], e[10], e[11]])
        np.testing.assert_allclose(orc.residual(logs[i], recs[i]), ref, rtol=2e-5, atol=2e-5)


def test_config5_golden_self_consistent(cm, orc):
    """The committed config-5 fixture replays through the oracle bit for bit."""
    g = load_golden("n20_config5")
    for i in range(4):
        st = np.zeros(orc.EST_WORDS, np.float32)
        seq = [orc.est_step(st, g["f3"][i, k], g["t"][k])[0] for k in range(g["f3"].shape[1])]
        np.testing.assert_array_equal(np.array(seq, np.float32), g["fest_ref"][i])


def test_fp64_pipeline_close_to_reference(cm, orc):
    """oracle.fp64_solve (the float64 optimum the parity rule at N >= 17 falls back to) agrees
    with the reference fp32 pipeline to the reference's own rounding: <= 2e-5 at N = 10 and
    <= 1.5e-4 at N = 20 (scripts/exact_gap.py)."""
    if not orc.ref_available():
        pytest.skip("oracle/_ref not present")
    for N, tol in ((10, 2e-5), (20, 1.5e-4)):
        prm = cm.make_params(N)
        recs = cm.make_instances(8, N, seed=4242 + N, random_contact_frac=0.5)
        q, st, _ = orc.ref_solve_batch(recs, prm, nthreads=4)
        for i in range(len(recs)):
            x64, ri = orc.fp64_solve(recs[i], prm)
            assert ri == 0 and st[i] == 0
            assert np.abs(q[i] - x64).max() / max(np.abs(x64).max(), 1.0) <= tol


@pytest.mark.parametrize("N", [10, 16, 20])
def test_blocked_condensation_bitwise(cm, orc, N):
    """The CPU baseline's register-tiled dense products (oracle_set_impl(1), cmpc_oracle.c
    condense_blocked) sum every dot product in the naive loops' order: the reference pipeline's
    forces, status and nWSR are bit for bit those of the default implementation."""
    if not orc.ref_available():
        pytest.skip("oracle/_ref not present")
    prm = cm.make_params(N)
    recs = cm.make_instances(64, N, seed=4400 + N, random_contact_frac=0.5)
    q0, s0, w0 = orc.ref_solve_batch(recs, prm, nthreads=4)
    q1, s1, w1 = orc.ref_solve_batch(recs, prm, nthreads=4, impl=1)
    np.testing.assert_array_equal(q0, q1)
    np.testing.assert_array_equal(s0, s1)
    np.testing.assert_array_equal(w0, w1)


def test_summation_orders_bracket_the_default(cm, orc):
    """The three summation orders of the restated condensation (oracle_set_sum_order) are three
    valid fp32 evaluations of SolverMPC.cpp:806-814: at N = 10 (well conditioned) they agree with
    each other within 1e-5 of the forces; order 0 is the golden fixtures' order (bitwise)."""
    if not orc.ref_available():
        pytest.skip("oracle/_ref not present")
    g = load_golden("n10_mixed")
    prm = golden_params(cm, g)
    recs = g["records"][:16]
    q = [orc.ref_solve_batch(recs, prm, nthreads=4, order=o)[0] for o in orc.SUM_ORDERS]
    np.testing.assert_array_equal(q[0], g["q_ref"][:16])
    for o in (1, 2):
        assert rel_force_err(q[o], q[0]).max() <= 1e-5
        assert not np.array_equal(q[o], q[0])   # the orders do round differently
