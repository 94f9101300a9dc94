"""GPU tests of config 5 (periodic-disturbance estimation fused ahead of the N = 20 solve):
the batched estimator kernel (cmpc_batch_estimate) against the oracle's restatement of
SolverMPC.cpp:688-811 step by step, the device residual against ConvexMPCLocomotion.cpp:639-771,
and the full estimate -> solve pipeline against the reference qpOASES forces (fixture
tests/golden/n20_config5.npz, made by tests/golden/make_golden.py config5).

Tolerances: flags and the moment compensation starts are exact; f_est(3) within 1e-5 relative
(double-precision filters and DFT on both sides, summation orders differ); forces 1e-4 as the
other N = 20 sets (tests/test_gpu_parity.py)."""
import importlib

import numpy as np
import pytest

from conftest import golden_params, load_golden, rel_force_err

pytestmark = pytest.mark.gpu


@pytest.fixture
def on_stream():
    """Every torch op of a test and the solver handle on ONE non-default stream, so kernels of
    the library and torch copies are ordered."""
    import torch
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        yield st
    torch.cuda.synchronize()


@pytest.fixture(scope="module")
def solver_mod():
    mod = importlib.import_module("quad-periodic-mpc_amd.solver")
    mod.load_library()
    return mod


def _run_sequence(torch, s, g, B):
    recs = torch.from_numpy(np.ascontiguousarray(g["records"][:B])).cuda()
    est = torch.zeros((B, 816), dtype=torch.float32, device="cuda")
    f3 = torch.from_numpy(np.ascontiguousarray(g["f3"][:B].T)).cuda()   # [steps, B]
    T = g["f3"].shape[1]
    fest = np.zeros((B, T), np.float32)
    flag = np.zeros((B, T), bool)
    fest_dev = torch.empty((T, B), dtype=torch.float32, device="cuda")
    flag_dev = torch.empty((T, B), dtype=torch.int32, device="cuda")
    for k in range(T):
        s.estimate(est, recs, fext3=f3[k], sim_time=float(g["t"][k]))
        fest_dev[k] = recs[:, 29]
        flag_dev[k] = recs[:, 30].view(torch.int32)
    torch.cuda.synchronize()
    fest[:] = fest_dev.cpu().numpy().T
    flag[:] = flag_dev.cpu().numpy().T != 0
    return recs, est, fest, flag


def test_estimator_sequence_matches_oracle(cm, solver_mod, on_stream):
    import torch
    g = load_golden("n20_config5")
    prm = golden_params(cm, g)
    B = g["records"].shape[0]
    s = solver_mod.BatchSolver(prm, max_batch=B, stream=on_stream)
    recs, est, fest, flag = _run_sequence(torch, s, g, B)
    s.close()
    np.testing.assert_array_equal(flag, g["flag_ref"])
    ref = g["fest_ref"]
    assert ((fest == 0) == (ref == 0)).all()           # compensation starts at 400 samples
    err = np.abs(fest - ref) / np.maximum(np.abs(ref), 1.0)
    assert err.max() <= 1e-5, err.max()
    # the device state holds the same frozen sine-fit parameters as the oracle would
    prm_dev = est.cpu().numpy()[:, 804:812].copy().view(np.float64)
    assert np.all(np.abs(prm_dev[:, 2] - 0.33) < 1 / (400 * 0.026))  # est_freq near 0.33 Hz


def test_config5_pipeline_forces_match_reference(cm, solver_mod, on_stream):
    """estimate (520 steps) -> solve at N = 20 with f_est in qg, against qpOASES."""
    import torch
    g = load_golden("n20_config5")
    prm = golden_params(cm, g)
    B = g["records"].shape[0]
    s = solver_mod.BatchSolver(prm, max_batch=B, stream=on_stream)
    recs, est, fest, flag = _run_sequence(torch, s, g, B)
    forces = torch.empty((B, 12 * prm.horizon), dtype=torch.float32, device="cuda")
    status = torch.empty(B, dtype=torch.uint8, device="cuda")
    s.solve(recs, forces, status)
    torch.cuda.synchronize()
    s.close()
    assert (status.cpu().numpy() == 0).all()
    err = rel_force_err(forces.cpu().numpy(), g["q_ref"])
    assert err.max() <= 1e-4, (err.max(), int(err.argmax()))


def test_device_residual_matches_oracle(cm, solver_mod, on_stream):
    import torch
    g = load_golden("n20_config5")
    prm = golden_params(cm, g)
    B = g["records"].shape[0]
    s = solver_mod.BatchSolver(prm, max_batch=B, stream=on_stream)
    recs = torch.from_numpy(np.ascontiguousarray(g["records"])).cuda()
    logs = torch.from_numpy(np.ascontiguousarray(g["logs"])).cuda()
    est = torch.zeros((B, 816), dtype=torch.float32, device="cuda")
    fext6 = torch.empty((B, 6), dtype=torch.float32, device="cuda")
    s.estimate(est, recs, logs=logs, sim_time=1.0, fext6=fext6)
    torch.cuda.synchronize()
    s.close()
    ref = g["fext6_ref"]
    got = fext6.cpu().numpy()
    # fp32 throughout; the torque rows cancel terms ~100x their result, and the summation order
    # of the 3x3 / 13x12 products differs (Eigen's is not fixed either): absolute tolerance
    # relative to the largest component
    np.testing.assert_allclose(got, ref, rtol=1e-5, atol=2e-6 * np.abs(ref).max())
    # the pushed sample is f_ext[3]
    assert np.array_equal(est.cpu().numpy()[:, 0], got[:, 3])
