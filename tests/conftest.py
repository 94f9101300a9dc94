import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


# One line per parity check (tests/test_gpu_parity.py assert_parity / assert_failed_reference):
# printed as a terminal-summary section, so a quiet run (-q, output captured) still shows how often
# each case took the fp64-optimum branch and against which cap.
PARITY_LEDGER = []


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if PARITY_LEDGER:
        terminalreporter.section("parity ledger: instances beyond 1e-4 of qpOASES per case")
        for line in PARITY_LEDGER:
            terminalreporter.write_line(line)


@pytest.fixture(scope="session")
def cm():
    return importlib.import_module("quad-periodic-mpc_amd")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False)
    return {k: d[k] for k in d.files}


def golden_params(cm, g):
    return cm.make_params(int(g["horizon"]), dt=float(g["dt"]), mu=float(g["mu"]),
                          f_max=float(g["f_max"]), weights=tuple(float(x) for x in g["weights"]),
                          alpha=float(g["alpha"]))


GOLDEN_SETS = ["n10_mixed", "n10_stress", "n10_edge", "n16_trot", "n19_mixed", "n20_trot",
               "n20_mixed", "n12_allstance", "n16_standing", "n20_standing", "n16_walking",
               "n20_walking"]


def rel_force_err(f, f_ref):
    """Norm-wise force error per instance: |f - f_ref|_inf / max(|f_ref|_inf, 1 N)."""
    f = np.asarray(f, np.float64).reshape(f_ref.shape[0], -1)
    f_ref = np.asarray(f_ref, np.float64).reshape(f_ref.shape[0], -1)
    return np.abs(f - f_ref).max(axis=1) / np.maximum(np.abs(f_ref).max(axis=1), 1.0)
