"""CPU tests of the host-side logic: record layout, generator, C-ABI library exports."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def test_record_layout_matches_header(cm):
    hdr = open(os.path.join(ROOT, "include", "cmpc_solver.h")).read()
    consts = dict(re.findall(r"#define (CMPC_REC_[A-Z0-9]+)\s+(\d+)", hdr))
    r = cm.records
    assert int(consts["CMPC_REC_P"]) == r.REC_P
    assert int(consts["CMPC_REC_V"]) == r.REC_V
    assert int(consts["CMPC_REC_Q"]) == r.REC_Q
    assert int(consts["CMPC_REC_W"]) == r.REC_W
    assert int(consts["CMPC_REC_R"]) == r.REC_R
    assert int(consts["CMPC_REC_XDRAG"]) == r.REC_XDRAG
    assert int(consts["CMPC_REC_FEST3"]) == r.REC_FEST3
    assert int(consts["CMPC_REC_FLAGS"]) == r.REC_FLAGS
    assert int(consts["CMPC_REC_HDR"]) == r.REC_HDR
    for N in range(1, 25):
        assert r.record_words(N) % 4 == 0 and r.record_words(N) >= 32 + 13 * N


def test_pack_roundtrip(cm):
    recs = cm.make_instances(8, 10, seed=3)
    gait = cm.unpack_gait(recs, 10)
    assert gait.shape == (8, 40) and set(np.unique(gait)) <= {0, 1}
    again = cm.pack_records(recs[:, 0:3], recs[:, 3:6], recs[:, 6:10], recs[:, 10:13],
                            recs[:, 13:25], recs[:, 32:152], gait, rpy=recs[:, 25:28],
                            x_drag=recs[:, 28])
    np.testing.assert_array_equal(again, recs)


def test_generator_deterministic_and_shaped(cm):
    a = cm.make_instances(64, 10, seed=42)
    b = cm.make_instances(64, 10, seed=42)
    np.testing.assert_array_equal(a, b)
    q = a[:, 6:10]
    np.testing.assert_allclose(np.linalg.norm(q, axis=1), 1.0, atol=1e-6)
    assert not np.array_equal(a, cm.make_instances(64, 10, seed=43))


def test_philox_known_answer(cm):
    """Philox4x32-10 of the per-instance generator against the Random123 known-answer vectors
    (counter 0, key 0 and counter/key all ones)."""
    import importlib
    ins = importlib.import_module("quad-periodic-mpc_amd.instances")
    out = ins.philox4x32(np.array([0]), np.array([0]), 1)[0]
    assert [int(x) for x in out] == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]


def test_trot_table_matches_gait_rule(cm):
    """OffsetDurationGait::getMpcTable (Gait.cpp:159-188), trot P=18."""
    it = np.arange(18)
    tab = cm.trot_table(10, it).reshape(18, 10, 4)
    for i0 in range(18):
        for i in range(10):
            row = (i + i0 + 1) % 18
            exp = [(row - o) % 18 < 9 for o in (0, 9, 9, 0)]
            assert list(tab[i0, i].astype(bool)) == exp
    assert (tab.sum(-1) == 2).all()  # trot: two legs in stance at every step


def test_library_exports_header_symbols(cm):
    from importlib import import_module
    solver = import_module("quad-periodic-mpc_amd.solver")
    path = solver.LIB_PATH
    if not os.path.exists(path):
        pytest.skip("libcmpc_hip.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True,
                         check=True).stdout
    names = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for sym in solver.EXPORTED_SYMBOLS:
        assert sym in names, sym
    # every prototype of a header is among the exports of its library (cmpc_multi.h:
    # libcmpc_multi.so, the RCCL sharding; every other header: libcmpc_hip.so)
    multi = os.path.join(os.path.dirname(path), "libcmpc_multi.so")
    libs = {path: names}
    if os.path.exists(multi):
        mout = subprocess.run(["nm", "-D", "--defined-only", multi], capture_output=True, text=True,
                              check=True).stdout
        libs[multi] = {line.split()[-1] for line in mout.splitlines() if line.strip()}
    seen = []
    for h in sorted(os.listdir(os.path.join(ROOT, "include"))):
        if not h.endswith(".h"):
            continue
        protos = re.findall(r"CMPC_EXTERNC\s+[\w\s\*]+?\b(\w+)\s*\(", open(os.path.join(ROOT, "include", h)).read())
        seen += protos
        target = multi if h == "cmpc_multi.h" else path
        if target not in libs:
            pytest.fail(f"{target} not built")
        for p in protos:
            assert p in libs[target], (h, p)
    assert "cmpc_batch_quadprog" in seen and "cmpc_multi_solve" in seen
    lib = ctypes.CDLL(path)  # loads without a GPU
    lib.cmpc_record_words.argtypes = [ctypes.c_int]
    assert lib.cmpc_record_words(10) == cm.record_words(10)
    ml = ctypes.CDLL(multi)  # loads without a GPU (librccl resolved, nothing initialised)
    ml.cmpc_multi_root_share.argtypes = [ctypes.c_int] * 3
    ml.cmpc_multi_root_share.restype = ctypes.c_float
    assert abs(ml.cmpc_multi_root_share(656, 481, 1) - (1 + 1137 / 3213.0)) < 1e-6


def test_gait_tables_match_offset_duration_rule(cm):
    """The controller's other OffsetDurationGaits (ConvexMPCLocomotion.cpp:41-51) through the
    generator: standing puts every foot in stance, walking follows (row - offset) mod P <
    duration (Gait.cpp:159-188)."""
    from importlib import import_module
    inst = import_module("quad-periodic-mpc_amd.instances")
    tabs = inst.loco_gaits(18)
    it = np.arange(18)
    for name in ("standing", "walking", "bounding", "galloping"):
        off, dur, _ = tabs[name]
        tab = inst.gait_table(10, it, off, dur, 18).reshape(18, 10, 4)
        for i0 in range(18):
            for i in range(10):
                row = (i + i0 + 1) % 18
                assert list(tab[i0, i].astype(bool)) == [(row - o) % 18 < d for o, d in zip(off, dur)]
    recs = cm.make_instances(64, 16, random_contact_frac=0.0, gait="standing")
    assert (cm.unpack_gait(recs, 16) == 1).all()
    recs = cm.make_instances(64, 16, random_contact_frac=0.0, gait="walking")
    n = 3 * (cm.unpack_gait(recs, 16) != 0).sum(1)
    assert set(np.unique(n)) <= {138, 141}


def test_horizon_beyond_max_is_rejected(cm):
    """CMPC_MAX_HORIZON = 20 (the reference's 19, lifted by one for config 5): longer horizons
    are refused by the host mirror and by the library (before any HIP call)."""
    from importlib import import_module
    solver = import_module("quad-periodic-mpc_amd.solver")
    with pytest.raises(ValueError):
        cm.make_params(21)
    if not os.path.exists(solver.LIB_PATH):
        pytest.skip("libcmpc_hip.so not built")
    lib = solver.load_library()
    prm = cm.make_params(20)
    prm.horizon = 21
    h = ctypes.c_void_p()
    assert lib.cmpc_batch_create(ctypes.byref(h), ctypes.byref(prm), 16, None) == -2
    assert b"horizon" in lib.cmpc_last_error()


_ABI_REFUSAL_CHILD = r"""
import ctypes, sys
import numpy as np
lib = ctypes.CDLL(sys.argv[1])
fp = ctypes.POINTER(ctypes.c_float); dp = ctypes.POINTER(ctypes.c_double); ip = ctypes.POINTER(ctypes.c_int)
lib.setup_problem.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double]
lib.update_problem_data_floats.argtypes = [fp] * 5 + [ctypes.c_float] * 3 + [fp, fp, ctypes.c_float, ip]
lib.update_problem_data.argtypes = [dp] * 5 + [ctypes.c_double, dp, dp, ctypes.c_double, ip]
lib.get_solution.argtypes = [ctypes.c_int]; lib.get_solution.restype = ctypes.c_double
for N in (0, -3, 21, 22, 24, 64):
    M = max(N, 1)
    f = [np.ones(k, np.float32) for k in (3, 3, 4, 3, 12, 12, 12 * M)]
    d = [np.ones(k, np.float64) for k in (3, 3, 4, 3, 12, 12, 12 * M)]
    gait = np.ones(4 * M, np.int32)
    lib.setup_problem(0.026, N, 0.4, 120.0)
    lib.update_problem_data_floats(*[a.ctypes.data_as(fp) for a in f[:5]], 0.0, 0.0, 0.0,
                                   f[5].ctypes.data_as(fp), f[6].ctypes.data_as(fp), 4e-5,
                                   gait.ctypes.data_as(ip))
    lib.update_problem_data(*[a.ctypes.data_as(dp) for a in d[:5]], 0.0, d[5].ctypes.data_as(dp),
                            d[6].ctypes.data_as(dp), 4e-5, gait.ctypes.data_as(ip))
    assert all(lib.get_solution(j) == 0.0 for j in (-1, 0, 12 * M - 1, 10 ** 6))
print("ok")
"""


def test_reference_abi_refuses_bad_horizon_without_gpu(cm):
    """setup_problem with a horizon outside 1..CMPC_MAX_HORIZON: both update_problem_data entry
    points print an error and return before any copy of the caller's 12N / 4N arrays or any HIP
    call (so this runs without a GPU), and get_solution stays 0 (nothing solved yet; an index
    outside the last solution also reads 0). The GPU-side counterpart, which checks that a
    previous solution is kept, is tests/test_gpu_parity.py::test_reference_abi_rejects_horizon_beyond_max."""
    from importlib import import_module
    solver = import_module("quad-periodic-mpc_amd.solver")
    if not os.path.exists(solver.LIB_PATH):
        pytest.skip("libcmpc_hip.so not built")
    import sys
    r = subprocess.run([sys.executable, "-c", _ABI_REFUSAL_CHILD, solver.LIB_PATH],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (r.returncode, r.stdout, r.stderr)
    assert r.stderr.count("previous solution kept") == 12, r.stderr
