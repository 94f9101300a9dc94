"""Host-side mirror of the reference's SolverMPC interface over the C ABI of libcmpc_hip.so.

Two surfaces (see include/cmpc_solver.h):

* the reference's single-instance functions, same names and argument meaning as
  ``convexMPC_interface.h:44-52`` (``setup_problem``, ``update_solver_settings``,
  ``update_x_drag``, ``update_problem_data_floats``, ``update_problem_data``,
  ``get_solution``), so parity tests read like the reference's call protocol
  (``ConvexMPCLocomotion.cpp:807-836``);
* :class:`BatchSolver`, the reentrant batched API over device buffers (torch tensors on
  ``cuda:*`` or raw pointers) — the hot path.

There is no CPU fallback: if ``libcmpc_hip.so`` is missing or no GPU is present, calls fail.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .records import CmpcParams, LocoParams, make_params, record_words

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CMPC_LIB", os.path.join(PKG, "libcmpc_hip.so"))

# every symbol include/cmpc_solver.h declares (C linkage unless noted)
EXPORTED_SYMBOLS = (
    "setup_problem", "update_problem_data", "get_solution", "update_solver_settings",
    "update_problem_data_floats", "_Z13update_x_dragf", "f_ext", "simulation_time",
    "f_est", "f_est_smoothed", "f_est_static",
    "cmpc_record_words", "cmpc_batch_create", "cmpc_batch_set_params", "cmpc_batch_destroy",
    "cmpc_batch_solve", "cmpc_batch_solve_host", "cmpc_batch_set_output_steps", "cmpc_batch_set_refine",
    "cmpc_batch_condense",
    "cmpc_batch_stream",
    "cmpc_last_error", "cmpc_batch_enable_timing", "cmpc_batch_enable_timing_every", "cmpc_batch_read_timing", "cmpc_batch_estimate",
    "cmpc_batch_assemble", "cmpc_batch_rollout", "cmpc_batch_admm", "cmpc_batch_expand",
    "cmpc_batch_quadprog",   # include/cmpc_quadprog.h
)

_lib = None
_fp = ctypes.POINTER(ctypes.c_float)
_dp = ctypes.POINTER(ctypes.c_double)
_ip = ctypes.POINTER(ctypes.c_int)
_u8p = ctypes.POINTER(ctypes.c_uint8)


class CmpcError(RuntimeError):
    pass


class AdmmSettings(ctypes.Structure):
    """cmpc_admm_settings (include/cmpc_solver.h); defaults = ros_config.yaml:73-77."""
    _fields_ = [("max_iter", ctypes.c_int), ("rho", ctypes.c_double), ("sigma", ctypes.c_double),
                ("alpha", ctypes.c_double), ("terminate", ctypes.c_double),
                ("reduced", ctypes.c_int)]


def admm_settings(max_iter: int = 10000, rho: float = 1e-7, sigma: float = 1e-8,
                  alpha: float = 1.5, terminate: float = 0.1, reduced: bool = False) -> AdmmSettings:
    return AdmmSettings(int(max_iter), float(rho), float(sigma), float(alpha), float(terminate),
                        int(bool(reduced)))


def load_library(path: str = LIB_PATH):
    """Load libcmpc_hip.so (fails loudly if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise CmpcError(f"{path} not built: run __graft_entry__.build() "
                        f"(or python quad-periodic-mpc_amd/build.py)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    lib.setup_problem.argtypes = [ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_double]
    lib.update_problem_data.argtypes = [_dp, _dp, _dp, _dp, _dp, ctypes.c_double, _dp, _dp,
                                        ctypes.c_double, _ip]
    lib.get_solution.argtypes = [ctypes.c_int]
    lib.get_solution.restype = ctypes.c_double
    lib.update_solver_settings.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_double, ctypes.c_double]
    lib.update_problem_data_floats.argtypes = [_fp, _fp, _fp, _fp, _fp, ctypes.c_float,
                                               ctypes.c_float, ctypes.c_float, _fp, _fp,
                                               ctypes.c_float, _ip]
    lib._Z13update_x_dragf.argtypes = [ctypes.c_float]
    lib.cmpc_record_words.argtypes = [ctypes.c_int]
    lib.cmpc_batch_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(CmpcParams),
                                      ctypes.c_int, ctypes.c_void_p]
    lib.cmpc_batch_set_params.argtypes = [ctypes.c_void_p, ctypes.POINTER(CmpcParams)]
    lib.cmpc_batch_destroy.argtypes = [ctypes.c_void_p]
    lib.cmpc_batch_destroy.restype = None
    lib.cmpc_batch_solve.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.cmpc_batch_solve_host.argtypes = [ctypes.c_void_p, _fp, ctypes.c_int, _fp, _u8p, _ip]
    lib.cmpc_batch_set_output_steps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if hasattr(lib, "cmpc_batch_set_refine"):  # (older A/B variant libraries lack it)
        lib.cmpc_batch_set_refine.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.cmpc_batch_condense.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.c_void_p, ctypes.c_void_p]
    lib.cmpc_batch_admm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(AdmmSettings),
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.cmpc_batch_stream.argtypes = [ctypes.c_void_p]
    lib.cmpc_batch_expand.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.cmpc_batch_stream.restype = ctypes.c_void_p
    lib.cmpc_last_error.restype = ctypes.c_char_p
    lib.cmpc_batch_enable_timing.argtypes = [ctypes.c_void_p, ctypes.c_int]
    if hasattr(lib, "cmpc_batch_enable_timing_every"):  # (A/B libraries built before round 4 lack it)
        lib.cmpc_batch_enable_timing_every.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    lib.cmpc_batch_read_timing.argtypes = [ctypes.c_void_p, _fp, _ip, _ip]
    lib.cmpc_batch_estimate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                        ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.cmpc_batch_assemble.argtypes = [ctypes.c_void_p, ctypes.c_void_p,
                                        ctypes.POINTER(LocoParams), ctypes.c_void_p,
                                        ctypes.c_void_p, ctypes.c_int]
    lib.cmpc_batch_rollout.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_int]
    lib.cmpc_batch_quadprog.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int] + \
        [ctypes.c_void_p] * 7 + [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int]
    _lib = lib
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().cmpc_last_error().decode(errors="replace")
        raise CmpcError(f"{what} failed ({rc}): {msg}")


# ---------------------------------------------------------------------------------------------
# Reference single-instance interface (convexMPC_interface.h:44-52)
# ---------------------------------------------------------------------------------------------
def _f32(a, n=None):
    a = np.ascontiguousarray(a, np.float32)
    if n is not None and a.size < n:
        raise ValueError(f"expected >= {n} floats, got {a.size}")
    return a


def setup_problem(dt: float, horizon: int, mu: float, f_max: float) -> None:
    load_library().setup_problem(dt, horizon, mu, f_max)


def update_solver_settings(max_iter, rho, sigma, solver_alpha, terminate, use_jcqp) -> None:
    load_library().update_solver_settings(int(max_iter), rho, sigma, solver_alpha, terminate, use_jcqp)


def update_x_drag(x_drag: float) -> None:
    load_library()._Z13update_x_dragf(float(x_drag))


def update_problem_data_floats(p, v, q, w, r, roll, pitch, yaw, weights, state_trajectory, alpha,
                               gait) -> None:
    arrs = [_f32(p, 3), _f32(v, 3), _f32(q, 4), _f32(w, 3), _f32(r, 12)]
    wts = _f32(weights, 12)
    traj = _f32(state_trajectory)
    g = np.ascontiguousarray(gait, np.int32)
    load_library().update_problem_data_floats(
        *[a.ctypes.data_as(_fp) for a in arrs], float(roll), float(pitch), float(yaw),
        wts.ctypes.data_as(_fp), traj.ctypes.data_as(_fp), float(alpha), g.ctypes.data_as(_ip))


def update_problem_data(p, v, q, w, r, yaw, weights, state_trajectory, alpha, gait) -> None:
    arrs = [np.ascontiguousarray(a, np.float64) for a in (p, v, q, w, r)]
    wts = np.ascontiguousarray(weights, np.float64)
    traj = np.ascontiguousarray(state_trajectory, np.float64)
    g = np.ascontiguousarray(gait, np.int32)
    load_library().update_problem_data(
        *[a.ctypes.data_as(_dp) for a in arrs], float(yaw), wts.ctypes.data_as(_dp),
        traj.ctypes.data_as(_dp), float(alpha), g.ctypes.data_as(_ip))


def get_solution(index: int) -> float:
    return load_library().get_solution(int(index))


def set_f_ext(values) -> None:
    """Write the caller-owned global ``f_ext`` (ConvexMPCLocomotion.cpp:610)."""
    arr = (ctypes.c_float * 6).in_dll(load_library(), "f_ext")
    for i, x in enumerate(values):
        arr[i] = float(x)


def set_simulation_time(t: float) -> None:
    ctypes.c_float.in_dll(load_library(), "simulation_time").value = float(t)


def get_f_est(name: str = "f_est") -> np.ndarray:
    """The solver's estimator globals (SolverMPC.h:72-74): ``f_est``, ``f_est_smoothed`` or
    ``f_est_static`` after the last update_problem_data* call."""
    if name not in ("f_est", "f_est_smoothed", "f_est_static"):
        raise ValueError(name)
    return np.array((ctypes.c_float * 6).in_dll(load_library(), name)[:], np.float32)


# ---------------------------------------------------------------------------------------------
# Batched API
# ---------------------------------------------------------------------------------------------
def _ptr(t) -> int:
    if t is None:
        return 0
    if hasattr(t, "data_ptr"):
        if not t.is_cuda:
            raise CmpcError("BatchSolver.solve expects device tensors")
        return t.data_ptr()
    return int(t)


class BatchSolver:
    """Reentrant batched solver bound to one HIP stream (``cmpc_batch_*``)."""

    def __init__(self, params: CmpcParams | None = None, max_batch: int = 65536, stream=None,
                 horizon: int = 10):
        self.lib = load_library()
        self.params = params if params is not None else make_params(horizon)
        self.max_batch = int(max_batch)
        h = ctypes.c_void_p()
        s = None
        if stream is not None:
            handle = stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)
            if not handle:
                # NULL would make the library create a private stream, unordered with the
                # caller's default-stream work: refuse instead of silently racing
                raise CmpcError("BatchSolver(stream=...) needs a non-default stream "
                                "(e.g. torch.cuda.Stream()); pass None for a private stream")
            s = ctypes.c_void_p(handle)
        _check(self.lib.cmpc_batch_create(ctypes.byref(h), ctypes.byref(self.params),
                                          self.max_batch, s), "cmpc_batch_create")
        self._h = h

    @property
    def horizon(self) -> int:
        return self.params.horizon

    @property
    def out_cols(self) -> int:
        """Forces kept per instance (12 x the output steps, 12 N by default)."""
        steps = getattr(self, "_out_steps", 0)
        return 12 * (steps if 0 < steps < self.horizon else self.horizon)

    def set_output_steps(self, steps: int) -> None:
        """Keep the forces of the first ``steps`` horizon steps only (0: every step);
        ``cmpc_batch_set_output_steps``: the forces' stride becomes 12 x steps."""
        _check(self.lib.cmpc_batch_set_output_steps(self._h, int(steps)), "set_output_steps")
        self._out_steps = int(steps)

    def set_refine(self, on: bool) -> None:
        """The wide classes' fp64 refinement (``cmpc_batch_set_refine``): on from N = 11 by
        default; off solves every horizon in fp32 only."""
        _check(self.lib.cmpc_batch_set_refine(self._h, 1 if on else 0), "set_refine")

    @property
    def record_words(self) -> int:
        return record_words(self.params.horizon)

    @property
    def stream_handle(self) -> int:
        return self.lib.cmpc_batch_stream(self._h)

    def set_params(self, params: CmpcParams) -> None:
        _check(self.lib.cmpc_batch_set_params(self._h, ctypes.byref(params)), "set_params")
        self.params = params

    def solve(self, records, forces, status, iters=None, batch: int | None = None) -> None:
        """Asynchronous device solve on the handle's stream (torch tensors or raw pointers)."""
        if batch is None:
            batch = records.shape[0]
        if batch > self.max_batch:
            raise CmpcError(f"batch {batch} > max_batch {self.max_batch}")
        if hasattr(records, "shape"):
            assert records.shape[-1] == self.record_words, "record stride mismatch"
            assert forces.numel() >= batch * self.out_cols and status.numel() >= batch
        _check(self.lib.cmpc_batch_solve(self._h, _ptr(records), int(batch), _ptr(forces),
                                         _ptr(status), _ptr(iters)), "cmpc_batch_solve")

    def solve_host(self, records: np.ndarray):
        """Host arrays in/out (H2D + solve + D2H, synchronous) -> (forces, status, iters)."""
        records = np.ascontiguousarray(records, np.float32)
        B = records.shape[0]
        assert records.shape[1] == self.record_words
        forces = np.zeros((B, self.out_cols), np.float32)
        status = np.zeros(B, np.uint8)
        iters = np.zeros(B, np.int32)
        _check(self.lib.cmpc_batch_solve_host(self._h, records.ctypes.data_as(_fp), B,
                                              forces.ctypes.data_as(_fp),
                                              status.ctypes.data_as(_u8p),
                                              iters.ctypes.data_as(_ip)), "cmpc_batch_solve_host")
        return forces, status, iters

    def condense(self, records, H, g, batch: int | None = None) -> None:
        """Full (no elimination) qH [B,12N,12N] / qg [B,12N] on device — parity hook."""
        if batch is None:
            batch = records.shape[0]
        _check(self.lib.cmpc_batch_condense(self._h, _ptr(records), int(batch), _ptr(H), _ptr(g)),
               "cmpc_batch_condense")

    def admm(self, records, H, g, forces, status, iters=None, settings: AdmmSettings | None = None,
             batch: int | None = None) -> None:
        """use_jcqp == 1 on device (``cmpc_batch_admm``): JCQP's ADMM over the full QP whose
        ``H`` / ``g`` came from :meth:`condense`."""
        if batch is None:
            batch = records.shape[0]
        s = settings if settings is not None else admm_settings()
        _check(self.lib.cmpc_batch_admm(self._h, _ptr(records), _ptr(H), _ptr(g), int(batch),
                                        ctypes.byref(s), _ptr(forces), _ptr(status), _ptr(iters)),
               "cmpc_batch_admm")

    def estimate(self, est_state, records, *, logs=None, fext3=None, times=None,
                 sim_time: float = 0.0, fext6=None, batch: int | None = None) -> None:
        """Config-5 estimator step on device (``cmpc_batch_estimate``): updates ``est_state``
        [B, EST_WORDS] and writes f_est(3) / the use-f_est flag into ``records``. Pass either
        ``logs`` [B, LOG_WORDS] (residual computed on device) or ``fext3`` [B]."""
        if batch is None:
            batch = records.shape[0]
        if logs is None and fext3 is None:
            raise CmpcError("estimate needs logs or fext3")
        _check(self.lib.cmpc_batch_estimate(self._h, _ptr(est_state), _ptr(logs), _ptr(fext3),
                                            _ptr(times), float(sim_time), _ptr(records),
                                            _ptr(fext6), int(batch)), "cmpc_batch_estimate")

    def assemble(self, loco, loco_params: LocoParams, records, due, batch: int | None = None) -> None:
        """One control tick of every instance's locomotion controller on device
        (``cmpc_batch_assemble``): updates ``loco`` [B, LOCO_WORDS] and, where an MPC step is
        due, writes that instance's solve record into ``records`` and ``due[i] = 1``."""
        if batch is None:
            batch = loco.shape[0]
        if hasattr(records, "shape"):
            assert records.shape[-1] == self.record_words, "record stride mismatch"
        _check(self.lib.cmpc_batch_assemble(self._h, _ptr(loco), ctypes.byref(loco_params),
                                            _ptr(records), _ptr(due), int(batch)),
               "cmpc_batch_assemble")

    def expand(self, compact, records, batch: int | None = None) -> None:
        """Compact records [B, CMPC_CREC_WORDS(N)] -> solve records [B, record_words] on device
        (``cmpc_batch_expand``: trajAll from its step-0 row, ConvexMPCLocomotion.cpp:554-585)."""
        if batch is None:
            batch = compact.shape[0]
        if hasattr(records, "shape"):
            assert records.shape[-1] == self.record_words, "record stride mismatch"
        _check(self.lib.cmpc_batch_expand(self._h, _ptr(compact), _ptr(records), int(batch)),
               "cmpc_batch_expand")

    def rollout(self, loco, records, forces, xi6=None, due=None, batch: int | None = None) -> None:
        """One single-rigid-body MPC step of every due instance on device
        (``cmpc_batch_rollout``): x+ = Adt x0 + Bdt u0 (+ Qdt xi) into ``loco``."""
        if batch is None:
            batch = loco.shape[0]
        _check(self.lib.cmpc_batch_rollout(self._h, _ptr(loco), _ptr(records), _ptr(forces),
                                           _ptr(xi6), _ptr(due), int(batch)), "cmpc_batch_rollout")

    def quadprog(self, G, g0, CE, ce0, CI, ci0, x, f, status, iters=None, dims=None,
                 max_iter: int = 1000, batch: int | None = None) -> None:
        """Batched QuadProg++ ``solve_quadprog`` on device (``cmpc_batch_quadprog``,
        include/cmpc_quadprog.h): fp64 blocks G [B,n,n], g0 [B,n], CE [B,n,p], ce0 [B,p],
        CI [B,n,m], ci0 [B,m]; optional per-instance ``dims`` [B,3] int32 (n, p, m)."""
        if batch is None:
            batch = G.shape[0]
        batch = int(batch)
        n, p, m = int(G.shape[-1]), int(ce0.shape[-1]), int(ci0.shape[-1])
        # (the QuadProg++ kernel keeps its state in LDS: batch is not bounded by max_batch)
        # the kernel reads / writes these blocks through raw pointers: check dtype, layout and
        # that every buffer holds `batch` instances before handing them over
        import torch
        shapes = {"G": (G, (n, n), torch.float64), "g0": (g0, (n,), torch.float64),
                  "CE": (CE, (n, p), torch.float64), "ce0": (ce0, (p,), torch.float64),
                  "CI": (CI, (n, m), torch.float64), "ci0": (ci0, (m,), torch.float64),
                  "x": (x, (n,), torch.float64), "f": (f, (), torch.float64),
                  "status": (status, (), torch.uint8)}
        if iters is not None:
            shapes["iters"] = (iters, (), torch.int32)
        if dims is not None:
            shapes["dims"] = (dims, (3,), torch.int32)
        for name, (t, tail, dt) in shapes.items():
            if t.dtype != dt:
                raise CmpcError(f"quadprog: {name} must be {dt}, got {t.dtype}")
            if not t.is_contiguous():
                raise CmpcError(f"quadprog: {name} must be contiguous")
            if t.dim() != 1 + len(tail) or tuple(t.shape[1:]) != tail or t.shape[0] < batch:
                raise CmpcError(f"quadprog: {name} has shape {tuple(t.shape)}, expected "
                                f"[>= {batch}, {', '.join(map(str, tail))}]")
        _check(self.lib.cmpc_batch_quadprog(self._h, n, p, m, _ptr(dims), _ptr(G), _ptr(g0),
                                            _ptr(CE), _ptr(ce0), _ptr(CI), _ptr(ci0), int(max_iter),
                                            _ptr(x), _ptr(f), _ptr(status), _ptr(iters), int(batch)),
               "cmpc_batch_quadprog")

    def enable_timing(self, steps: int, every: int = 1) -> None:
        """Record HIP events around each size-class launch of the next ``steps`` solves (of every
        ``every``-th solve only, ``steps`` of them, when ``every`` > 1)."""
        self._timing_steps = int(steps)
        if not hasattr(self.lib, "cmpc_batch_enable_timing_every"):
            if every != 1:
                raise CmpcError("this libcmpc_hip.so has no cmpc_batch_enable_timing_every")
            _check(self.lib.cmpc_batch_enable_timing(self._h, int(steps)), "enable_timing")
            return
        _check(self.lib.cmpc_batch_enable_timing_every(self._h, int(steps), int(every)), "enable_timing")

    def read_timing(self):
        """-> (ms [steps, 2] per class launch, class-1 overflow count of the last solve)."""
        n = getattr(self, "_timing_steps", 0)
        ms = np.zeros(2 * max(n, 1), np.float32)
        rec = ctypes.c_int(0)
        ovf = ctypes.c_int(0)
        _check(self.lib.cmpc_batch_read_timing(self._h, ms.ctypes.data_as(_fp), ctypes.byref(rec),
                                               ctypes.byref(ovf)), "read_timing")
        return ms[:2 * rec.value].reshape(rec.value, 2), ovf.value

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.lib.cmpc_batch_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
