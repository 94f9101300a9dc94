"""Instance-record layout shared by the HIP solver, the C ABI and the oracle.

One record holds one ``solve_mpc`` call's per-instance data (reference:
``be2r_cmpc_unitree/src/controllers/convexMPC/SolverMPC.cpp:566-655``, the fields of
``update_data_t`` in ``convexMPC_interface.h:23-41``). The word offsets mirror the ``CMPC_REC_*``
macros of ``include/cmpc_solver.h``; keep the two in sync.
"""
from __future__ import annotations

import ctypes

import numpy as np

REC_P = 0        # p[3]
REC_V = 3        # v[3]
REC_Q = 6        # q[4] (w, x, y, z)
REC_W = 10       # omega[3]
REC_R = 13       # r[12] axis-major 3x4: r[axis * 4 + leg]
REC_RPY = 25     # roll, pitch, yaw (stored; the solve recomputes rpy from q)
REC_XDRAG = 28   # x_drag
REC_FEST3 = 29   # f_est(3) compensation force (config 5)
REC_FLAGS = 30   # uint32 bit-cast; bit 0: use f_est in qg
REC_HDR = 32
MAX_HORIZON = 20
# config 5 (include/cmpc_solver.h CMPC_LOG_* / CMPC_EST_*)
LOG_POS, LOG_EUL, LOG_ANG, LOG_LIN, LOG_FORCE, LOG_XDRAG, LOG_R, LOG_ROT = 0, 3, 6, 9, 12, 24, 25, 37
LOG_WORDS = 48
EST_WINDOW = 400
EST_STOP = 500
EST_F, EST_T, EST_COUNT, EST_HEAD, EST_FEST3, EST_PARAMS = 0, 400, 800, 801, 802, 804
EST_WORDS = 816

STATUS_NAMES = {0: "ok", 1: "max_iter", 2: "infeasible", 3: "not_pd", 4: "bad_input"}
# locomotion-controller state for batched input assembly (include/cmpc_solver.h CMPC_LOCO_*)
LOCO_POS, LOCO_ZGT, LOCO_Q, LOCO_RPY, LOCO_VW, LOCO_WW, LOCO_PFOOT = 0, 3, 4, 8, 11, 14, 17
LOCO_CMD, LOCO_HEIGHT, LOCO_VDES, LOCO_WPD, LOCO_RPYINT, LOCO_XCI = 29, 32, 33, 35, 37, 39
LOCO_COUNTER, LOCO_GAIT, LOCO_FLAGS, LOCO_STAND = 40, 41, 50, 51
LOCO_SWREM, LOCO_SWST, LOCO_P0, LOCO_PF, LOCO_PDES = 56, 60, 64, 76, 88
LOCO_WORDS = 104
LOCO_OMNI, LOCO_STANDING, LOCO_PRONK, LOCO_FIRST, LOCO_SIMFEET = 1, 2, 4, 8, 16
LOCO_FSWING0 = 256          # firstSwing[l] = bit 8 + l
LOCO_FSWING_ALL = 0xF00

# A1 geometry (MiniCheetah.h:30-37, Quadruped.h:95-102) and swing parameters (ros_config.yaml:62,70)
A1_HIP_X, A1_HIP_Y, A1_ABAD_LINK = 0.1805, 0.047, 0.0838
SWING_HEIGHT, BONUS_SWING = 0.17, 0.0


class LocoParams(ctypes.Structure):
    """cmpc_loco_params (include/cmpc_solver.h)."""
    _fields_ = [("dt", ctypes.c_float), ("iters_between_mpc", ctypes.c_int),
                ("x_drag_gain", ctypes.c_float), ("pad", ctypes.c_int),
                ("hip_x", ctypes.c_float), ("hip_y", ctypes.c_float),
                ("abad_link", ctypes.c_float), ("swing_height", ctypes.c_float),
                ("bonus_swing", ctypes.c_float), ("pad2", ctypes.c_float * 3)]


def make_loco_params(dt: float = 0.002, iters_between_mpc: int = 13, x_drag_gain: float = 0.0,
                     hip_x: float = A1_HIP_X, hip_y: float = A1_HIP_Y,
                     abad_link: float = A1_ABAD_LINK, swing_height: float = SWING_HEIGHT,
                     bonus_swing: float = BONUS_SWING) -> LocoParams:
    return LocoParams(dt, iters_between_mpc, x_drag_gain, 0, hip_x, hip_y, abad_link,
                      swing_height, bonus_swing)


def record_words(horizon: int) -> int:
    """fp32 words per record: header + traj[12N] + gait[4N] bytes, padded to 16 B."""
    return (REC_HDR + 13 * horizon + 3) & ~3


def traj_offset(horizon: int) -> int:
    return REC_HDR


def gait_offset(horizon: int) -> int:
    return REC_HDR + 12 * horizon


class CmpcParams(ctypes.Structure):
    """ctypes mirror of ``cmpc_params`` (include/cmpc_solver.h)."""

    _fields_ = [
        ("dt", ctypes.c_float),
        ("mu", ctypes.c_float),
        ("f_max", ctypes.c_float),
        ("horizon", ctypes.c_int),
        ("weights", ctypes.c_float * 12),
        ("alpha", ctypes.c_float),
        ("max_iter", ctypes.c_int),
    ]


# ConvexMPCLocomotion.cpp:617 (Q), :623 (alpha), :807 (mu = 0.4, f_max = 120); dtMPC = 0.002 * 13
DEFAULT_WEIGHTS = (0.25, 0.25, 10, 10, 2, 50, 0, 0, 0.3, 0.2, 0.2, 0.1)


def make_params(horizon: int = 10, dt: float = 0.026, mu: float = 0.4, f_max: float = 120.0,
                weights=DEFAULT_WEIGHTS, alpha: float = 4e-5, max_iter: int = 100) -> CmpcParams:
    if not 1 <= horizon <= MAX_HORIZON:
        raise ValueError(f"horizon {horizon} outside 1..{MAX_HORIZON}")
    prm = CmpcParams()
    prm.dt = dt
    prm.mu = mu
    prm.f_max = f_max
    prm.horizon = horizon
    for i, w in enumerate(weights):
        prm.weights[i] = w
    prm.alpha = alpha
    prm.max_iter = max_iter
    return prm


def pack_records(p, v, q, w, r, traj, gait, *, rpy=None, x_drag=None, f_est3=None,
                 use_f_est=None) -> np.ndarray:
    """Pack per-instance arrays (leading batch dim) into a [B, record_words(N)] fp32 array.

    ``r`` is axis-major [B, 12] (``r[axis*4 + leg]``, ConvexMPCLocomotion.cpp:786-790),
    ``traj`` [B, 12N] step-major, ``gait`` [B, 4N] integers cast to uint8 as
    ``convexMPC_interface.cpp:139`` does.
    """
    p = np.asarray(p, np.float32)
    B = p.shape[0]
    traj = np.asarray(traj, np.float32).reshape(B, -1)
    N = traj.shape[1] // 12
    gait = np.asarray(gait).reshape(B, 4 * N).astype(np.uint8)
    rec = np.zeros((B, record_words(N)), np.float32)
    rec[:, REC_P:REC_P + 3] = p
    rec[:, REC_V:REC_V + 3] = v
    rec[:, REC_Q:REC_Q + 4] = q
    rec[:, REC_W:REC_W + 3] = w
    rec[:, REC_R:REC_R + 12] = r
    if rpy is not None:
        rec[:, REC_RPY:REC_RPY + 3] = rpy
    if x_drag is not None:
        rec[:, REC_XDRAG] = x_drag
    if f_est3 is not None:
        rec[:, REC_FEST3] = f_est3
    if use_f_est is not None:
        rec[:, REC_FLAGS] = np.asarray(use_f_est, np.uint32).astype(np.uint32).view(np.float32)
    off = gait_offset(N)
    rec[:, REC_HDR:REC_HDR + 12 * N] = traj
    gbytes = rec[:, off:off + N].view(np.uint8)
    gbytes[:, :] = gait
    return rec


def unpack_gait(rec: np.ndarray, horizon: int) -> np.ndarray:
    off = gait_offset(horizon)
    return np.ascontiguousarray(rec[:, off:off + horizon]).view(np.uint8).reshape(rec.shape[0], 4 * horizon)


# ---- compact records (include/cmpc_solver.h CMPC_CREC_*, cmpc_batch_expand) -------------------
CREC_TRAJ0 = REC_HDR          # trajAll's step-0 row (12 words)
CREC_GAIT = REC_HDR + 12      # the gait words


def compact_words(horizon: int) -> int:
    """CMPC_CREC_WORDS(N): header + trajAll's step-0 row + gait words, 16-B aligned."""
    return (REC_HDR + 12 + horizon + 3) & ~3


def expand_records(crec: np.ndarray, horizon: int, dt: float) -> np.ndarray:
    """Host restatement of cmpc_batch_expand: trajAll per updateMPCIfNeeded
    (ConvexMPCLocomotion.cpp:554-585) from its step-0 row, fp32 product then fp32 sum."""
    N = horizon
    crec = np.ascontiguousarray(crec, np.float32)
    B = crec.shape[0]
    out = np.zeros((B, record_words(N)), np.float32)
    out[:, :REC_HDR] = crec[:, :REC_HDR]
    row0 = crec[:, CREC_TRAJ0:CREC_TRAJ0 + 12]
    traj = np.repeat(row0[:, None, :], N, axis=1)
    d = np.float32(dt) * row0[:, [8, 9, 10]]          # yaw rate, v_x, v_y
    for k in range(1, N):
        traj[:, k, [2, 3, 4]] = traj[:, k - 1, [2, 3, 4]] + d
    out[:, REC_HDR:REC_HDR + 12 * N] = traj.reshape(B, 12 * N)
    out[:, gait_offset(N):gait_offset(N) + N] = crec[:, CREC_GAIT:CREC_GAIT + N]
    return out


def compact_records(recs: np.ndarray, horizon: int, dt: float) -> np.ndarray:
    """Solve records -> compact records, for records whose trajAll has the form the controller
    builds (ConvexMPCLocomotion.cpp:554-585; instances.make_instances and cmpc_batch_assemble
    produce it). Raises ValueError when a record's trajectory is not that expansion of its step-0
    row, bit for bit (such records must be sent whole)."""
    N = horizon
    recs = np.ascontiguousarray(recs, np.float32)
    B = recs.shape[0]
    out = np.zeros((B, compact_words(N)), np.float32)
    out[:, :REC_HDR] = recs[:, :REC_HDR]
    out[:, CREC_TRAJ0:CREC_TRAJ0 + 12] = recs[:, REC_HDR:REC_HDR + 12]
    out[:, CREC_GAIT:CREC_GAIT + N] = recs[:, gait_offset(N):gait_offset(N) + N]
    back = expand_records(out, N, dt)
    bad = np.nonzero((back.view(np.uint32) != recs.view(np.uint32)).any(axis=1))[0]
    if bad.size:
        raise ValueError(f"{bad.size} records do not follow the controller's trajAll expansion "
                         f"(first: {bad[0]}); send them as full records")
    return out

