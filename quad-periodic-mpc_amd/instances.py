"""Synthetic batched MPC instances (SURVEY.md §8(d) generator).

Each instance is one ``solveDenseMPC`` call of a Unitree A1 in trot
(``ConvexMPCLocomotion.cpp:612-870``): a randomised body state, foot offsets around the A1
nominal stance, a trot contact table at a random phase (``Gait.cpp:159-188``,
``OffsetDurationGait`` with P = 18, offsets (0, 9, 9, 0), durations 9:
``ConvexMPCLocomotion.cpp:41``), and the reference trajectory ``trajAll`` built exactly as
``updateMPCIfNeeded`` does (``ConvexMPCLocomotion.cpp:554-585``). A fraction of instances get
Bernoulli(0.5) contacts instead (stress / ragged reduced sizes).

Deterministic and shard-reproducible: one Philox4x32-10 stream per instance id, fully
vectorised.
"""
from __future__ import annotations

import numpy as np

from .records import pack_records

BASE_SEED = 20251015
# A1 hip offsets (MiniCheetah-style leg order FR, FL, RR, RL): x = +-0.1805, y = -+0.047,
# plus the abad link +-0.0838 in y (common/Dynamics/MiniCheetah.h:27-40, Quadruped.h:95-102).
_HIP_X = np.array([0.1805, 0.1805, -0.1805, -0.1805])
_HIP_Y = np.array([-0.047, 0.047, -0.047, 0.047]) + np.array([-0.0838, 0.0838, -0.0838, 0.0838])


def trot_table(horizon: int, iteration: np.ndarray, period: int = 18) -> np.ndarray:
    """OffsetDurationGait::getMpcTable (Gait.cpp:159-188) for the trot gait; rows i < N.

    For N > P the reference would read past its P-row table; the period is stretched to N
    there."""
    P = max(period, horizon)
    offsets = np.array([0, P // 2, P // 2, 0])
    durations = np.array([P // 2] * 4)
    i = np.arange(horizon)[None, :, None]
    it = (i + iteration[:, None, None] + 1) % P
    prog = it - offsets[None, None, :]
    prog = np.where(prog < 0, prog + P, prog)
    return (prog < durations[None, None, :]).astype(np.int32).reshape(iteration.shape[0], 4 * horizon)


def gait_table(horizon: int, iteration: np.ndarray, offsets, durations, period: int = 18) -> np.ndarray:
    """OffsetDurationGait::getMpcTable (Gait.cpp:159-188) for any offset/duration gait: row i is
    iteration (i + it + 1) mod P, foot j in stance iff (row - offset_j) mod P < duration_j.
    Returns int32 [len(iteration), 4 * horizon] (step-major, foot-minor). The caller chooses P;
    for N > P the reference would read past its P-row table."""
    P = int(period)
    off = np.asarray(offsets, np.int64)
    dur = np.asarray(durations, np.int64)
    i = np.arange(horizon)[None, :, None]
    it = (i + np.asarray(iteration)[:, None, None] + 1) % P
    prog = it - off[None, None, :]
    prog = np.where(prog < 0, prog + P, prog)
    return (prog < dur[None, None, :]).astype(np.int32).reshape(len(iteration), 4 * horizon)


def euler_zyx_to_quat(roll, pitch, yaw):
    cr, sr = np.cos(roll / 2), np.sin(roll / 2)
    cp, sp = np.cos(pitch / 2), np.sin(pitch / 2)
    cy, sy = np.cos(yaw / 2), np.sin(yaw / 2)
    w = cr * cp * cy + sr * sp * sy
    x = sr * cp * cy - cr * sp * sy
    y = cr * sp * cy + sr * cp * sy
    z = cr * cp * sy - sr * sp * cy
    return np.stack([w, x, y, z], axis=-1)


# ---------------------------------------------------------------------------------------------
# Per-instance counter-based randomness: instance ``id`` draws from
# Philox4x32-10 with key (base seed, 0x5EED0000 + id) and counters 0, 1, 2, ... Any contiguous
# shard [first_id, first_id + batch) therefore reproduces exactly the instances a 1-GPU run
# generates for those ids, whatever the world size.
# ---------------------------------------------------------------------------------------------
_PHILOX_M0, _PHILOX_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_PHILOX_W0, _PHILOX_W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_MASK32 = np.uint64(0xFFFFFFFF)
SEED_TAG = 0x5EED0000


def philox4x32(key0: np.ndarray, key1: np.ndarray, blocks: int) -> np.ndarray:
    """Philox4x32-10 (Salmon et al., SC'11) over counters (c, 0, 0, 0), c < ``blocks``, one key
    per row: returns uint32 [len(key0), 4 * blocks]."""
    k0 = np.broadcast_to(np.asarray(key0, np.uint64)[:, None], (len(key0), blocks)).copy()
    k1 = np.broadcast_to(np.asarray(key1, np.uint64)[:, None], (len(key0), blocks)).copy()
    c0 = np.broadcast_to(np.arange(blocks, dtype=np.uint64)[None, :], k0.shape).copy()
    c1 = np.zeros_like(c0)
    c2 = np.zeros_like(c0)
    c3 = np.zeros_like(c0)
    for r in range(10):
        p0 = _PHILOX_M0 * c0
        p1 = _PHILOX_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
        if r < 9:
            k0 = (k0 + _PHILOX_W0) & _MASK32
            k1 = (k1 + _PHILOX_W1) & _MASK32
    out = np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)
    return out.reshape(len(key0), 4 * blocks)


# fixed draw slots per instance (uniforms in (0, 1); a normal takes two slots, Box-Muller)
_S_ROLL, _S_PITCH, _S_YAW, _S_PX, _S_PY, _S_PZ = 0, 2, 4, 5, 6, 8
_S_VX, _S_VY, _S_VZ, _S_W, _S_BX, _S_BY, _S_RZ = 10, 11, 12, 14, 20, 28, 36
_S_PHASE, _S_RND, _S_VDX, _S_VDY, _S_YAWRATE, _S_XS, _S_YS, _S_YAWN, _S_XDRAG = (
    44, 45, 46, 47, 48, 49, 50, 51, 53)
_S_FIXED = 64          # then 4N Bernoulli slots of the random contact tables


class _Draws:
    def __init__(self, u32: np.ndarray):
        self.u = (u32.astype(np.float64) + 0.5) * (1.0 / 4294967296.0)

    def uniform(self, slot, lo=0.0, hi=1.0, count=1):
        x = self.u[:, slot:slot + count]
        x = lo + (hi - lo) * x
        return x[:, 0] if count == 1 else x

    def normal(self, slot, mu=0.0, sd=1.0, count=1):
        u1 = self.u[:, slot:slot + 2 * count:2]
        u2 = self.u[:, slot + 1:slot + 2 * count:2]
        z = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
        x = mu + sd * z
        return x[:, 0] if count == 1 else x


def instance_draws(first_id: int, batch: int, horizon: int, seed: int = BASE_SEED) -> _Draws:
    ids = np.arange(first_id, first_id + batch, dtype=np.uint64)
    key0 = np.full(batch, seed & 0xFFFFFFFF, np.uint64)
    key1 = (ids + np.uint64(SEED_TAG)) & _MASK32
    blocks = (_S_FIXED + 4 * horizon + 3) // 4
    return _Draws(philox4x32(key0, key1, blocks))


def make_instances(batch: int, horizon: int = 10, seed: int = BASE_SEED, dt: float = 0.026,
                   random_contact_frac: float = 0.25, body_height: float = 0.29,
                   x_drag_range: float = 0.5, stress: bool = False, first_id: int = 0,
                   chunk: int = 65536, gait: str = "trotting") -> np.ndarray:
    """Return packed records [batch, record_words(horizon)] (float32) for instance ids
    ``first_id .. first_id + batch - 1``.

    Every instance draws from its own Philox stream (key = (seed, 0x5EED0000 + id)), so a shard
    of ids reproduces the same instances as a whole-batch call. ``stress`` widens the
    velocity/orientation errors so friction cones bind (active sets). ``gait`` names one of the
    controller's OffsetDurationGait tables (``loco_gaits``, ConvexMPCLocomotion.cpp:41-51), with
    the period stretched to N when N > 18: "standing" puts every foot in stance at every step
    (n = 12 N), "walking" three feet on average."""
    if batch > chunk:  # bounded temporaries for very large batches
        return np.concatenate([
            make_instances(min(chunk, batch - a), horizon, seed, dt, random_contact_frac,
                           body_height, x_drag_range, stress, first_id + a, chunk, gait)
            for a in range(0, batch, chunk)], axis=0)
    B, N = batch, horizon
    d = instance_draws(first_id, B, N, seed)
    scale = 3.0 if stress else 1.0
    roll = np.clip(d.normal(_S_ROLL, 0, 0.05 * scale), -0.3 * scale, 0.3 * scale)
    pitch = np.clip(d.normal(_S_PITCH, 0, 0.05 * scale), -0.3 * scale, 0.3 * scale)
    yaw = d.uniform(_S_YAW, -np.pi, np.pi)
    q = euler_zyx_to_quat(roll, pitch, yaw)
    p = np.stack([d.uniform(_S_PX, -1, 1), d.uniform(_S_PY, -1, 1),
                  body_height + d.normal(_S_PZ, 0, 0.02)], -1)
    v = np.stack([d.uniform(_S_VX, -0.7, 0.7) * scale, d.uniform(_S_VY, -0.4, 0.4) * scale,
                  d.normal(_S_VZ, 0, 0.05)], -1)
    w = d.normal(_S_W, 0, 0.3 * scale, count=3)
    # foot offsets r = pFoot - p in world frame (axis-major, ConvexMPCLocomotion.cpp:786-790)
    cy, sy = np.cos(yaw)[:, None], np.sin(yaw)[:, None]
    bx = _HIP_X[None, :] + d.normal(_S_BX, 0, 0.03, count=4)
    by = _HIP_Y[None, :] + d.normal(_S_BY, 0, 0.03, count=4)
    rx = cy * bx - sy * by
    ry = sy * bx + cy * by
    rz = -p[:, 2:3] + d.normal(_S_RZ, 0, 0.02, count=4)
    r = np.concatenate([rx, ry, rz], axis=1)
    # contact table: trot at a random phase; a fraction with Bernoulli(0.5) contacts
    phase = np.minimum((d.uniform(_S_PHASE) * 18).astype(np.int64), 17)
    if gait == "trotting":
        table = trot_table(N, phase)
    else:
        P = max(18, N)
        off, dur, _ = loco_gaits(P)[gait]
        table = gait_table(N, phase % P, off, dur, P)
    rnd = d.uniform(_S_RND) < random_contact_frac
    if rnd.any():
        bern = d.uniform(_S_FIXED, count=4 * N).reshape(B, 4 * N)
        table[rnd] = (bern[rnd] < 0.5).astype(np.int32)
    # trajectory (ConvexMPCLocomotion.cpp:554-585)
    vdes_x = d.uniform(_S_VDX, -0.7, 0.7) * scale
    vdes_y = d.uniform(_S_VDY, -0.4, 0.4) * scale
    yaw_rate = d.uniform(_S_YAWRATE, -2.5, 2.5)
    x_start = p[:, 0] + d.uniform(_S_XS, -0.1, 0.1)
    y_start = p[:, 1] + d.uniform(_S_YS, -0.1, 0.1)
    traj = np.zeros((B, N, 12), np.float32)
    traj[:, :, 2] = (yaw + d.normal(_S_YAWN, 0, 0.05))[:, None]   # _yaw_des
    traj[:, :, 3] = x_start[:, None]
    traj[:, :, 4] = y_start[:, None]
    traj[:, :, 5] = body_height
    traj[:, :, 8] = yaw_rate[:, None]
    traj[:, :, 9] = vdes_x[:, None]
    traj[:, :, 10] = vdes_y[:, None]
    traj[:, 0, 2] = yaw                                  # trajAll[2] = seResult.rpy[2]
    for i in range(1, N):                                # fp32 recurrence as the caller
        traj[:, i, 3] = traj[:, i - 1, 3] + np.float32(dt) * traj[:, i, 9]
        traj[:, i, 4] = traj[:, i - 1, 4] + np.float32(dt) * traj[:, i, 10]
        traj[:, i, 2] = traj[:, i - 1, 2] + np.float32(dt) * traj[:, i, 8]
    x_drag = d.uniform(_S_XDRAG, -x_drag_range, x_drag_range)
    rpy = np.stack([roll, pitch, yaw], -1)
    return pack_records(p, v, q, w, r, traj.reshape(B, 12 * N), table, rpy=rpy, x_drag=x_drag)


def make_disturbance(batch: int, steps: int, seed: int = BASE_SEED + 5, dt: float = 0.026,
                     d_s: float = -10.0, d_n: float = 15.0, freq: float = 0.33, noise: float = 1.0,
                     t0: float = 0.0):
    """Config-5 residual samples f_ext[3] for ``steps`` MPC steps of ``batch`` instances:
    ``d_s + d_n sin(2 pi f t + phi) + N(0, noise^2)`` with a random phase per instance and
    t_k = t0 + k dt (the disturbance of raisim_unitree_ros_driver.hpp:126-129).
    Returns (f3 [batch, steps] float32, t [steps] float32)."""
    g = np.random.Generator(np.random.Philox(seed))
    t = (t0 + dt * np.arange(steps)).astype(np.float32)
    phi = g.uniform(0, 2 * np.pi, batch)
    f3 = d_s + d_n * np.sin(2 * np.pi * freq * t[None, :].astype(np.float64) + phi[:, None])
    f3 = f3 + noise * g.normal(0, 1, (batch, steps))
    return f3.astype(np.float32), t


def make_logs(records: np.ndarray, seed: int = BASE_SEED + 6) -> np.ndarray:
    """LogData records (include/cmpc_solver.h CMPC_LOG_*) of a previous step near each
    instance's current state: perturbed pose / twist, stance-like foot forces, the body rotation
    and foot offsets of that step (fields read by ConvexMPCLocomotion.cpp:639-771)."""
    from .records import (LOG_ANG, LOG_EUL, LOG_FORCE, LOG_LIN, LOG_POS, LOG_R, LOG_ROT,
                          LOG_WORDS, LOG_XDRAG, REC_P, REC_R, REC_RPY, REC_V, REC_W, REC_XDRAG)
    g = np.random.Generator(np.random.Philox(seed))
    B = records.shape[0]
    lg = np.zeros((B, LOG_WORDS), np.float32)
    lg[:, LOG_POS:LOG_POS + 3] = records[:, REC_P:REC_P + 3] + g.normal(0, 0.01, (B, 3))
    eul = records[:, REC_RPY:REC_RPY + 3] + g.normal(0, 0.01, (B, 3))
    lg[:, LOG_EUL:LOG_EUL + 3] = eul
    lg[:, LOG_ANG:LOG_ANG + 3] = records[:, REC_W:REC_W + 3] + g.normal(0, 0.05, (B, 3))
    lg[:, LOG_LIN:LOG_LIN + 3] = records[:, REC_V:REC_V + 3] + g.normal(0, 0.05, (B, 3))
    f = np.zeros((B, 4, 3))
    f[:, :, 2] = g.uniform(20, 80, (B, 4))
    f[:, :, :2] = g.normal(0, 5, (B, 4, 2))
    lg[:, LOG_FORCE:LOG_FORCE + 12] = f.reshape(B, 12)
    lg[:, LOG_XDRAG] = records[:, REC_XDRAG]
    lg[:, LOG_R:LOG_R + 12] = records[:, REC_R:REC_R + 12]
    q = euler_zyx_to_quat(eul[:, 0].astype(np.float64), eul[:, 1].astype(np.float64),
                          eul[:, 2].astype(np.float64))
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = np.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], -1)
    lg[:, LOG_ROT:LOG_ROT + 9] = R
    return lg


# OffsetDurationGait tables of the controller (ConvexMPCLocomotion.cpp:41-51, gait_period P;
# Vec4<int> of doubles truncates): name -> (offsets, durations, cmpc_gait number)
def loco_gaits(P: int = 18):
    return {
        "trotting": ((0, int(P / 2.0), int(P / 2.0), 0), (int(P / 2.0),) * 4, 9),
        "bounding": ((5, 5, 0, 0), (4, 4, 4, 4), 1),
        "pronking": ((0, 0, 0, 0), (8, 8, 8, 8), 2),
        "galloping": ((0, 2, 7, 9), (4, 4, 4, 4), 6),
        "standing": ((0, 0, 0, 0), (P, P, P, P), 4),
        "walking": ((int(2 * P / 4.0), 0, int(P / 4.0), int(3 * P / 4.0)), (int(0.75 * P),) * 4, 10),
        "pacing": ((5, 0, 5, 0), (5, 5, 5, 5), 8),  # gait 8: rpy_comp[0] off (:230)
    }


def make_loco_states(batch: int, seed: int = BASE_SEED + 11, P: int = 18, first_run_frac: float = 0.1,
                     gaits=("trotting", "trotting", "trotting", "bounding", "pronking", "galloping",
                            "standing", "walking", "pacing"), omni_frac: float = 0.1,
                     sim_feet_frac: float = 0.0) -> np.ndarray:
    """Locomotion-controller states [batch, LOCO_WORDS] (include/cmpc_solver.h CMPC_LOCO_*):
    A1-like body states, world foot positions around the nominal stance, stick commands, a
    random gait from ``gaits`` at a random iteration counter, and warm integrator states."""
    from .records import (LOCO_CMD, LOCO_COUNTER, LOCO_FIRST, LOCO_FLAGS, LOCO_GAIT, LOCO_HEIGHT,
                          LOCO_OMNI, LOCO_PFOOT, LOCO_POS, LOCO_PRONK, LOCO_Q, LOCO_RPY,
                          LOCO_RPYINT, LOCO_STAND, LOCO_STANDING, LOCO_VDES, LOCO_VW, LOCO_WORDS,
                          LOCO_WPD, LOCO_WW, LOCO_XCI, LOCO_ZGT)
    g = np.random.Generator(np.random.Philox(seed))
    B = batch
    s = np.zeros((B, LOCO_WORDS), np.float32)
    roll = np.clip(g.normal(0, 0.05, B), -0.3, 0.3)
    pitch = np.clip(g.normal(0, 0.05, B), -0.3, 0.3)
    yaw = g.uniform(-np.pi, np.pi, B)
    pos = np.stack([g.uniform(-1, 1, B), g.uniform(-1, 1, B), 0.29 + g.normal(0, 0.02, B)], -1)
    s[:, LOCO_POS:LOCO_POS + 3] = pos
    s[:, LOCO_ZGT] = pos[:, 2] + g.normal(0, 0.005, B)
    s[:, LOCO_Q:LOCO_Q + 4] = euler_zyx_to_quat(roll, pitch, yaw)
    s[:, LOCO_RPY:LOCO_RPY + 3] = np.stack([roll, pitch, yaw], -1)
    vw = np.stack([g.uniform(-0.7, 0.7, B), g.uniform(-0.4, 0.4, B), g.normal(0, 0.05, B)], -1)
    vw[g.random(B) < 0.2, 0] *= 0.2     # some slow instances: the |v| thresholds of :218-222
    s[:, LOCO_VW:LOCO_VW + 3] = vw
    s[:, LOCO_WW:LOCO_WW + 3] = g.normal(0, 0.3, (B, 3))
    cy, sy = np.cos(yaw)[:, None], np.sin(yaw)[:, None]
    bx = _HIP_X[None, :] + g.normal(0, 0.03, (B, 4))
    by = _HIP_Y[None, :] + g.normal(0, 0.03, (B, 4))
    pf = np.stack([pos[:, 0:1] + cy * bx - sy * by, pos[:, 1:2] + sy * bx + cy * by,
                   g.normal(0, 0.01, (B, 4))], -1)          # [B, leg, axis]
    s[:, LOCO_PFOOT:LOCO_PFOOT + 12] = pf.reshape(B, 12)
    s[:, LOCO_CMD] = g.uniform(-0.7, 0.7, B)
    s[:, LOCO_CMD + 1] = g.uniform(-0.4, 0.4, B)
    s[:, LOCO_CMD + 2] = g.uniform(-2.5, 2.5, B)
    s[:, LOCO_HEIGHT] = 0.29
    s[:, LOCO_VDES] = s[:, LOCO_CMD] * g.uniform(0, 1, B)
    s[:, LOCO_VDES + 1] = s[:, LOCO_CMD + 1] * g.uniform(0, 1, B)
    s[:, LOCO_WPD:LOCO_WPD + 2] = pos[:, :2] + g.uniform(-0.2, 0.2, (B, 2))
    s[:, LOCO_RPYINT:LOCO_RPYINT + 2] = g.uniform(-0.3, 0.3, (B, 2))
    s[:, LOCO_XCI] = g.uniform(-0.5, 0.5, B)
    tab = loco_gaits(P)
    names = [gaits[k] for k in g.integers(0, len(gaits), B)]
    ints = np.zeros((B, 10), np.int32)
    flags = np.zeros(B, np.uint32)
    for b, nm in enumerate(names):
        off, dur, num = tab[nm]
        ints[b, 0] = P
        ints[b, 1:5] = off
        ints[b, 5:9] = dur
        if num == 4:
            flags[b] |= LOCO_STANDING
        if num == 8:
            flags[b] |= LOCO_PRONK
    ints[:, 9] = g.integers(0, 100000, B)                   # iterationCounter
    flags[g.random(B) < omni_frac] |= LOCO_OMNI
    flags[g.random(B) < first_run_frac] |= LOCO_FIRST
    s[:, LOCO_GAIT:LOCO_GAIT + 9] = ints[:, :9].view(np.float32)
    s[:, LOCO_COUNTER] = ints[:, 9].view(np.float32)
    s[:, LOCO_FLAGS] = flags.view(np.float32)
    s[:, LOCO_STAND] = pos[:, 0]
    s[:, LOCO_STAND + 1] = pos[:, 1]
    s[:, LOCO_STAND + 2] = yaw
    # swing state (:276-331, :350-431): a swing in progress from / towards the current feet
    from .records import LOCO_FSWING0, LOCO_P0, LOCO_PDES, LOCO_PF, LOCO_SIMFEET, LOCO_SWREM
    s[:, LOCO_SWREM:LOCO_SWREM + 4] = g.uniform(0.0, 0.25, (B, 4))
    for w in (LOCO_P0, LOCO_PF, LOCO_PDES):
        s[:, w:w + 12] = s[:, LOCO_PFOOT:LOCO_PFOOT + 12]
    fs = (g.random((B, 4)) < 0.5).astype(np.uint32)
    flags = flags | (fs * (LOCO_FSWING0 << np.arange(4, dtype=np.uint32))).sum(1).astype(np.uint32)
    flags[g.random(B) < sim_feet_frac] |= LOCO_SIMFEET
    s[:, LOCO_FLAGS] = flags.view(np.float32)
    return s
