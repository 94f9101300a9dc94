"""LogData wire format and bag replay.

The controller publishes one ``unitree_legged_msgs/LogData`` per MPC step on ``/log_data``
(``ConvexMPCLocomotion::publishLogData``, ``ConvexMPCLocomotion.cpp:978-1070``) and reads the
previous one back for the config-5 residual (``logDataCallback``, ``:639-771``). This module:

- reads and writes that message in the ROS1 wire format (little-endian, no padding; message
  definition ``unitree_legged_msgs/msg/LogData.msg``);
- converts messages to the solver's ``CMPC_LOG_*`` records (``include/cmpc_solver.h``), with the
  geometry_msgs doubles cast to fp32 as the reference's float Eigen matrices do (``:651-750``);
- reads and writes ROS bag v2.0 files (``launch/unitree_bag_play.launch`` replays such bags),
  uncompressed or bz2 chunks;
- replays B logged streams through the batched estimator and solver on the GPU
  (:class:`LogReplay`): step k uses message k-1 as the previous step's log and message k as the
  current state, as the live controller does one MPC step later.

Host-side data plumbing only: every solve and residual runs in ``libcmpc_hip.so``.
"""
from __future__ import annotations

import bz2
import hashlib
import io
import struct
from typing import Iterable, Sequence

import numpy as np

from .records import (LOG_ANG, LOG_EUL, LOG_FORCE, LOG_LIN, LOG_POS, LOG_R, LOG_ROT, LOG_WORDS,
                      LOG_XDRAG, pack_records)

TOPIC = "/log_data"                               # ConvexMPCLocomotion.cpp:55-56
MSG_TYPE = "unitree_legged_msgs/LogData"

# Fixed part after the Header, in LogData.msg order: three pose/twist groups "act" then "des"
# (Point 3 f64, Vector3 3 f64, Twist = linear 3 f64 + angular 3 f64), then 34 float32 fields.
_F64_FIELDS = [f"{g}_{k}" for g in ("pos_act", "euler_act") for k in "xyz"] + \
    [f"vel_act_{p}_{k}" for p in ("linear", "angular") for k in "xyz"] + \
    [f"{g}_{k}" for g in ("pos_des", "euler_des") for k in "xyz"] + \
    [f"vel_des_{p}_{k}" for p in ("linear", "angular") for k in "xyz"]
_F32_FIELDS = [f"foot_force{j}_{k}" for j in range(4) for k in "xyz"] + ["x_drag"] + \
    [f"r_{a}_{j}" for a in "xyz" for j in range(1, 5)] + \
    [f"R_{i}{j}" for i in range(3) for j in range(3)]
BODY_DTYPE = np.dtype([(n, "<f8") for n in _F64_FIELDS] + [(n, "<f4") for n in _F32_FIELDS])
assert BODY_DTYPE.itemsize == 24 * 8 + 34 * 4 == 328

# ROS md5sum of LogData, by the genmsg rule: the definition text with comments stripped and
# every nested message type replaced by its own md5sum (std_msgs/Header, geometry_msgs/Point,
# Vector3, Twist are the published ROS1 sums). Written into bag connection headers; readers
# here do not check it.
_DEP_MD5 = {"Header": "2176decaecbce78abc3b96ef049fabed",
            "geometry_msgs/Point": "4a842b65f413084dc2b10fb484ea7f17",
            "geometry_msgs/Vector3": "4a842b65f413084dc2b10fb484ea7f17",
            "geometry_msgs/Twist": "9f195f881246fdfa2798d1d3eebca84a"}
_DEF_LINES = [("Header", "header"),
              ("geometry_msgs/Point", "pos_act"), ("geometry_msgs/Vector3", "euler_act"),
              ("geometry_msgs/Twist", "vel_act"),
              ("geometry_msgs/Point", "pos_des"), ("geometry_msgs/Vector3", "euler_des"),
              ("geometry_msgs/Twist", "vel_des")] + [("float32", n) for n in _F32_FIELDS]
MESSAGE_DEFINITION = "\n".join(f"{t} {n}" for t, n in _DEF_LINES) + "\n"
MD5SUM = hashlib.md5("\n".join(f"{_DEP_MD5.get(t, t)} {n}" for t, n in _DEF_LINES)
                     .encode()).hexdigest()


# ---- message (de)serialisation ---------------------------------------------------------------
def empty_messages(n: int) -> np.ndarray:
    """Zeroed structured array of ``n`` message bodies (fields named as LogData.msg, nested
    geometry fields flattened: ``pos_act_x``, ``vel_act_angular_z`` ...)."""
    return np.zeros(n, BODY_DTYPE)


def serialize(body: np.ndarray, stamps_ns: Sequence[int] | None = None, seq0: int = 0,
              frame_id: str = "") -> list[bytes]:
    """ROS1 serialisation of each message: Header {uint32 seq, time stamp (uint32 sec, uint32
    nsec), string frame_id (uint32 length + bytes)} followed by the 328-byte body."""
    body = np.ascontiguousarray(body, BODY_DTYPE)
    fid = frame_id.encode()
    out = []
    for i in range(body.shape[0]):
        t = int(stamps_ns[i]) if stamps_ns is not None else 0
        hdr = struct.pack("<IIII", (seq0 + i) & 0xFFFFFFFF, t // 1_000_000_000,
                          t % 1_000_000_000, len(fid)) + fid
        out.append(hdr + body[i:i + 1].tobytes())
    return out


def deserialize(msgs: Iterable[bytes]):
    """Inverse of :func:`serialize` -> (body structured array [n], stamps_ns int64 [n],
    seq uint32 [n]). Raises ValueError on a truncated or over-long message."""
    msgs = list(msgs)
    body = np.empty(len(msgs), BODY_DTYPE)
    stamps = np.empty(len(msgs), np.int64)
    seq = np.empty(len(msgs), np.uint32)
    for i, m in enumerate(msgs):
        if len(m) < 16:
            raise ValueError(f"LogData message {i}: {len(m)} bytes, header needs 16")
        s, sec, nsec, flen = struct.unpack_from("<IIII", m, 0)
        off = 16 + flen
        if len(m) != off + BODY_DTYPE.itemsize:
            raise ValueError(f"LogData message {i}: {len(m)} bytes, expected "
                             f"{off + BODY_DTYPE.itemsize} (frame_id of {flen} bytes)")
        body[i] = np.frombuffer(m, BODY_DTYPE, 1, off)[0]
        stamps[i] = sec * 1_000_000_000 + nsec
        seq[i] = s
    return body, stamps, seq


def to_log_records(body: np.ndarray) -> np.ndarray:
    """Message bodies -> CMPC_LOG records [n, LOG_WORDS] fp32 (the fields
    ConvexMPCLocomotion.cpp:643-750 reads; doubles cast to float)."""
    n = body.shape[0]
    lg = np.zeros((n, LOG_WORDS), np.float32)

    def put(off, names):
        for k, name in enumerate(names):
            lg[:, off + k] = body[name].astype(np.float32)

    put(LOG_POS, [f"pos_act_{k}" for k in "xyz"])
    put(LOG_EUL, [f"euler_act_{k}" for k in "xyz"])
    put(LOG_ANG, [f"vel_act_angular_{k}" for k in "xyz"])
    put(LOG_LIN, [f"vel_act_linear_{k}" for k in "xyz"])
    put(LOG_FORCE, [f"foot_force{j}_{k}" for j in range(4) for k in "xyz"])
    put(LOG_XDRAG, ["x_drag"])
    put(LOG_R, [f"r_{a}_{j}" for a in "xyz" for j in range(1, 5)])
    put(LOG_ROT, [f"R_{i}{j}" for i in range(3) for j in range(3)])
    return lg


def from_log_records(lg: np.ndarray, des: np.ndarray | None = None) -> np.ndarray:
    """CMPC_LOG records [n, LOG_WORDS] (+ optional desired pose/twist [n, 12]: pos_des,
    euler_des, vel_des.linear, vel_des.angular) -> message bodies, as publishLogData fills them
    (ConvexMPCLocomotion.cpp:985-1070)."""
    lg = np.asarray(lg, np.float32)
    body = empty_messages(lg.shape[0])

    def get(off, names):
        for k, name in enumerate(names):
            body[name] = lg[:, off + k]

    get(LOG_POS, [f"pos_act_{k}" for k in "xyz"])
    get(LOG_EUL, [f"euler_act_{k}" for k in "xyz"])
    get(LOG_ANG, [f"vel_act_angular_{k}" for k in "xyz"])
    get(LOG_LIN, [f"vel_act_linear_{k}" for k in "xyz"])
    get(LOG_FORCE, [f"foot_force{j}_{k}" for j in range(4) for k in "xyz"])
    get(LOG_XDRAG, ["x_drag"])
    get(LOG_R, [f"r_{a}_{j}" for a in "xyz" for j in range(1, 5)])
    get(LOG_ROT, [f"R_{i}{j}" for i in range(3) for j in range(3)])
    if des is not None:
        names = [f"pos_des_{k}" for k in "xyz"] + [f"euler_des_{k}" for k in "xyz"] + \
            [f"vel_des_linear_{k}" for k in "xyz"] + [f"vel_des_angular_{k}" for k in "xyz"]
        for k, name in enumerate(names):
            body[name] = des[:, k]
    return body


# ---- ROS bag v2.0 ----------------------------------------------------------------------------
_MAGIC = b"#ROSBAG V2.0\n"
_OP_MSG, _OP_BAGHDR, _OP_INDEX, _OP_CHUNK, _OP_CHUNKINFO, _OP_CONN = 2, 3, 4, 5, 6, 7


def _fields(buf: bytes) -> dict:
    out, i = {}, 0
    while i < len(buf):
        (n,) = struct.unpack_from("<i", buf, i)
        k, _, v = buf[i + 4:i + 4 + n].partition(b"=")
        out[k.decode()] = v
        i += 4 + n
    return out


def _hdr(**kv) -> bytes:
    parts = []
    for k, v in kv.items():
        f = k.encode() + b"=" + v
        parts.append(struct.pack("<i", len(f)) + f)
    return b"".join(parts)


def _record(header: bytes, data: bytes) -> bytes:
    return struct.pack("<i", len(header)) + header + struct.pack("<i", len(data)) + data


def _records(buf: bytes, start: int = 0):
    i = start
    while i + 4 <= len(buf):
        (hl,) = struct.unpack_from("<i", buf, i)
        h = _fields(buf[i + 4:i + 4 + hl])
        (dl,) = struct.unpack_from("<i", buf, i + 4 + hl)
        d0 = i + 8 + hl
        if d0 + dl > len(buf):
            raise ValueError("truncated bag record")
        yield h, buf[d0:d0 + dl]
        i = d0 + dl


def _time(v: bytes) -> int:
    sec, nsec = struct.unpack("<II", v)
    return sec * 1_000_000_000 + nsec


def read_bag(path_or_bytes, topic: str | None = TOPIC):
    """Messages of a ROS bag v2.0 -> list of (topic, stamp_ns, raw bytes) in file order,
    filtered to ``topic`` (None: all). Chunks: ``none`` and ``bz2``; ``lz4`` raises."""
    buf = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else \
        open(path_or_bytes, "rb").read()
    if not buf.startswith(_MAGIC):
        raise ValueError("not a ROS bag v2.0 file")
    conns, msgs = {}, []

    def visit(h, d):
        op = h.get("op", b"\0")[0]
        if op == _OP_CONN:
            conns[struct.unpack("<i", h["conn"])[0]] = h["topic"].decode()
        elif op == _OP_MSG:
            msgs.append((struct.unpack("<i", h["conn"])[0], _time(h["time"]), bytes(d)))

    for h, d in _records(buf, len(_MAGIC)):
        if h.get("op", b"\0")[0] == _OP_CHUNK:
            comp = h["compression"].decode()
            if comp == "bz2":
                d = bz2.decompress(d)
            elif comp != "none":
                raise ValueError(f"bag chunk compression {comp!r} not supported (none, bz2)")
            for hh, dd in _records(d):
                visit(hh, dd)
        else:
            visit(h, d)
    out = [(conns.get(c, ""), t, m) for c, t, m in msgs]
    return [x for x in out if topic is None or x[0] == topic]


def write_bag(path, messages: Sequence[bytes], stamps_ns: Sequence[int], topic: str = TOPIC,
              compression: str = "none") -> bytes:
    """One-connection, one-chunk ROS bag v2.0 (bag header padded to 4096 bytes, connection,
    chunk, index data and chunk info records, as rosbag writes them). Returns the bytes and
    writes them to ``path`` unless it is None."""
    if compression not in ("none", "bz2"):
        raise ValueError(compression)
    conn_id = struct.pack("<i", 0)
    conn_rec = _record(_hdr(op=bytes([_OP_CONN]), conn=conn_id, topic=topic.encode()),
                       _hdr(topic=topic.encode(), type=MSG_TYPE.encode(), md5sum=MD5SUM.encode(),
                            message_definition=MESSAGE_DEFINITION.encode()))
    tpack = [struct.pack("<II", int(t) // 1_000_000_000, int(t) % 1_000_000_000)
             for t in stamps_ns]
    inner, offs = io.BytesIO(), []
    inner.write(conn_rec)
    for m, tp in zip(messages, tpack):
        offs.append(inner.tell())
        inner.write(_record(_hdr(op=bytes([_OP_MSG]), conn=conn_id, time=tp), m))
    raw = inner.getvalue()
    data = bz2.compress(raw) if compression == "bz2" else raw
    chunk = _record(_hdr(op=bytes([_OP_CHUNK]), compression=compression.encode(),
                         size=struct.pack("<I", len(raw))), data)
    index = _record(_hdr(op=bytes([_OP_INDEX]), ver=struct.pack("<i", 1), conn=conn_id,
                         count=struct.pack("<i", len(offs))),
                    b"".join(tp + struct.pack("<I", o) for tp, o in zip(tpack, offs)))
    chunk_pos = len(_MAGIC) + 4096
    index_pos = chunk_pos + len(chunk) + len(index)
    t0 = tpack[0] if tpack else b"\0" * 8
    t1 = tpack[-1] if tpack else b"\0" * 8
    info = _record(_hdr(op=bytes([_OP_CHUNKINFO]), ver=struct.pack("<i", 1),
                        chunk_pos=struct.pack("<Q", chunk_pos), start_time=t0, end_time=t1,
                        count=struct.pack("<i", 1)), conn_id + struct.pack("<i", len(offs)))
    bh = _hdr(op=bytes([_OP_BAGHDR]), index_pos=struct.pack("<Q", index_pos),
              conn_count=struct.pack("<i", 1), chunk_count=struct.pack("<i", 1))
    pad = 4096 - (len(bh) + 8)
    out = _MAGIC + _record(bh, b" " * pad) + chunk + index + conn_rec + info
    if path is not None:
        with open(path, "wb") as f:
            f.write(out)
    return out


def load_streams(bags: Sequence, topic: str = TOPIC):
    """B bags (paths or bytes) -> (CMPC_LOG records [T, B, LOG_WORDS], desired pose/twist
    [T, B, 12], stamps_ns [T, B]) truncated to the shortest bag's message count."""
    per = [deserialize([m for _, _, m in read_bag(b, topic)]) for b in bags]
    T = min(p[0].shape[0] for p in per)
    logs = np.stack([to_log_records(p[0][:T]) for p in per], 1)
    des_names = [f"pos_des_{k}" for k in "xyz"] + [f"euler_des_{k}" for k in "xyz"] + \
        [f"vel_des_linear_{k}" for k in "xyz"] + [f"vel_des_angular_{k}" for k in "xyz"]
    des = np.stack([np.stack([p[0][n][:T] for n in des_names], -1) for p in per], 1)
    stamps = np.stack([p[1][:T] for p in per], 1)
    return logs, des.astype(np.float32), stamps


# ---- records for the current step -----------------------------------------------------------
def euler_to_quat(rpy: np.ndarray) -> np.ndarray:
    """ZYX Euler (roll, pitch, yaw) -> (w, x, y, z)."""
    r, p, y = (rpy[:, i].astype(np.float64) / 2 for i in range(3))
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.stack([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                     cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy], -1)


def records_from_logs(lg: np.ndarray, des: np.ndarray, horizon: int, dt: float) -> np.ndarray:
    """Solve records for the step a LogData message describes.

    State: p = pos_act (z is the ground-truth height, :987), v, ω, rpy = euler_act, q from rpy,
    r = r_{x,y,z}_{1..4}, x_drag. Trajectory per ``updateMPCIfNeeded`` (:537-585): roll, pitch,
    z from the desired pose, yaw / x / y advanced k·dt at the desired rates, with step 0's yaw
    the measured one. Replay convention (LogData carries no contact table): a leg is in stance
    over the whole horizon iff its logged vertical force is positive."""
    lg = np.asarray(lg, np.float32)
    des = np.asarray(des, np.float32)
    B, N = lg.shape[0], horizon
    rpy = lg[:, LOG_EUL:LOG_EUL + 3]
    traj = np.zeros((B, N, 12), np.float32)
    k = np.arange(N, dtype=np.float32)[None, :]
    dtf = np.float32(dt)
    traj[:, :, 0] = des[:, None, 3]
    traj[:, :, 1] = des[:, None, 4]
    traj[:, :, 2] = des[:, None, 5] + k * dtf * des[:, None, 11]
    traj[:, 0, 2] = rpy[:, 2]
    traj[:, :, 3] = des[:, None, 0] + k * dtf * des[:, None, 6]
    traj[:, :, 4] = des[:, None, 1] + k * dtf * des[:, None, 7]
    traj[:, :, 5] = des[:, None, 2]
    traj[:, :, 8] = des[:, None, 11]
    traj[:, :, 9] = des[:, None, 6]
    traj[:, :, 10] = des[:, None, 7]
    stance = (lg[:, LOG_FORCE + 2:LOG_FORCE + 12:3] > 0).astype(np.uint8)   # [B, 4]
    gait = np.repeat(stance[:, None, :], N, 1).reshape(B, 4 * N)
    return pack_records(lg[:, LOG_POS:LOG_POS + 3], lg[:, LOG_LIN:LOG_LIN + 3],
                        euler_to_quat(rpy), lg[:, LOG_ANG:LOG_ANG + 3], lg[:, LOG_R:LOG_R + 12],
                        traj.reshape(B, 12 * N), gait, rpy=rpy, x_drag=lg[:, LOG_XDRAG])


class LogReplay:
    """Replays B logged streams ([T, B] messages) through the device estimator and solver.

    Per step k = 1..T-1 (one MPC step of the controller): build the records of message k,
    ``cmpc_batch_estimate`` with message k-1 as the previous log (the residual of
    ConvexMPCLocomotion.cpp:639-771, then SolverMPC.cpp:688-811), ``cmpc_batch_solve``. Returns
    the step-0 forces [T-1, B, 12], status [T-1, B] and f_ext(6) [T-1, B, 6] of every step."""

    def __init__(self, solver, logs: np.ndarray, des: np.ndarray, stamps_ns: np.ndarray,
                 dt: float):
        import torch
        self.s, self.torch = solver, torch
        T, B, _ = logs.shape
        if T < 2:
            raise ValueError("replay needs at least two messages per stream")
        self.T, self.B, self.dt = T, B, dt
        N = solver.horizon
        recs = np.stack([records_from_logs(logs[k], des[k], N, dt) for k in range(T)])
        dev = torch.device("cuda")
        self.recs = torch.from_numpy(recs).to(dev)
        self.logs = torch.from_numpy(np.ascontiguousarray(logs, np.float32)).to(dev)
        self.t = (stamps_ns[:, 0] - stamps_ns[0, 0]) * 1e-9
        self.est = torch.zeros((B, 816), dtype=torch.float32, device=dev)

    def run(self):
        torch = self.torch
        T, B, N = self.T, self.B, self.s.horizon
        dev = self.recs.device
        forces = torch.empty((T - 1, B, 12 * N), dtype=torch.float32, device=dev)
        status = torch.empty((T - 1, B), dtype=torch.uint8, device=dev)
        fext6 = torch.empty((T - 1, B, 6), dtype=torch.float32, device=dev)
        for k in range(1, T):
            self.s.estimate(self.est, self.recs[k], logs=self.logs[k - 1],
                            sim_time=float(self.t[k]), fext6=fext6[k - 1])
            self.s.solve(self.recs[k], forces[k - 1], status[k - 1])
        torch.cuda.synchronize()
        return (forces[:, :, :12].cpu().numpy(), status.cpu().numpy(), fext6.cpu().numpy())
