"""Multi-GPU sharding of a batch of independent MPC instances.

Every instance is one ``solve_mpc`` call (``SolverMPC.cpp:566-982``) with no data shared between
instances, so a batch shards into contiguous per-rank blocks and the solve itself needs no
exchange step. One process per GPU over ``torch.distributed``: backend ``"nccl"`` is RCCL on
ROCm (xGMI between the GPUs of a node), ``"gloo"`` runs the same code on CPU tensors (tests).

The only collectives are the optional ones around the solve, for callers whose records live on
ONE rank (the driver of a simulation farm, say):

* :func:`scatter_records` — root's ``[B, W]`` records → each rank's contiguous block
  (one ``scatter``; blocks padded to the largest block for the collective, trimmed after);
* :func:`gather_forces` — each rank's ``[b, 12N]`` forces (or any per-instance rows) → root's
  ``[B, 12N]`` (one ``gather``).

At B = 262144, N = 10 that is ≈21 MB of records and ≈16 MB of forces per peer, against tens of
milliseconds of solve per GPU; callers that generate their instances per rank skip both.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist


def shard_bounds(batch: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block ``[start, stop)`` of ``rank``; the first ``batch % world`` ranks take one
    extra instance, so block sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    if batch < 0:
        raise ValueError("negative batch")
    base, extra = divmod(batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def shard_sizes(batch: int, world: int) -> list[int]:
    return [b - a for a, b in (shard_bounds(batch, world, r) for r in range(world))]


def _group_info(group):
    if not dist.is_available() or not dist.is_initialized():
        return 1, 0          # single process: no collectives
    return dist.get_world_size(group), dist.get_rank(group)


def scatter_records(records: Optional[torch.Tensor], batch: int, row_words: int, *,
                    src: int = 0, group=None, device=None, dtype=torch.float32) -> torch.Tensor:
    """Root ``src`` holds ``records`` [batch, row_words]; every rank returns its block.

    Non-root ranks pass ``records=None``. One ``scatter`` collective of ``world`` equal-size
    chunks (the largest block; the short blocks are zero-padded, then trimmed)."""
    world, rank = _group_info(group)
    sizes = shard_sizes(batch, world)
    chunk = max(sizes) if sizes else 0
    out = torch.empty((chunk, row_words), dtype=dtype, device=device)
    scatter_list = None
    if rank == src:
        if records is None or tuple(records.shape) != (batch, row_words):
            raise ValueError(f"root must pass records of shape ({batch}, {row_words})")
        scatter_list = []
        for r in range(world):
            a, b = shard_bounds(batch, world, r)
            blk = records[a:b].to(device=device, dtype=dtype)
            if b - a < chunk:
                pad = torch.zeros((chunk - (b - a), row_words), dtype=dtype, device=device)
                blk = torch.cat([blk, pad], 0)
            scatter_list.append(blk.contiguous())
    dist.scatter(out, scatter_list, src=src, group=group)
    return out[:sizes[rank]]


def gather_forces(local: torch.Tensor, batch: int, *, dst: int = 0,
                  group=None) -> Optional[torch.Tensor]:
    """Inverse of :func:`scatter_records` for per-instance output rows: root ``dst`` returns the
    full ``[batch, cols]`` array in instance order, other ranks return ``None``."""
    world, rank = _group_info(group)
    sizes = shard_sizes(batch, world)
    if local.shape[0] != sizes[rank]:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, its block has {sizes[rank]}")
    chunk = max(sizes) if sizes else 0
    cols = local.shape[1]
    send = local
    if local.shape[0] < chunk:
        pad = torch.zeros((chunk - local.shape[0], cols), dtype=local.dtype, device=local.device)
        send = torch.cat([local, pad], 0)
    send = send.contiguous()
    gather_list = None
    if rank == dst:
        gather_list = [torch.empty_like(send) for _ in range(world)]
    dist.gather(send, gather_list, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([g[:s] for g, s in zip(gather_list, sizes)], 0)


class ShardedSolver:
    """One rank's share of a batched solve: its contiguous block of the global batch on its own
    GPU (``BatchSolver`` over the C ABI), plus the optional root scatter / gather.

    ``solve_fn`` replaces the device solve (``records -> forces``); tests use it to exercise the
    collectives on CPU ranks. Left ``None``, the HIP solver runs and there is no fallback."""

    def __init__(self, params, global_batch: int, *, group=None, device=None,
                 solve_fn: Optional[Callable[[torch.Tensor], torch.Tensor]] = None):
        self.params = params
        self.global_batch = int(global_batch)
        self.group = group
        self.world, self.rank = _group_info(group)
        self.start, self.stop = shard_bounds(self.global_batch, self.world, self.rank)
        self.local_batch = self.stop - self.start
        self.device = device
        self._solve_fn = solve_fn
        self._solver = None
        if solve_fn is None:
            import importlib
            solver_mod = importlib.import_module(__package__ + ".solver")
            self._solver = solver_mod.BatchSolver(params, max_batch=max(1, self.local_batch))

    def solve_local(self, records: torch.Tensor):
        """Solve this rank's block (device tensors) -> (forces [b, 12N], status [b])."""
        N = self.params.horizon
        b = records.shape[0]
        if self._solve_fn is not None:
            forces = self._solve_fn(records)
            return forces, torch.zeros(b, dtype=torch.uint8, device=forces.device)
        forces = torch.empty((b, 12 * N), dtype=torch.float32, device=records.device)
        status = torch.empty(b, dtype=torch.uint8, device=records.device)
        # the solver runs on its own stream: order it after whatever produced `records`
        # (e.g. the scatter) and order torch's stream after the solve
        solver_stream = torch.cuda.ExternalStream(self._solver.stream_handle, device=records.device)
        solver_stream.wait_stream(torch.cuda.current_stream(records.device))
        self._solver.solve(records, forces, status)
        torch.cuda.current_stream(records.device).wait_stream(solver_stream)
        return forces, status

    def solve_from_root(self, records_root: Optional[torch.Tensor], src: int = 0):
        """Root scatter -> per-rank solve -> gather to root. Returns the full forces on
        ``src`` (None elsewhere) and this rank's status block."""
        from .records import record_words
        words = record_words(self.params.horizon)
        local = scatter_records(records_root, self.global_batch, words, src=src,
                                group=self.group, device=self.device)
        forces, status = self.solve_local(local)
        return gather_forces(forces, self.global_batch, dst=src, group=self.group), status

    def close(self):
        if self._solver is not None:
            self._solver.close()
            self._solver = None


# Smallest pipeline piece worth cutting. Every solve ends in a tail (its slowest instances, the
# wide size classes) that a piece pays again; measured on one MI355X (round 5, the bench's
# scaling model, profiles/r05_w/bench.log): 32768 instances in one solve 0.91 ms, in two pieces of
# 16384 1.31 ms; 65536 in one 1.47 ms, in two pieces 2.31 ms. The xGMI time a second piece could
# hide at 8 ranks (~0.14 ms of scatter per step) is far less than the ~0.4 ms it costs, so pieces
# stay at >= 65536 instances.
MIN_PIECE = 65536
MAX_CHUNKS = 4


def auto_chunks(local_batch: int, world: int = 2, min_piece: int = MIN_PIECE,
                max_chunks: int = MAX_CHUNKS) -> int:
    """Pieces per rank for the config-4 pipeline: one when there is no traffic to hide (world
    1: 262144 records in one solve 5.4 ms on one MI355X, round 5; in four pieces ~12 % more,
    round 4), else as many
    as keep every piece >= ``min_piece`` instances, at most ``max_chunks`` (262144 over 1 / 2 /
    4 / 8 ranks -> 1 / 2 / 1 / 1)."""
    if world <= 1:
        return 1
    return max(1, min(max_chunks, local_batch // max(1, min_piece)))


# Root's share of the batch (RootPipeline): root solves its own rows where they lie, while every
# other rank's rows first cross one xGMI link and their forces cross back. With C pieces per rank
# only the first piece's records and the last piece's forces are exposed on a peer (the rest
# overlaps the solve), so balancing the ranks' finishing times gives root
# 1 + (bytes moved per instance) / (C x ROOT_EQUIV_BYTES) times a peer's rows. ROOT_EQUIV_BYTES is
# what one link (153 GB/s per direction) carries in the marginal solve time of one instance at
# N = 10: 21 ns between 59192 and 84568 instances on one MI355X (the round-5 scaling model rows,
# BENCH_r05.json). Round 5 used 2650 B and no 1 / C: 2 and 4 ranks were root-bound.
ROOT_EQUIV_BYTES = 3213.0


def root_share_auto(record_words: int, cols: int, chunks: int = 1) -> float:
    return 1.0 + 4.0 * (record_words + cols) / (max(1, chunks) * ROOT_EQUIV_BYTES)


def rank_sizes(batch: int, world: int, src: int = 0, root_share: float = 1.0) -> list[int]:
    """Rows per rank: root ``src`` about ``root_share`` times a peer's, the peers within one of
    each other (root_share 1: :func:`shard_sizes`)."""
    if world <= 1 or root_share == 1.0:
        return shard_sizes(batch, world)
    peer = int(batch // (world - 1 + root_share))
    root = batch - peer * (world - 1)
    sizes = [peer] * world
    sizes[src] = root
    return sizes


def _chunk_plan(batch: int, world: int, chunks: int, src: int = 0, root_share: float = 1.0):
    """Per rank r and chunk c: rows [a_rc, b_rc) of the global batch (contiguous rank blocks of
    :func:`rank_sizes`, each split into ``chunks`` contiguous pieces), and S_c = the largest
    piece c over ranks (the solver handles' capacity)."""
    sizes_r = rank_sizes(batch, world, src, root_share)
    plan, a = [], 0
    for r in range(world):
        b = a + sizes_r[r]
        plan.append([(a + lo, a + hi) for lo, hi in
                     (shard_bounds(b - a, chunks, c) for c in range(chunks))])
        a = b
    sizes = [max(plan[r][c][1] - plan[r][c][0] for r in range(world)) for c in range(chunks)]
    return plan, sizes


def issue_order(chunks: int) -> list[tuple[str, int]]:
    """The order in which every rank posts RootPipeline's point-to-point batches for one step:
    scatter 0, scatter 1, gather 0, scatter 2, gather 1, ..., gather C-1. Root and each peer post
    the SAME sequence: under the nccl backend every ``batch_isend_irecv`` is queued in issue order
    on one communication stream and a large send completes only once its receive is posted, so a
    pair of ranks that posted these in different orders could each wait on the other's later op
    (root posting every scatter before any gather deadlocks from three pieces)."""
    order = [("scatter", 0)] if chunks > 0 else []
    for c in range(chunks):
        if c + 1 < chunks:
            order.append(("scatter", c + 1))
        order.append(("gather", c))
    return order


class RootPipeline:
    """BASELINE config 4 / SURVEY.md §8(e): the records of the whole batch live on root ``src``;
    one :meth:`step` scatters them over the ranks (RCCL over xGMI under the ``nccl`` backend),
    solves every rank's contiguous shard on its own GPU and gathers the forces back to root.

    The transfers are point-to-point (``batch_isend_irecv``: root sends each peer its rows and
    receives its forces straight into :attr:`forces`, no staging or padding). Root solves its own
    rows where they lie, without waiting for any transfer, so it takes ``root_share`` times a
    peer's rows (default :func:`root_share_auto`: the ranks then finish together).

    The shard of every rank is cut into ``chunks`` pieces (default :func:`auto_chunks`) and the
    three stages are software-pipelined: the transfers run on the process group's
    communication stream, the solve on the caller's current stream, so piece c+1 is in flight
    over xGMI while piece c is being solved and piece c-1 is being gathered. Issue order per step
    (communication stream, :func:`issue_order`, the same on every rank): scatter 0, scatter 1,
    gather 0, scatter 2, gather 1, ... — a gather never delays the next piece's scatter.

    ``solve_fn(records, forces, status)`` solves rows in place (device tensors of this rank).
    The default solves the pieces on ``lanes`` (two) :class:`BatchSolver` handles, each on its
    own stream, alternating: piece c + 1's solve (its class-1 launch) starts while piece c's
    slowest instances (the wide size classes) are still running, instead of queueing behind
    piece c's join, and piece c's gather waits for piece c's solve only. Each handle has its own
    work lists, so the overlapping solves never share scratch; every piece is still solved by
    the same kernels, so the forces are bitwise those of one solve. Every buffer is allocated
    here, none inside :meth:`step`."""

    LANES = 2   # solver handles (streams) the pieces alternate over

    def __init__(self, params, global_batch: int, chunks: Optional[int] = None, *, group=None,
                 device=None, src: int = 0, solve_fn=None, record_words: Optional[int] = None,
                 lanes: Optional[int] = None, out_steps: int = 0,
                 root_share: Optional[float] = None, record_format: str = "full"):
        from .records import compact_words, record_words as _rw
        self.params = params
        self.N = params.horizon
        if record_format not in ("full", "compact"):
            raise ValueError(f"record_format {record_format!r}: 'full' or 'compact'")
        # "compact": root holds and sends compact records (include/cmpc_solver.h CMPC_CREC_*: trajAll's
        # step-0 row instead of trajAll, 224 B instead of 656 B at N = 10); every rank expands its
        # rows on its own GPU (cmpc_batch_expand) before solving them
        self.compact = record_format == "compact"
        self.full_words = _rw(self.N)
        self.words = record_words or (compact_words(self.N) if self.compact else self.full_words)
        self.batch = int(global_batch)
        self.group = group
        self.src = src
        self.world, self.rank = _group_info(group)
        # forces kept per instance: every step (12 N) or, with out_steps, the leading steps only
        # (cmpc_batch_set_output_steps: a caller of get_solution(0..11) gathers 48 B, not 480 B)
        self.out_steps = int(out_steps) if 0 < int(out_steps) < self.N else 0
        cols = 12 * (self.out_steps or self.N)
        self.cols = cols
        if chunks is None:   # adaptive: pieces of >= MIN_PIECE instances (auto_chunks)
            chunks = auto_chunks(max(shard_sizes(self.batch, self.world)), self.world)
        self.chunks = max(1, min(int(chunks), max(1, self.batch // max(1, self.world))))
        if root_share is None:
            root_share = root_share_auto(self.words, cols, self.chunks) if self.world > 1 else 1.0
        self.root_share = float(root_share)
        self.plan, self.sizes = _chunk_plan(self.batch, self.world, self.chunks, src, self.root_share)
        self.start, self.stop = self.plan[self.rank][0][0], self.plan[self.rank][-1][1]
        self.local_batch = self.stop - self.start
        self.device = device
        dev = device
        # this rank's rows: records in, forces / status out (chunk c = rows of plan[rank][c])
        self._last_root = None
        # (kind, piece, peers) of every point-to-point batch this rank posted, in order (tests
        # check that root and each peer post theirs in the same order; bounded to the last step)
        self.op_log: list[tuple[str, int, tuple[int, ...]]] = []
        # root (and world 1) solves its rows where they lie, into its rows of `forces`: no copies
        is_root = self.rank == src
        self.forces = (torch.zeros((self.batch, cols), dtype=torch.float32, device=dev)
                       if is_root else None)
        self.local_recs = torch.zeros((0 if is_root else self.local_batch, self.words),
                                      dtype=torch.float32, device=dev)
        self.local_forces = (self.forces[self.start:self.stop] if is_root else
                             torch.zeros((self.local_batch, cols), dtype=torch.float32, device=dev))
        self.local_status = torch.zeros(self.local_batch, dtype=torch.uint8, device=dev)
        # compact format: this rank's rows expanded into solve records before each piece's solve
        self.full_recs = (torch.zeros((self.local_batch, self.full_words), dtype=torch.float32, device=dev)
                          if self.compact else None)
        self._solve_fn = solve_fn
        self._solver = None
        self._solvers = []
        self._streams = []
        if solve_fn is None:
            import importlib
            solver_mod = importlib.import_module(__package__ + ".solver")
            nl = max(1, min(self.LANES if lanes is None else int(lanes), self.chunks))
            if nl == 1:   # one lane: the caller's stream itself (no fork / join)
                self._solvers = [solver_mod.BatchSolver(params, max_batch=max(1, max(self.sizes)),
                                                        stream=torch.cuda.current_stream(dev))]
            else:
                self._streams = [torch.cuda.Stream(dev) for _ in range(nl)]
                self._solvers = [solver_mod.BatchSolver(params, max_batch=max(1, max(self.sizes)), stream=st)
                                 for st in self._streams]
            for sv in self._solvers:
                if self.out_steps:
                    sv.set_output_steps(self.out_steps)
            self._solver = self._solvers[0]

    def _lane(self, c):
        """(solver, stream) of piece c: stream None means the caller's current stream (one lane,
        or a solve_fn)."""
        if not self._solvers:
            return None, None
        k = c % len(self._solvers)
        return self._solvers[k], (self._streams[k] if self._streams else None)

    def enable_timing(self, steps: int) -> None:
        """Per-launch HIP events on every handle for the next ``steps`` solves of each."""
        for sv in self._solvers:
            sv.enable_timing(steps)

    def read_timing(self):
        """(ms [solves, 2] over all handles, wide-class count of handle 0's last solve)."""
        import numpy as np
        if not self._solvers:
            return np.zeros((0, 2)), 0
        parts = [sv.read_timing() for sv in self._solvers]
        return np.concatenate([p[0] for p in parts], 0), parts[0][1]

    def _local(self, c):
        a, b = self.plan[self.rank][c]
        return a - self.start, b - self.start

    def _solve_piece(self, c, recs=None, forces=None, status=None):
        """Solve piece c (this rank's rows of it, or the given rows) on its lane: the lane's
        stream is the current one when this runs (step / solve_only arrange that)."""
        a, b = self._local(c)
        if b <= a:
            return
        if recs is None and self.rank == self.src:  # root: its rows of the records it holds
            recs = self._last_root[self.start + a:self.start + b]
        recs = self.local_recs[a:b] if recs is None else recs
        forces = self.local_forces[a:b] if forces is None else forces
        status = self.local_status[a:b] if status is None else status
        if self.compact:   # trajAll from its step-0 row, on this rank's GPU (cmpc_batch_expand)
            full = self.full_recs[a:b]
            if self._solve_fn is not None:
                from .records import expand_records
                full.copy_(torch.from_numpy(expand_records(recs.cpu().numpy(), self.N, self.params.dt)))
            else:
                self._lane(c)[0].expand(recs, full)
            recs = full
        if self._solve_fn is not None:
            self._solve_fn(recs, forces, status)
        else:
            self._lane(c)[0].solve(recs, forces, status)

    def _fork(self):
        """Every lane stream waits for the caller's stream (inputs ready, earlier work done)."""
        cur = torch.cuda.current_stream(self.device) if self._streams else None
        for st in self._streams:
            st.wait_stream(cur)
        return cur

    def _join(self, cur):
        for st in self._streams:
            cur.wait_stream(st)

    def _p2p(self, kind, c, ops):
        self.op_log.append((kind, c, tuple(op.peer for op in ops)))
        return dist.batch_isend_irecv(ops) if ops else []

    def _scatter(self, records_root, c):
        """Piece c's records to the peers (root: one send per peer; a peer: one receive)."""
        if self.rank == self.src:
            ops = [dist.P2POp(dist.isend, records_root[ra:rb], self._peer(r), self.group)
                   for r, (ra, rb) in ((r, self.plan[r][c]) for r in range(self.world))
                   if r != self.src and rb > ra]
        else:
            a, b = self._local(c)
            ops = ([dist.P2POp(dist.irecv, self.local_recs[a:b], self._peer(self.src), self.group)]
                   if b > a else [])
        return self._p2p("scatter", c, ops)

    def _gather(self, c):
        """Piece c's forces back to root, straight into its rows of `forces`."""
        if self.rank == self.src:
            ops = [dist.P2POp(dist.irecv, self.forces[ra:rb], self._peer(r), self.group)
                   for r, (ra, rb) in ((r, self.plan[r][c]) for r in range(self.world))
                   if r != self.src and rb > ra]
        else:
            a, b = self._local(c)
            ops = ([dist.P2POp(dist.isend, self.local_forces[a:b], self._peer(self.src), self.group)]
                   if b > a else [])
        return self._p2p("gather", c, ops)

    def _peer(self, r):
        """Global rank of group rank r (P2POp takes global ranks)."""
        return r if self.group is None else dist.get_global_rank(self.group, r)

    @staticmethod
    def _wait(works):
        for w in works:
            w.wait()

    def step(self, records_root: Optional[torch.Tensor]) -> None:
        """One pass: scatter -> solve -> gather, pipelined over the chunks. On root the forces of
        the whole batch land in :attr:`forces` (complete once the current stream reaches the
        point after this call)."""
        self._last_root = records_root
        if self.rank == self.src and (records_root is None or
                                      tuple(records_root.shape) != (self.batch, self.words)):
            raise ValueError(f"root must pass records of shape ({self.batch}, {self.words})")
        C = self.chunks
        cur = self._fork()
        if self.world == 1:   # nothing to move: solve the resident records in place
            for c in range(C):
                a, b = self.plan[0][c]
                if b > a:
                    with _on(self._lane(c)[1]):
                        self._solve_piece(c, records_root[a:b], self.forces[a:b], self.local_status[a:b])
            if cur is not None:
                self._join(cur)
            return
        self.op_log = []
        if self.rank == self.src:
            # root: every send and every receive of the peers' forces, posted at once from the
            # caller's stream in issue_order (the order each peer posts its receives and sends:
            # the nccl backend runs them in issue order), so no peer waits for root's own solve;
            # then root solves its rows where they lie
            sc, ga = [None] * C, [None] * C
            for kind, c in issue_order(C):
                if kind == "scatter":
                    sc[c] = self._scatter(records_root, c)
                else:
                    ga[c] = self._gather(c)
            for c in range(C):
                with _on(self._lane(c)[1]):
                    self._solve_piece(c)
            for c in range(C):
                self._wait(ga[c])
                self._wait(sc[c])
            if cur is not None:
                self._join(cur)
            return
        sc = [None] * C
        ga = [None] * C
        for kind, c in issue_order(C):
            if kind == "scatter":
                sc[c] = self._scatter(records_root, c)
                continue
            # on piece c's lane: wait for its records, solve, then send its forces (the send waits
            # for this stream, i.e. for piece c's solve, not for the other lane's)
            with _on(self._lane(c)[1]):
                self._wait(sc[c])
                self._solve_piece(c)
                ga[c] = self._gather(c)
        for c in range(C):
            self._wait(ga[c])
        if cur is not None:
            self._join(cur)

    def solve_only(self) -> None:
        """The same pieces solved with no collective (kernel-only rate of the shard)."""
        if self.rank == self.src and self._last_root is None:
            raise RuntimeError("RootPipeline.solve_only: root holds no records yet (call step first)")
        if self.world == 1:
            return self.step(self._last_root)
        cur = self._fork()
        for c in range(self.chunks):
            with _on(self._lane(c)[1]):
                self._solve_piece(c)
        if cur is not None:
            self._join(cur)

    def close(self):
        for sv in self._solvers:
            sv.close()
        self._solvers = []
        self._solver = None


class _on:
    """``torch.cuda.stream(st)`` when st is a stream, else a no-op (CPU ranks, solve_fn)."""

    def __init__(self, st):
        self.ctx = torch.cuda.stream(st) if st is not None else None

    def __enter__(self):
        if self.ctx is not None:
            self.ctx.__enter__()

    def __exit__(self, *a):
        if self.ctx is not None:
            self.ctx.__exit__(*a)
