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
