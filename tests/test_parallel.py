"""Multi-rank path on CPU: world_size 2 (and 3) over gloo, exercising the same scatter / gather
code the GPU ranks run over RCCL (quad-periodic-mpc_amd/parallel.py).

The device solve is replaced by a deterministic per-instance function of the record, so the
test checks the sharding and the collectives: each rank gets exactly its contiguous block, and
the gathered rows come back in instance order for uneven block sizes too."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _fake_solve(records, N):
    # per-instance and order-sensitive: row i depends only on record i
    out = records[:, :12 * N] * 2.0 + records[:, 0:1]
    return out.contiguous()


def _worker(rank, world, port, batch, N, q):
    try:
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cm = importlib.import_module("quad-periodic-mpc_amd")
        par = importlib.import_module("quad-periodic-mpc_amd.parallel")
        prm = cm.make_params(N)
        full = torch.from_numpy(cm.make_instances(batch, N, seed=99))
        ss = par.ShardedSolver(prm, batch, solve_fn=lambda r: _fake_solve(r, N))
        a, b = ss.start, ss.stop
        # every rank can regenerate the deterministic batch to check its own block
        local = par.scatter_records(full if rank == 0 else None, batch, full.shape[1])
        assert torch.equal(local, full[a:b])
        forces, status = ss.solve_from_root(full if rank == 0 else None)
        assert status.shape[0] == b - a
        if rank == 0:
            assert torch.equal(forces, _fake_solve(full, N))
        else:
            assert forces is None
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, repr(e)))


@pytest.mark.parametrize("world,batch", [(2, 37), (2, 64), (3, 10), (2, 1)])
def test_scatter_solve_gather_gloo(world, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, 10, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert results == {r: "ok" for r in range(world)}, results


def test_shard_bounds_cover_batch():
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    for batch in (0, 1, 7, 64, 262144, 262145):
        for world in (1, 2, 3, 8):
            bounds = [par.shard_bounds(batch, world, r) for r in range(world)]
            assert bounds[0][0] == 0 and bounds[-1][1] == batch
            assert all(bounds[i][1] == bounds[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in bounds]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        par.shard_bounds(10, 2, 2)


def test_rank_sizes_root_share():
    """RootPipeline's plan: root keeps about root_share times a peer's rows (it solves them where
    they lie), the peers split the rest evenly, the blocks cover the batch in rank order."""
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    share = par.root_share_auto(164, 120)   # N = 10 records, every step's forces, one piece
    assert 1.33 < share < 1.38
    # two pieces: only half the transfer is exposed; compact records move 56 words, not 164
    assert abs(par.root_share_auto(164, 120, 2) - 1 - (share - 1) / 2) < 1e-12
    assert 1.18 < par.root_share_auto(56, 120) < 1.24
    for batch, world in ((262144, 8), (262144, 2), (10007, 3), (5, 4)):
        sizes = par.rank_sizes(batch, world, 0, share)
        assert sum(sizes) == batch and len(sizes) == world
        assert max(sizes[1:]) - min(sizes[1:]) <= 1
        if batch >= 1000:
            assert abs(sizes[0] / sizes[1] - share) < 0.01
        plan, _ = par._chunk_plan(batch, world, 2, 0, share)
        rows = [r for rank in plan for piece in rank for r in range(*piece)]
        assert rows == list(range(batch))
    assert par.rank_sizes(100, 3, 0, 1.0) == par.shard_sizes(100, 3)


def test_issue_order_interleaves():
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    assert par.issue_order(1) == [("scatter", 0), ("gather", 0)]
    assert par.issue_order(3) == [("scatter", 0), ("scatter", 1), ("gather", 0), ("scatter", 2),
                                  ("gather", 1), ("gather", 2)]


def _pipe_worker(rank, world, port, batch, N, chunks, q, record_format="full"):
    try:
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cm = importlib.import_module("quad-periodic-mpc_amd")
        par = importlib.import_module("quad-periodic-mpc_amd.parallel")
        prm = cm.make_params(N)
        full = torch.from_numpy(cm.make_instances(batch, N, seed=7))

        def fn(recs, forces, status):
            forces.copy_(_fake_solve(recs[:, 32:], N))
            status.zero_()

        pipe = par.RootPipeline(prm, batch, chunks=chunks, solve_fn=fn, record_format=record_format)
        held = full
        if record_format == "compact":   # root holds the compact rows; every rank expands its own
            R = importlib.import_module("quad-periodic-mpc_amd.records")
            held = torch.from_numpy(R.compact_records(full.numpy(), N, prm.dt))
            assert pipe.words == R.compact_words(N) and held.shape[1] == pipe.words
        if rank == 0:
            with pytest.raises(RuntimeError):
                pipe.solve_only()   # root holds no records before its first step
        for _ in range(2):
            pipe.step(held if rank == 0 else None)
        if rank == 0:
            assert torch.equal(pipe.forces, _fake_solve(full[:, 32:], N))
        log = pipe.op_log
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, ("ok", log)))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, (repr(e), None)))


@pytest.mark.parametrize("world,chunks", [(3, 3), (2, 4), (3, 4)])
def test_root_pipeline_pairwise_op_order(world, chunks):
    """under the nccl backend the point-to-point batches of a rank pair run in
    issue order, so root and every peer must post theirs in the same sequence. Each rank's op
    log, restricted to one peer, must read scatter/gather by piece in the same order on both
    sides (world 2 and 3, 3 and 4 pieces), and the gathered forces must be complete."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    batch = 97
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, batch, 10, chunks, q))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v[0] == "ok" for v in results.values()), results
    root_log = results[0][1]
    for peer in range(1, world):
        root_seq = [(k, c) for k, c, peers in root_log if peer in peers]
        peer_seq = [(k, c) for k, c, peers in results[peer][1] if 0 in peers]
        assert root_seq == peer_seq, (peer, root_seq, peer_seq)
        assert len(peer_seq) == 2 * chunks


@pytest.mark.parametrize("world,chunks", [(2, 1), (3, 2)])
def test_root_pipeline_compact_records(world, chunks):
    """record_format="compact": root sends each peer the compact rows (trajAll's step-0 row, 56
    words at N = 10 instead of 164) and every rank expands its own rows before the solve
    (records.expand_records here, cmpc_batch_expand on a GPU): the gathered rows equal those of
    the full records."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, 101, 10, chunks, q, "compact"))
             for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    assert all(v[0] == "ok" for v in results.values()), results


def test_compact_records_roundtrip(cm):
    """compact_records / expand_records: the generator's records (trajAll built as
    ConvexMPCLocomotion.cpp:554-585 builds it) survive the round trip bit for bit at every
    horizon; a record whose trajectory is not that expansion is refused."""
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    for N in (1, 5, 10, 16, 20):
        recs = cm.make_instances(257, N, seed=31 + N, random_contact_frac=0.5)
        c = R.compact_records(recs, N, 0.026)
        assert c.shape == (257, R.compact_words(N))
        back = R.expand_records(c, N, 0.026)
        np.testing.assert_array_equal(back.view(np.uint32), recs.view(np.uint32))
    bad = recs.copy()
    bad[3, R.REC_HDR + 12 * 4 + 5] += 0.01        # a height that is not the step-0 row's
    with pytest.raises(ValueError):
        R.compact_records(bad, 20, 0.026)

