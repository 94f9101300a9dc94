"""BASELINE config 4 on the GPU: 262144 N = 10 instances through parallel.RootPipeline, the path
bench.py --config 4 times.

* world 1 on one MI355X: the records resident on the GPU, cut into 4 pieces and solved in place
  on the current stream. The forces must be bitwise equal to ONE cmpc_batch_solve over the same
  262144 records (every instance is solved by the same kernel whatever the piece), every status
  ok, and 512 sampled instances within 1e-4 of the reference pipeline (restated condensation +
  the reference's own qpOASES, oracle/_ref) run live on the same records.
* world 2 over gloo with the real HIP solve: both ranks share cuda:0, the pipeline's buffers and
  collectives are CPU tensors (gloo), and each piece is staged through the GPU solver. The root's
  gathered forces must equal the world-1 result bitwise. The collectives under RCCL are the same
  calls (parallel.py); the 8-GPU node is the driver's.
"""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT, rel_force_err

pytestmark = pytest.mark.gpu

BATCH = 262144
N = 10
SEED = 0x5EED


@pytest.fixture(scope="module")
def config4(cm):
    solver_mod = importlib.import_module("quad-periodic-mpc_amd.solver")
    solver_mod.load_library()
    prm = cm.make_params(N)
    recs = cm.make_instances(BATCH, N, seed=SEED)
    return prm, recs, solver_mod


def _one_launch(solver_mod, prm, recs_dev):
    s = solver_mod.BatchSolver(prm, max_batch=recs_dev.shape[0])
    try:
        f = torch.empty((recs_dev.shape[0], 12 * N), dtype=torch.float32, device="cuda")
        st = torch.empty(recs_dev.shape[0], dtype=torch.uint8, device="cuda")
        s.solve(recs_dev, f, st)
        torch.cuda.synchronize()
        return f.cpu().numpy(), st.cpu().numpy()
    finally:
        s.close()


def test_root_pipeline_world1_bitwise_and_parity(cm, orc, config4):
    prm, recs, solver_mod = config4
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    recs_dev = torch.from_numpy(recs).cuda()
    # the pipeline launches on the caller's current stream, which must not be the null stream
    # (as bench.py does: one non-default stream per rank)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        f_pipe, st_pipe = _pipeline_world1(par, prm, recs_dev)
    torch.cuda.synchronize()
    assert (st_pipe == 0).all(), np.bincount(st_pipe)
    f_one, st_one = _one_launch(solver_mod, prm, recs_dev)
    assert (st_one == 0).all()
    np.testing.assert_array_equal(f_pipe, f_one)
    if orc.ref_available():
        idx = np.random.default_rng(4).choice(BATCH, 512, replace=False)
        q, st_ref, _ = orc.ref_solve_batch(recs[idx], prm, nthreads=16)
        ok = st_ref == 0
        err = rel_force_err(f_pipe[idx][ok], q[ok])
        print(f"[config4] 512 sampled of {BATCH}: max rel err vs qpOASES {err.max():.2e}")
        assert err.max() <= 1e-4


def _pipeline_world1(par, prm, recs_dev):
    pipe = par.RootPipeline(prm, BATCH, chunks=4, device="cuda")
    try:
        assert pipe.chunks == 4 and pipe.sizes == [BATCH // 4] * 4
        pipe.step(recs_dev)
        torch.cuda.synchronize()
        f_pipe = pipe.forces.cpu().numpy()
        st_pipe = pipe.local_status.cpu().numpy()
        # a second step over the same records reproduces the first bit for bit
        pipe.step(recs_dev)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(pipe.forces.cpu().numpy(), f_pipe)
    finally:
        pipe.close()
    return f_pipe, st_pipe


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path, q):
    try:
        sys.path.insert(0, ROOT)
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        cm = importlib.import_module("quad-periodic-mpc_amd")
        par = importlib.import_module("quad-periodic-mpc_amd.parallel")
        solver_mod = importlib.import_module("quad-periodic-mpc_amd.solver")
        solver_mod.load_library()
        prm = cm.make_params(N)
        recs = torch.from_numpy(cm.make_instances(BATCH, N, seed=SEED)) if rank == 0 else None
        solver = solver_mod.BatchSolver(prm, max_batch=BATCH // 4 + 1)  # root keeps the larger share

        def gpu_piece(r, f, st):   # CPU rows in, CPU rows out, solved on cuda:0
            rd = r.cuda()
            fd = torch.empty((r.shape[0], 12 * N), dtype=torch.float32, device="cuda")
            sd = torch.empty(r.shape[0], dtype=torch.uint8, device="cuda")
            solver.solve(rd, fd, sd)
            torch.cuda.synchronize()
            f.copy_(fd.cpu())
            st.copy_(sd.cpu())

        pipe = par.RootPipeline(prm, BATCH, chunks=4, solve_fn=gpu_piece)
        pipe.step(recs)
        assert (pipe.local_status == 0).all()
        if rank == 0:
            np.save(out_path, pipe.forces.numpy())
        dist.barrier()
        dist.destroy_process_group()
        solver.close()
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent instead of hanging it
        q.put((rank, repr(e)))


def test_root_pipeline_world2_gloo_real_solve(config4, tmp_path):
    import torch.multiprocessing as mp
    prm, recs, solver_mod = config4
    world = 2
    out_path = str(tmp_path / "f_world2.npy")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, out_path, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=240) for _ in range(world))
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert results == {r: "ok" for r in range(world)}, results
    f_one, _ = _one_launch(solver_mod, prm, torch.from_numpy(recs).cuda())
    np.testing.assert_array_equal(np.load(out_path), f_one)


def test_compact_records_expand_on_device_bitwise(cm, config4):
    """cmpc_batch_expand (CMPC_CREC_* -> solve records, trajAll per ConvexMPCLocomotion.cpp:
    554-585) reproduces the generator's records bit for bit at every horizon, and a world-1
    RootPipeline over compact records gives the forces of the full ones."""
    prm, recs, solver_mod = config4
    R = importlib.import_module("quad-periodic-mpc_amd.records")
    par = importlib.import_module("quad-periodic-mpc_amd.parallel")
    for n in (1, 10, 16, 20):
        p = cm.make_params(n)
        full = cm.make_instances(5000, n, seed=61 + n, random_contact_frac=0.5)
        comp = torch.from_numpy(R.compact_records(full, n, p.dt)).cuda()
        out = torch.full((5000, R.record_words(n)), -7.0, dtype=torch.float32, device="cuda")
        s = solver_mod.BatchSolver(p, max_batch=5000)
        try:
            s.expand(comp, out)
            torch.cuda.synchronize()
        finally:
            s.close()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), full.view(np.uint32))
    B = 40000
    comp = torch.from_numpy(R.compact_records(recs[:B], N, prm.dt)).cuda()
    f_one, st_one = _one_launch(solver_mod, prm, torch.from_numpy(recs[:B]).cuda())
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(stream):
        pipe = par.RootPipeline(prm, B, chunks=2, device="cuda", record_format="compact")
        pipe.step(comp)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pipe.forces.cpu().numpy(), f_one)
    np.testing.assert_array_equal(pipe.local_status.cpu().numpy(), st_one)
    pipe.close()
