"""CPU baseline probe on the GPU box's host: CPU model, the reference pipeline's per-call
latency on one core (naive and register-tiled condensation) and the stage split at N = 10."""
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as orc  # noqa: E402

cm = importlib.import_module("quad-periodic-mpc_amd")
print([l.strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0])
flags = [l for l in open("/proc/cpuinfo") if l.startswith("flags")][0]
print("avx512f" in flags, "avx2" in flags, "affinity", len(os.sched_getaffinity(0)))
for N in (10, 16, 20):
    prm = cm.make_params(N)
    recs = cm.make_instances(256, N)
    for impl in (0, 1):
        orc.ref_solve_batch(recs[:16], prm, nthreads=1, impl=impl)
        t = time.perf_counter()
        orc.ref_solve_batch(recs, prm, nthreads=1, impl=impl)
        print(f"N={N} impl {impl}: {(time.perf_counter() - t) / 256 * 1e6:.1f} us per call, 1 core", flush=True)
    for th in (16, 64):
        r = cm.make_instances(4096, N)
        t = time.perf_counter()
        orc.ref_solve_batch(r, prm, nthreads=th, impl=1)
        print(f"N={N} impl 1, {th} threads: {4096 / (time.perf_counter() - t):.0f} QP/s", flush=True)
