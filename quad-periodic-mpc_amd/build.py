"""Build the HIP extension in-tree: libcmpc_hip.so (kernels + C ABI) for gfx950.

Plain ``hipcc`` (no torch extension machinery): the library exposes only the C ABI of
``include/cmpc_solver.h`` and is loaded with ctypes.
"""
from __future__ import annotations

import os
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libcmpc_hip.so")
# one translation unit per size class so the (large, fully unrolled) kernels compile in parallel
SOURCES = ["cmpc_class1.hip", "cmpc_class2.hip", "cmpc_condense.hip", "cmpc_launch.hip",
           "cmpc_abi.cpp"]
HEADERS = ["cmpc_kernels.h", "cmpc_device.h", os.path.join("..", "..", "include", "cmpc_solver.h")]
ARCH = os.environ.get("CMPC_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(os.path.join(CSRC, f)) > t for f in SOURCES + HEADERS)


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: tuple = ()) -> str:
    lib = out or LIB
    if not force and out is None and not _stale():
        return LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    tmpdir = tempfile.mkdtemp(prefix="cmpc_build_")

    def compile_one(src: str) -> str:
        obj = os.path.join(tmpdir, src + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-result", *[f"-D{d}" for d in defines], "-c", os.path.join(CSRC, src),
               "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = lib + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.run(cmd, check=True)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    os.rmdir(tmpdir)
    return lib


if __name__ == "__main__":
    print(build(force=True, verbose=True))
