"""Build the HIP extension in-tree: libcmpc_hip.so (kernels + C ABI) for gfx950.

Plain ``hipcc`` (no torch extension machinery): the library exposes only the C ABI of
``include/cmpc_solver.h`` and is loaded with ctypes.
"""
from __future__ import annotations

import os
import subprocess
import tempfile

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libcmpc_hip.so")
SOURCES = ["cmpc_kernels.hip", "cmpc_abi.cpp"]
HEADERS = ["cmpc_kernels.h", os.path.join("..", "..", "include", "cmpc_solver.h")]
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
    objs = []
    tmpdir = tempfile.mkdtemp(prefix="cmpc_build_")
    for src in SOURCES:
        obj = os.path.join(tmpdir, src + ".o")
        cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
               "-Wno-unused-result", *[f"-D{d}" for d in defines], "-c", os.path.join(CSRC, src),
               "-o", obj]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
        objs.append(obj)
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
