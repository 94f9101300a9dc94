"""Build the HIP extension in-tree: libcmpc_hip.so (kernels + C ABI) for gfx950.

Plain ``hipcc`` (no torch extension machinery): the library exposes only the C ABI of
``include/cmpc_solver.h`` and is loaded with ctypes. Each translation unit is compiled in
parallel into ``build/obj`` and recompiled only when it or a header it includes changed (the
fully unrolled register kernels take minutes per TU).
"""
from __future__ import annotations

import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libcmpc_hip.so")
OBJ = os.path.join(ROOT, "build", "obj")
# one translation unit per kernel family so the large unrolled kernels compile in parallel
SOURCES = ["cmpc_tail.hip", "cmpc_wide_w256.hip", "cmpc_wide_w192.hip", "cmpc_class1.hip", "cmpc_wide_w80.hip", "cmpc_wide_w96.hip",
           "cmpc_wide_w120.hip", "cmpc_wide_w128.hip", "cmpc_wide_w144.hip", "cmpc_wide_w80p.hip",
           "cmpc_wide_w96p.hip", "cmpc_wide_w120p.hip", "cmpc_wide_w128p.hip", "cmpc_wide_w80r.hip",
           "cmpc_wide_w96r.hip", "cmpc_wide_w120r.hip", "cmpc_wide_w80pr.hip", "cmpc_wide_w96pr.hip",
           "cmpc_wide_w120pr.hip", "cmpc_condense.hip", "cmpc_launch.hip", "cmpc_estimator.hip", "cmpc_assemble.hip",
           "cmpc_admm.hip", "cmpc_quadprog.hip", "cmpc_abi.cpp"]
ARCH = os.environ.get("CMPC_OFFLOAD_ARCH", "gfx950")
# -fno-slp-vectorize: the SLP pass packs adjacent row updates into v_pk_fma_f32, which ties
# slot registers into 64-bit pairs and made the register-resident rows spill
# -ffp-contract=on: multiply-adds fuse only inside one source expression (clang's front end emits
# llvm.fmuladd), never across statements in the back end, so a kernel body rounds the same in
# every launch form it is inlined into (the one-per-entry and persistent wide builds, the
# single-instance path); with `fast` the back end fused differently per form and the same record
# could get different forces in batches of different sizes
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-result", "-fno-slp-vectorize", "-ffp-contract=on"]


def _deps(path: str, seen=None) -> set:
    """The file plus every quoted #include it pulls in, recursively."""
    seen = set() if seen is None else seen
    path = os.path.normpath(path)
    if path in seen or not os.path.exists(path):
        return seen
    seen.add(path)
    for inc in re.findall(r'#include\s+"([^"]+)"', open(path).read()):
        _deps(os.path.join(os.path.dirname(path), inc), seen)
    return seen


def _obj(src: str, defines: tuple) -> str:
    tag = ("_" + "_".join(d.replace("=", "-") for d in defines)) if defines else ""
    return os.path.join(OBJ, f"{src}{tag}.o")


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False, out: str | None = None,
          defines: tuple = ()) -> str:
    lib = out or LIB
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    os.makedirs(OBJ, exist_ok=True)

    def compile_one(src: str) -> str:
        path = os.path.join(CSRC, src)
        obj = _obj(src, defines)
        if not force and not _stale(obj, _deps(path)):
            return obj
        cmd = [hipcc, f"--offload-arch={ARCH}", *FLAGS, *[f"-D{d}" for d in defines], "-c", path,
               "-o", obj + ".tmp"]
        if src.endswith(".cpp"):
            cmd[1:1] = ["-x", "hip"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(obj + ".tmp", obj)
        return obj

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    if not force and not _stale(lib, objs):
        return lib
    tmp = lib + ".tmp"
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs,
                   check=True)
    os.replace(tmp, lib)
    if out is None:
        build_tools(lib)
        build_multi(lib)
    return lib


MULTI_LIB = os.path.join(PKG, "libcmpc_multi.so")


def build_multi(lib: str = LIB) -> str:
    """libcmpc_multi.so (include/cmpc_multi.h): the config-4 sharding over RCCL as a C ABI, linked
    against libcmpc_hip.so and librccl; plus its C++ test caller cmpc_multi_test."""
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    src = os.path.join(CSRC, "cmpc_multi.cpp")
    hdrs = [os.path.join(ROOT, "include", h) for h in ("cmpc_multi.h", "cmpc_solver.h")]
    if _stale(MULTI_LIB, [src, lib] + hdrs):
        subprocess.run([hipcc, "-x", "hip", "--offload-arch=" + ARCH, "-O2", "-std=c++17", "-fPIC",
                        "-Wall", "-shared", "-o", MULTI_LIB + ".tmp", src, f"-L{PKG}", "-lcmpc_hip",
                        "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{PKG}",
                        "-Wl,-rpath,/opt/rocm/lib"], check=True)
        os.replace(MULTI_LIB + ".tmp", MULTI_LIB)
    exe = os.path.join(PKG, "cmpc_multi_test")
    tsrc = os.path.join(CSRC, "tools", "cmpc_multi_test.cpp")
    if _stale(exe, [tsrc, MULTI_LIB] + hdrs):
        subprocess.run([hipcc, "-x", "hip", "--offload-arch=" + ARCH, "-O2", "-std=c++17", "-o", exe + ".tmp",
                        tsrc, f"-L{PKG}", "-lcmpc_multi", "-lcmpc_hip", "-Wl,-rpath,$ORIGIN",
                        f"-Wl,-rpath,{PKG}"], check=True)
        os.replace(exe + ".tmp", exe)
    return MULTI_LIB


def build_tools(lib: str = LIB) -> str:
    """cmpc_abi_latency: a plain C++ caller of the reference ABI, linked against the library
    the way the be2r controller links it (only include/cmpc_solver.h)."""
    exe = os.path.join(PKG, "cmpc_abi_latency")
    src = os.path.join(CSRC, "tools", "cmpc_abi_latency.cpp")
    if not _stale(exe, [src, lib]):
        return exe
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe + ".tmp", src, f"-L{PKG}", "-lcmpc_hip",
                    f"-Wl,-rpath,$ORIGIN", f"-Wl,-rpath,{PKG}"], check=True)
    os.replace(exe + ".tmp", exe)
    return exe


if __name__ == "__main__":
    import sys
    print(build(force="--force" in sys.argv, verbose=True))
