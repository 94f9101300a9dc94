"""Summarise a gpu_profile.sh run (rocprofv3 --kernel-trace --stats + FETCH_SIZE / WRITE_SIZE
passes) into profiles/<tag>/ and profiles/pmc_summary.json (read by bench.py for `traffic`).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so it is doubled;
WRITE_SIZE is taken as is.

usage: python scripts/pmc_summary.py <tag> [--horizon N --batch B]
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import shutil
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    return name.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "").strip()


def counters(path):
    out = defaultdict(list)
    meta = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            out[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[k] = dict(vgpr=int(r["VGPR_Count"]), agpr=int(r["Accum_VGPR_Count"]),
                           sgpr=int(r["SGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                           scratch=int(r["Scratch_Size"]), wg=int(r["Workgroup_Size"]))
    return out, meta


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--batch", type=int, default=65536)
    a = ap.parse_args()
    src = os.path.join(ROOT, "gpurun_out", a.tag)
    dst = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(dst, exist_ok=True)
    for name in ("bench.log", "smoke.log", "pytest_gpu.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            lines = [ln for ln in open(p) if "amdgpu.ids" not in ln]
            open(os.path.join(dst, name), "w").writelines(lines[-40:])
    stats = os.path.join(src, "prof", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
    fetch, meta = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write, meta2 = counters(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    meta.update(meta2)
    kernels = {}
    for (k, c), v in fetch.items():
        if c != "FETCH_SIZE" or "cmpc" not in k:
            continue
        f_kib = sum(v) / len(v)
        w = write.get((k, "WRITE_SIZE"), [0.0])
        w_kib = sum(w) / len(w)
        kernels[k] = dict(fetch_kib_raw=f_kib, write_kib=w_kib,
                          hbm_bytes_per_launch=int(2 * f_kib * 1024 + w_kib * 1024),
                          launches=len(v), **meta.get(k, {}))
    dom = max(kernels, key=lambda k: kernels[k]["hbm_bytes_per_launch"]) if kernels else None
    summary = dict(tag=a.tag, horizon=a.horizon, batch=a.batch, kernels=kernels,
                   dominant=dom,
                   # the roofline's kernel: the 64-lane class (every instance with n <= 64)
                   hbm_bytes_per_launch=kernels.get("cmpc::cmpc_solve_c1_kernel", {}).get(
                       "hbm_bytes_per_launch"),
                   note="FETCH_SIZE x2 (gfx950 half-count of wide reads) + WRITE_SIZE, KiB->B; "
                        "per launch, averaged over the profiled launches")
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    with open(os.path.join(ROOT, "profiles", "pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
