"""Summarise the counter passes of scripts/gpu_pmc_all.sh into profiles/<tag>/pmc_summary.json
and profiles/pmc_summary.json (read by bench.py for `traffic` and `valu_pmc`).

Per case (cfg3: N = 10, cfg5: N = 20 + estimator, n16: N = 16 trot; batch 65536) and per kernel,
averaged over the profiled launches:
  hbm_bytes_per_launch  = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B). MI355X_MICROARCH.md §HBM:
                          FETCH_SIZE counts half the bytes of wide coalesced reads on gfx950;
                          WRITE_SIZE is exact for 16-B-per-lane stores.
  valu_busy             = SQ_ACTIVE_INST_VALU x 4 / (SIMDs x GRBM_GUI_ACTIVE): the fraction of
                          SIMD cycles issuing VALU work during the dispatch (1024 SIMDs; the SQ
                          counters tick per quad-cycle). Concurrent kernels share the window.
  valu_insts_per_wave, lds_insts_per_wave, salu_insts_per_wave, vmem_rd/wr_per_wave
  lds_bank_conflict_frac = SQ_LDS_BANK_CONFLICT / SQ_ACTIVE_INST_LDS
  wait_frac / issue_stall_frac / active_frac = SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
                          SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES (disjoint, sum ~ 1)

usage: python scripts/pmc_collect.py <tag>    (reads gpurun_out/<tag>/<case>/<pass>/)
"""
from __future__ import annotations

import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = {"cfg2": dict(horizon=10, batch=4096, config=2),
         "cfg3": dict(horizon=10, batch=65536, config=3),
         "cfg5": dict(horizon=20, batch=65536, config=5),
         "n16": dict(horizon=16, batch=65536, config=3)}
SIMDS = 1024


def short(name: str) -> str:
    return name.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "").strip()


def read(path):
    vals = defaultdict(list)
    meta = {}
    if not os.path.exists(path):
        return vals, meta
    with open(path) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            if "cmpc" not in k:
                continue
            vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
            meta[k] = dict(vgpr=int(r["VGPR_Count"]), agpr=int(r["Accum_VGPR_Count"]),
                           sgpr=int(r["SGPR_Count"]), lds=int(r["LDS_Block_Size"]),
                           scratch=int(r["Scratch_Size"]), wg=int(r["Workgroup_Size"]),
                           grid=int(r["Grid_Size"]))
    return vals, meta


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    cases = []
    for case, info in CASES.items():
        cdir = os.path.join(src, case)
        if not os.path.isdir(cdir):
            continue
        allv = {}
        meta = {}
        for p in ("fetch", "write", "sq1", "sq2"):
            v, m = read(os.path.join(cdir, p, "run_counter_collection.csv"))
            allv.update(v)
            meta.update(m)
            f = os.path.join(cdir, p, "run_counter_collection.csv")
            if os.path.exists(f):
                shutil.copy(f, os.path.join(dst, f"{case}_{p}_counters.csv"))
        kernels = {}
        for k in sorted({k for k, _ in allv}):
            def avg(c):
                x = allv.get((k, c))
                return sum(x) / len(x) if x else None
            d = dict(meta.get(k, {}))
            fetch, write = avg("FETCH_SIZE"), avg("WRITE_SIZE")
            if fetch is not None and write is not None:
                d["hbm_bytes_per_launch"] = int(2 * fetch * 1024 + write * 1024)
                d["fetch_kib_raw"], d["write_kib"] = fetch, write
            waves = avg("SQ_WAVES")
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_SMEM",
                      "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
                x = avg(c)
                if x is not None and waves:
                    d[c.lower().replace("sq_insts_", "") + "_insts_per_wave"] = round(x / waves, 1)
            if waves:
                d["waves"] = waves
            act_valu, gui = avg("SQ_ACTIVE_INST_VALU"), avg("GRBM_GUI_ACTIVE")
            if act_valu is not None and gui:
                d["valu_busy"] = round(act_valu * 4 / (SIMDS * gui), 4)
            lds_act, conf = avg("SQ_ACTIVE_INST_LDS"), avg("SQ_LDS_BANK_CONFLICT")
            if lds_act and conf is not None:
                d["lds_bank_conflict_frac"] = round(conf / lds_act, 4)
            wc = avg("SQ_WAVE_CYCLES")
            if wc:
                for c, nm in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "issue_stall_frac"),
                              ("SQ_ACTIVE_INST_ANY", "active_frac"),
                              ("SQ_WAIT_INST_LDS", "lds_issue_stall_frac")):
                    x = avg(c)
                    if x is not None:
                        d[nm] = round(x / wc, 4)
            d["pmc_tag"] = tag
            kernels[k] = d
        cases.append(dict(case=case, **info, kernels=kernels))
    summary = dict(tag=tag, cases=cases,
                   note="per launch, averaged over the profiled launches (bench.py --steps 2 "
                        "--warmup 1); HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE; valu_busy = "
                        "SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE)")
    for path in (os.path.join(dst, "pmc_summary.json"), os.path.join(ROOT, "profiles", "pmc_summary.json")):
        with open(path, "w") as f:
            json.dump(summary, f, indent=1)
    for c in cases:
        print(c["case"])
        for k, d in c["kernels"].items():
            print(f"  {k:45s} hbm {d.get('hbm_bytes_per_launch')}  valu_busy {d.get('valu_busy')}  "
                  f"valu/wave {d.get('valu_insts_per_wave')}  lds/wave {d.get('lds_insts_per_wave')} "
                  f"conf {d.get('lds_bank_conflict_frac')} vgpr {d.get('vgpr')} scratch {d.get('scratch')} "
                  f"wait {d.get('wait_frac')} stall {d.get('issue_stall_frac')} act {d.get('active_frac')}")


if __name__ == "__main__":
    main()
