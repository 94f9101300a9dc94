"""Where class-1 wavefronts run and for how long: a CMPC_PLACE_PROF build of the library records
per instance the hardware wave id (SE / SH / CU / SIMD / wave slot), the XCC and the wall-clock
start / end of its wavefront. For each batch size this prints how many CUs / SIMDs were used,
the waves per SIMD at the busiest moment, the per-wave latency distribution and the makespan.

  CMPC_LIB=variants/libplace.so python scripts/place_prof.py [--horizon 10] [--batches 256,4096]
(build the variant: scripts/build_diag_variant.sh variants/libplace.so cmpc_class1.hip -DCMPC_PLACE_PROF)
"""
import argparse
import ctypes
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def decode(hw):
    """gfx9 HW_REG_HW_ID: wave[3:0] simd[5:4] pipe[7:6] cu[11:8] sh[12] se[15:13]."""
    return {"wave": hw & 0xF, "simd": (hw >> 4) & 3, "cu": (hw >> 8) & 0xF, "sh": (hw >> 12) & 1,
            "se": (hw >> 13) & 7}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--horizon", type=int, default=10)
    ap.add_argument("--batches", default="256,1024,4096,16384,65536")
    ap.add_argument("--random-contact-frac", type=float, default=0.0)
    a = ap.parse_args()
    import torch
    cm = importlib.import_module("quad-periodic-mpc_amd")
    sm = importlib.import_module("quad-periodic-mpc_amd.solver")
    lib = sm.load_library()
    fn = lib.cmpc_debug_place_read
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    N = a.horizon
    batches = [int(x) for x in a.batches.split(",")]
    B = max(batches)
    recs = torch.from_numpy(cm.make_instances(B, N, random_contact_frac=a.random_contact_frac)).cuda()
    prm = cm.make_params(N)
    torch.cuda.set_stream(torch.cuda.Stream())
    s = sm.BatchSolver(prm, max_batch=B, stream=torch.cuda.current_stream())
    f = torch.empty((B, 12 * N), device="cuda")
    st = torch.empty(B, dtype=torch.uint8, device="cuda")
    it = torch.empty(B, dtype=torch.int32, device="cuda")
    for b in batches:
        for _ in range(3):
            s.solve(recs[:b], f[:b], st[:b], it[:b])
        torch.cuda.synchronize()
        buf = np.zeros((b, 4), np.uint32)
        assert fn(buf.ctypes.data, b) == 0
        hw, xcc, t0, t1 = buf[:, 0].astype(np.int64), buf[:, 1] & 0xF, buf[:, 2].astype(np.int64), buf[:, 3].astype(np.int64)
        t0 = t0 - t0.min()
        t1 = t1 - buf[:, 2].astype(np.int64).min()
        d = decode(hw)
        cu_key = xcc * 1024 + d["se"] * 64 + d["sh"] * 16 + d["cu"]
        simd_key = cu_key * 4 + d["simd"]
        lat = (t1 - t0) * 10e-3  # 100 MHz ticks -> us
        # busiest SIMD: max concurrent waves (sweep over start/end events)
        conc = 0
        for k in np.unique(simd_key)[:4096]:
            m = simd_key == k
            ev = np.concatenate([np.stack([t0[m], np.ones(m.sum())], 1), np.stack([t1[m], -np.ones(m.sum())], 1)])
            ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
            conc = max(conc, int(np.cumsum(ev[:, 1]).max()))
        per_cu = np.bincount(np.unique(cu_key, return_inverse=True)[1])
        per_xcc = np.bincount(xcc, minlength=8)
        print(f"batch {b:6d}: CUs {len(np.unique(cu_key)):4d}  SIMDs {len(np.unique(simd_key)):5d}  "
              f"waves/CU min/med/max {per_cu.min()}/{int(np.median(per_cu))}/{per_cu.max()}  "
              f"max concurrent waves/SIMD {conc}  per XCC {per_xcc.tolist()}  "
              f"wave latency us p10/p50/p90/max {np.percentile(lat, 10):.1f}/{np.percentile(lat, 50):.1f}/"
              f"{np.percentile(lat, 90):.1f}/{lat.max():.1f}  makespan {t1.max() * 10e-3:.1f} us  "
              f"last start {t0.max() * 10e-3:.1f} us", flush=True)
        its = it[:b].cpu().numpy()
        row = []
        for k in range(0, min(its.max(), 40) + 1):
            m = its == k
            if m.sum() >= 4:
                row.append(f"{k}:{m.sum()}@{np.median(lat[m]):.0f}")
        print("    iters:count@median-latency-us  " + " ".join(row), flush=True)
    s.close()


if __name__ == "__main__":
    main()
