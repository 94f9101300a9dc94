"""Per-dispatch timeline from a rocprofv3 --kernel-trace CSV: for the last K occurrences of an
anchor kernel (one per solve step), every kernel dispatched in that step with its start and end
relative to the step's first dispatch, and the step's makespan.

  python scripts/trace_timeline.py <run_kernel_trace.csv> [--anchor cmpc_classify_kernel] [--steps 2]
"""
import argparse
import csv
import re


def short(name):
    m = re.search(r"cmpc_(\w+?)_kernel(<[^>]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "").replace(" ", "")
    return name.split("(")[0][-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="cmpc_classify_kernel")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--gaps", action="store_true",
                    help="one line per step: makespan and the idle gap until the next step's anchor")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if a.anchor in r["Kernel_Name"]]
    if len(idx) < 2:
        print("anchor not found"); return
    if a.gaps:
        mk, gp = [], []
        for s in range(len(idx) - 1):
            seg = rows[idx[s]:idx[s + 1]]
            start = int(rows[idx[s]]["Start_Timestamp"])
            end = max(int(r["End_Timestamp"]) for r in seg)
            last = max(seg, key=lambda r: int(r["End_Timestamp"]))
            nxt = int(rows[idx[s + 1]]["Start_Timestamp"])
            mk.append((end - start) / 1e3)
            gp.append((nxt - end) / 1e3)
            if s >= len(idx) - 1 - a.steps:
                print(f"step {s}: makespan {mk[-1]:8.1f} us, last {short(last['Kernel_Name']):24s} "
                      f"gap to next {gp[-1]:6.1f} us")
        k = len(mk) // 2   # the later half (warm)
        print(f"later half: makespan median {sorted(mk[k:])[len(mk[k:]) // 2]:.1f} us, "
              f"gap median {sorted(gp[k:])[len(gp[k:]) // 2]:.1f} us")
        return
    for s in range(max(0, len(idx) - 1 - a.steps), len(idx) - 1):
        lo, hi = idx[s], idx[s + 1]
        # the step also holds the dispatches just before the anchor (estimator, memset)
        start = int(rows[lo]["Start_Timestamp"])
        seg = rows[lo:hi]
        end = max(int(r["End_Timestamp"]) for r in seg)
        print(f"-- step {s}: makespan {(end - start) / 1e6:.3f} ms (from {short(rows[lo]['Kernel_Name'])})")
        for r in seg:
            t0 = (int(r["Start_Timestamp"]) - start) / 1e6
            t1 = (int(r["End_Timestamp"]) - start) / 1e6
            print(f"   {short(r['Kernel_Name']):26s} grid {r.get('Grid_Size', r.get('Grid_Size_X', '?')):>9s}  "
                  f"{t0:8.3f} -> {t1:8.3f} ms  ({t1 - t0:7.3f})")


if __name__ == "__main__":
    main()
