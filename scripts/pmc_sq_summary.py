"""Per-kernel averages of the SQ counter passes written by scripts/gpu_pmc_sq.sh, per wave."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if "cmpc" not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    waves = avg.get("SQ_WAVES", 1.0)
    print(k)
    for c in sorted(avg):
        print(f"  {c:24s} {avg[c]:16.0f}   per wave {avg[c] / waves:12.1f}")
