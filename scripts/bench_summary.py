"""One line per workload of a bench.py JSON line (main + other_configs + scaling model)."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])


def line(name, x):
    r = x.get("roofline") or {}
    print(f"{name:10s} {x['value'] / 1e6:8.3f} M QP/s  {x['ms_per_step']:8.4f} ms/step  launch {r.get('avg_launch_ms')}"
          f"  tail {r.get('tail_avg_ms')}  frac {r.get('frac')}  traffic {r.get('traffic')}  status {x.get('status_counts')}")


line("main", d)
for k, v in (d.get("other_configs") or {}).items():
    line(k, v)
sm = d.get("scaling_model")
if sm:
    print("scaling", [(r["gpus"], r.get("speedup"), r.get("t_solve_ms_measured")) for r in sm["rows"]])
    print("scaling step-0 output", [(r["gpus"], r.get("step0_speedup"), r.get("step0_t_solve_ms_measured"))
                                    for r in sm["rows"]])
if d.get("cpu_baseline"):
    print("cpu", d["cpu_baseline"].get("value"))
