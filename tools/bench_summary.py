"""One-line summary of a bench.py JSON line: value, ms/step, roofline, kernels by time."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(f"{d['dtype']:7s} {d['value']:.4g} px/s  {d['ms_per_step']:.3f} ms/step  roof {r.get('kernel')} "
      f"{r.get('kernel_ms_per_step', r.get('avg_launch_ms', 0)):.3f} ms/step x{r.get('launches_per_step', 1):.0f} frac {r.get('frac', 0):.4f}  cpu {d.get('cpu_baseline', {}).get('value')}")
for k, v in sorted(d["kernels"].items(), key=lambda kv: -kv[1]["avg_ms"] * kv[1]["launches_per_step"])[:8]:
    print(f"    {k:20s} {v['avg_ms']:8.3f} ms x {v['launches_per_step']:.0f}")
