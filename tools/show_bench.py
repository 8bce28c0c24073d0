"""Print the headline of a bench.py JSON line (value + per-kernel ms per generation)."""
import json
import sys

d = json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bench.json"))
k = d.get("kernels_avg_ms_per_generation", {})
print("VALUE %.1fM evals/s" % (d["value"] / 1e6),
      {a: (round(b, 4) if isinstance(b, float) else b) for a, b in k.items()})
if "roofline" in d:
    r = d["roofline"]
    print("roofline", r["kernel"], "%.1f %s frac %.3f" % (r["achieved"], r["unit"], r["frac"]))
