"""Print the headline and per-line figures of a bench.py JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("state49", round(d["value"] / 1e6, 2), "M traj*steps/s,", round(d["ms_per_step"], 3), "ms/step, frac",
      round(d["roofline"]["frac"], 3), "bwd", round(d["kernels"]["bwd_ms"], 3), "fwd", round(d["kernels"]["fwd_ms"], 3))
for k, v in d.items():
    if isinstance(v, dict) and k not in ("config", "roofline", "kernels"):
        print(k, {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()
                  if not isinstance(vv, (dict, str))})
        for kk, vv in v.items():
            if isinstance(vv, dict) and kk.startswith("kernel_ms"):
                print("   ", kk, {a: round(b, 4) for a, b in vv.items()})
