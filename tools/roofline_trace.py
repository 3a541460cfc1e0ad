"""Recompute the bench line's roofline from a rocprofv3 kernel trace of the SAME command (VERDICT r5
item 5): the time from each timed ude_bwd_kernel's start to its ude_bwd_tail_kernel's end (one
ude_rk4_backward_ex call, what the bench's HIP events bracket), averaged over the last `steps` calls --
the timed region, not the warm-up ones (the stats CSV averages every call, warm-up included).

    python tools/roofline_trace.py <kernel_trace.csv> <bench.json> [commit] > roofline_rocprof.json
"""
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
commit = sys.argv[3] if len(sys.argv) > 3 else None
rows = list(csv.DictReader(open(trace)))
name = lambda r: r.get("Kernel_Name") or r.get("Kernel-Name") or ""
ts = lambda r, k: int(r[k + "_Timestamp"])
bw = [r for r in rows if "ude_bwd_kernel" in name(r)]
tl = [r for r in rows if "ude_bwd_tail_kernel" in name(r)]
fw = [r for r in rows if "ude_fwd_kernel" in name(r)]
b = json.load(open(bench))
K = int(b["steps"])
span = [(ts(t, "End") - ts(s, "Start")) / 1e6 for s, t in zip(bw[-K:], tl[-K:])]
kern = [(ts(s, "End") - ts(s, "Start")) / 1e6 for s in bw[-K:]]
fwd = [(ts(s, "End") - ts(s, "Start")) / 1e6 for s in fw[-K:]]
ms = sum(span) / len(span)
flop = b["roofline"]["algorithmic_flop_per_launch"]
peak = b["roofline"]["peak"]
out = {"source": {"trace": trace, "bench": bench, "commit": commit},
       "timed_calls": len(span),
       "rocprof_bwd_call_ms": ms, "rocprof_bwd_kernel_ms": sum(kern) / len(kern),
       "rocprof_tail_ms": ms - sum(kern) / len(kern), "rocprof_fwd_ms": sum(fwd) / len(fwd),
       "rocprof_frac": flop / (ms * 1e-3) / 1e12 / peak,
       "bench_avg_launch_ms": b["roofline"]["avg_launch_ms"], "bench_frac": b["roofline"]["frac"]}
out["frac_rel_diff"] = abs(out["bench_frac"] - out["rocprof_frac"]) / out["rocprof_frac"]
print(json.dumps(out, indent=1))
