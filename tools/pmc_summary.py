"""Turn two rocprofv3 --pmc runs (FETCH_SIZE, WRITE_SIZE; separate passes because they do
not fit one pass on gfx950) into per-launch HBM bytes per kernel.

gfx950 corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE / WRITE_SIZE are KiB.
FETCH_SIZE reads half the bytes of a WIDE (16 B/lane) coalesced stream; other widths are
uncalibrated.  Calibrated here on the backward kernel, whose HBM reads are 4-B dword loads
of the checkpoint + output cotangents (674 MB algorithmic at the state49 workload): raw
FETCH_SIZE = 661 MB, i.e. no x2 for this access width.  So the raw values are used and the
x2-corrected read figure is recorded beside them.  Writes profiles/pmc_<workload>_<kernel>.json.

    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write state49
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = {"bwd": "ude_bwd_kernel", "fwd": "ude_fwd_kernel", "finalize": "ude_grad_finalize_kernel"}


def per_kernel(d, counter):
    path = glob.glob(os.path.join(d, "*counter_collection.csv"))[0]
    vals = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            for k, pat in KERNELS.items():
                if pat in row["Kernel_Name"]:
                    vals[k].append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, workload = sys.argv[1:4]
    fe = per_kernel(fetch_dir, "FETCH_SIZE")
    wr = per_kernel(write_dir, "WRITE_SIZE")
    out_dir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    for k in KERNELS:
        if not fe.get(k) or not wr.get(k):
            continue
        f_kib = sum(fe[k]) / len(fe[k])
        w_kib = sum(wr[k]) / len(wr[k])
        import subprocess
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True,
                                cwd=os.path.dirname(out_dir)).stdout.strip() or os.environ.get("UDE_COMMIT")
        rec = {"kernel": KERNELS[k], "workload": workload, "launches": [len(fe[k]), len(wr[k])],
               "commit": commit,
               "FETCH_SIZE_KiB_avg": f_kib, "WRITE_SIZE_KiB_avg": w_kib,
               "hbm_bytes_per_launch": (f_kib + w_kib) * 1024.0,
               "hbm_bytes_per_launch_if_fetch_x2": (2.0 * f_kib + w_kib) * 1024.0,
               "correction": "raw FETCH_SIZE + WRITE_SIZE (calibrated: dword-load reads count 1:1, see header)"}
        # the kernel's average duration over the timed calls of the same commit (tools/roofline_trace.py
        # output named by UDE_ROOFLINE_JSON), so the line's traffic and time come from one measured tree
        rj = os.environ.get("UDE_ROOFLINE_JSON")
        if rj and os.path.exists(rj):
            t = json.load(open(rj))
            key = {"bwd": "rocprof_bwd_kernel_ms", "fwd": "rocprof_fwd_ms"}.get(k)
            if key in t:
                rec["kernel_avg_ms"] = t[key]
                rec["kernel_avg_ms_source"] = os.path.basename(rj) + " (kernel trace, timed calls)"
        with open(os.path.join(out_dir, f"pmc_{workload}_{k}.json"), "w") as f:
            json.dump(rec, f, indent=1)
        print(k, json.dumps(rec))


if __name__ == "__main__":
    main()
