#!/usr/bin/env python3
"""Condense tools/round_profile.sh output into the files committed under profiles/.

    python tools/prof_summary.py gpurun_out/round profiles r01

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats, per kernel: calls,
total/avg/min/max ns), profiles/<tag>_bench.json, and profiles/pmc_traffic.json:
HBM bytes per launch of each codec kernel from FETCH_SIZE / WRITE_SIZE (KB
units; FETCH_SIZE doubled: on gfx950 it counts half the bytes of wide
streaming reads, MI355X_MICROARCH.md "HBM").
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

src, dst, tag = sys.argv[1], sys.argv[2], sys.argv[3]
os.makedirs(dst, exist_ok=True)

KERNELS = {"decode_kernel": "decode_kernel", "encode_kernel<true>": "encode_kernel",
           "encode_kernel<false>": "encode_len_kernel", "encode_len_kernel": "encode_len_kernel",
           "encode_coop_kernel": "encode_coop_kernel",
           "scan_apply_kernel": "scan_apply_kernel",
           "scan_reduce_kernel": "scan_reduce_kernel", "scan_kernel": "scan_kernel",
           "encode_packed_kernel": "encode_packed_kernel"}


def short(name):
    for k, v in KERNELS.items():
        if k in name:
            return v
    return None


stats = glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    with open(os.path.join(dst, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "percent"])
        for r in rows:
            nm = short(r["Name"]) or r["Name"][:60]
            w.writerow([nm, r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["MinNs"], r["MaxNs"],
                        r["Percentage"]])
    print(open(os.path.join(dst, f"{tag}_kernel_stats.csv")).read())

# Launches that overlap no other kernel: bench.py alternates batches over
# streams, so the step's launches share the GPU with their neighbours and
# their spans stretch; the isolated launches (bench.py's per-kernel event runs
# and every single-stream launch) are the ones whose duration the roofline uses.
traces = glob.glob(os.path.join(src, "stats", "**", "*kernel_trace.csv"), recursive=True)
if traces:
    tr = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                 for r in csv.DictReader(open(traces[0]))))
    iso = defaultdict(list)
    allk = defaultdict(list)
    run_end = -1
    for idx, (s0, e0, nm) in enumerate(tr):
        k = short(nm) or nm[:60]
        nxt = tr[idx + 1][0] if idx + 1 < len(tr) else None
        tol = 500  # ns: same-stream back-to-back launches touch (or overlap by a few ns in the trace)
        alone = s0 > run_end - tol and (nxt is None or nxt > e0 - tol)
        run_end = max(run_end, e0)
        allk[k].append(e0 - s0)
        if alone:
            iso[k].append(e0 - s0)
    with open(os.path.join(dst, f"{tag}_kernel_isolated.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "avg_ns", "isolated_calls", "isolated_avg_ns", "isolated_min_ns"])
        for k in sorted(allk, key=lambda x: -sum(allk[x])):
            v, u = allk[k], iso.get(k, [])
            w.writerow([k, len(v), round(sum(v) / len(v), 1), len(u), round(sum(u) / len(u), 1) if u else "",
                        min(u) if u else ""])
    print(open(os.path.join(dst, f"{tag}_kernel_isolated.csv")).read())

bench = os.path.join(src, "bench.json")
if os.path.exists(bench):
    shutil.copy(bench, os.path.join(dst, f"{tag}_bench.json"))

per = defaultdict(dict)
for which, counter in (("pmc_fetch", "FETCH_SIZE"), ("pmc_write", "WRITE_SIZE")):
    vals = defaultdict(list)
    for fn in glob.glob(os.path.join(src, which, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(fn)):
            k = short(r.get("Kernel_Name", ""))
            if k and r["Counter_Name"] == counter:
                vals[k].append(float(r["Counter_Value"]))
    for k, v in vals.items():
        per[k][counter] = sum(v) / len(v)
out = {}
for k, d in per.items():
    if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
        rd = 2 * d["FETCH_SIZE"] * 1024
        wr = d["WRITE_SIZE"] * 1024
        out[k] = {"hbm_bytes_per_launch": int(rd + wr), "read_bytes": int(rd), "write_bytes": int(wr),
                  "fetch_size_kb_raw": d["FETCH_SIZE"], "write_size_kb_raw": d["WRITE_SIZE"],
                  "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, bench.py default; {tag}"}
if out:
    json.dump(out, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))
