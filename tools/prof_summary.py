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
           "scan_apply_kernel": "scan_apply_kernel",
           "scan_reduce_kernel": "scan_reduce_kernel", "scan_kernel": "scan_kernel"}


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
