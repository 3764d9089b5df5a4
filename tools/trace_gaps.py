#!/usr/bin/env python3
"""Per-launch durations and the idle gap before each launch, from a
rocprofv3 --kernel-trace CSV: python3 tools/trace_gaps.py <kernel_trace.csv> [last N]."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 20
prev = None
out = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("mhq::(anonymous namespace)::", "").replace("void ", "")
    name = name.split("(")[0].split("<")[0]
    out.append((name, (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0))
    prev = e
for name, dur, gap in out[-last:]:
    print(f"{name:28s} dur={dur:8.2f} us  gap_before={gap:7.2f} us")
