#!/usr/bin/env python3
"""Summarise tools/prof_pmc.sh output: per-kernel mean counter values per dispatch."""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
vals = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            k = r.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
            if filt not in k:
                continue
            vals[k.split("(")[0][-40:]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:24s} mean/dispatch {sum(v)/len(v):16.1f}  (n={len(v)})")
