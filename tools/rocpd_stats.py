"""Per-kernel duration statistics from a rocprofv3 SQLite output (rocpd
`*_results.db`), as `--stats` would give, but split by launch geometry so the
bench's configs (different grids) come out as separate rows.

  python tools/rocpd_stats.py gpurun_out/prof/run_results.db [out.csv]
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def short(name: str) -> str:
    s = name.replace("(anonymous namespace)::", "")
    for pre in ("void ", "mhq::dev::", "mhq::"):
        s = s.replace(pre, "")
    return s.split("(")[0]


def main():
    db = sqlite3.connect(sys.argv[1])
    rows = db.execute("select name, grid_x, workgroup_x, lds_size, vgpr_count, duration from kernels").fetchall()
    groups = defaultdict(list)
    meta = {}
    for name, gx, wx, lds, vgpr, dur in rows:
        k = (short(name), gx // max(wx, 1))
        groups[k].append(dur)
        meta[k] = (wx, lds, vgpr)
    out = []
    for (name, wgs), d in groups.items():
        d.sort()
        wx, lds, vgpr = meta[(name, wgs)]
        out.append({"kernel": name, "workgroups": wgs, "threads": wx, "lds": lds, "vgpr": vgpr, "calls": len(d),
                    "avg_us": round(sum(d) / len(d) / 1e3, 3), "median_us": round(d[len(d) // 2] / 1e3, 3),
                    "min_us": round(d[0] / 1e3, 3), "total_ms": round(sum(d) / 1e6, 3)})
    out.sort(key=lambda r: -r["total_ms"])
    w = csv.DictWriter(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout, fieldnames=list(out[0]))
    w.writeheader()
    w.writerows(out)


if __name__ == "__main__":
    main()
