#!/bin/bash
# read_strings and the other 8(f) rows: bench_rows.py, then its kernel trace.
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/rows}
mkdir -p "$OUT"
timeout -k 10 300 python3 -W ignore tools/bench_rows.py > "$OUT/rows.json" 2> "$OUT/rows.err" || { tail "$OUT/rows.err"; exit 1; }
cat "$OUT/rows.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats" -o run -- python3 -W ignore tools/bench_rows.py > "$OUT/stats.log" 2>&1 || { tail "$OUT/stats.log"; exit 1; }
f=$(find "$OUT/stats" -name '*kernel_stats.csv' | head -1); head -14 "$f" | cut -c1-150
