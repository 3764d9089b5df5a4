#!/bin/bash
# Round 5 call bg: the packed encode's shape bound, 19,200 (base: a 37.5-B mean) against 19,712 B a range (38.5 B), on batches of 37.5-38.5-B means.
set -o pipefail
OUT=${1:-gpurun_out/r05bg}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs uniform:30:46,uniform:8:68,uniform:20:56,config2 \
  --libs b19200=minhq_amd/libmhq_huff.so,b19712=build/v/lib_t19712.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
