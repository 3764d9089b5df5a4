#!/bin/bash
# Round 5 call bh: means past 37.5 B at four workgroups per CU with 448-literal ranges (sr) against three with 512 (nosr); packed tests.
set -o pipefail
OUT=${1:-gpurun_out/r05bh}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs uniform:24:56,uniform:8:72,uniform:30:46,uniform:8:68,config2 \
  --libs sr=minhq_amd/libmhq_huff.so,nosr=build/v/lib_nosr.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_encode_packed.py > "$OUT/tests.txt" 2>&1 || { tail -30 "$OUT/tests.txt"; exit 1; }
tail -1 "$OUT/tests.txt"
