#!/bin/bash
# Round 5 call bb: packed encode 4 (base) vs 3 workgroups per CU on skewed and near-40-B-mean batches (staging overflow at 20 KB).
set -o pipefail
OUT=${1:-gpurun_out/r05bb}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs zipf:4:96,zipf:4:128,uniform:24:56,uniform:30:46,uniform:36:44 \
  --libs pk4=minhq_amd/libmhq_huff.so,pk3=build/v/lib_pk3.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
