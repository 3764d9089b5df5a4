#!/bin/bash
# Round 5 call bj: Zipf batches (config 4) through the decode's long-literal form (MHQ_DEC_LONG_MEAN 16) against the tile kernel, sized calls.
set -o pipefail
OUT=${1:-gpurun_out/r05bj}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --reps 3 --sized --configs config4,zipf:4:128 \
  --libs base=minhq_amd/libmhq_huff.so,lm16=build/v/lib_lm16.so --check lm16 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
