#!/bin/bash
# Round 5 call x: 3-step groups (pair + step) against 2-step groups (one pair), more reps.
set -o pipefail
OUT=${1:-gpurun_out/r05x}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3 --reps 6 \
  --libs base=minhq_amd/libmhq_huff.so,pair2=build/v/lib_pair2.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids\|check" "$OUT/ab.txt"
