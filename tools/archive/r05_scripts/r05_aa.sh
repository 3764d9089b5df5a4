#!/bin/bash
# Round 5 call aa: decode loop priority by wave age (MHQ_DEC_AGEPRIO) A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05aa}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print --reps 4 \
  --libs base=minhq_amd/libmhq_huff.so,age1=build/v/lib_age1.so,age2=build/v/lib_age2.so \
  --check age1,age2 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
