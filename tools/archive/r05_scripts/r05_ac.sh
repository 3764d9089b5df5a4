#!/bin/bash
# Round 5 call ac: every step resolving long codes (MHQ_DEC_LONGALL), with 3- and 2-step groups, A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05ac}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel decode --configs northstar,config2,config3,config2print,config4 --reps 4 \
  --libs base=minhq_amd/libmhq_huff.so,longall=build/v/lib_longall.so,longall2=build/v/lib_longall2.so,pair2=build/v/lib_pair2.so \
  --check longall,longall2 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v "amdgpu.ids" "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
