#!/bin/bash
# Round 5 call ak: where the long-literal decode form starts to pay (kLongMean 64 / 48 / 40 / 32 encoded bytes), sized.
set -o pipefail
OUT=${1:-gpurun_out/r05ak}
mkdir -p "$OUT"
timeout -k 10 900 python3 tools/abmulti.py --kernel decode --reps 3 --sized \
  --configs uniform:8:100,uniform:16:110,uniform:16:140,uniform:32:160,config4 \
  --libs base=minhq_amd/libmhq_huff.so,lm48=build/v/lib_lm48.so,lm40=build/v/lib_lm40.so,lm32=build/v/lib_lm32.so \
  --check lm48,lm40,lm32 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
