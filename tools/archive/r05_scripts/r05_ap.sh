#!/bin/bash
# Round 5 call ap: more, shorter tiles per wave (MHQ_DEC_XROUNDS 1, 2), A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05ap}
mkdir -p "$OUT"
timeout -k 10 900 python3 tools/abmulti.py --kernel decode --reps 3 --configs northstar,config2,config3,config4 \
  --libs base=minhq_amd/libmhq_huff.so,xr1=build/v/lib_xr1.so,xr2=build/v/lib_xr2.so --check xr1,xr2 > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt" | grep -v SAME
grep -c SAME "$OUT/ab.txt"
