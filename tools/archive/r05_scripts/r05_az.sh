#!/bin/bash
# Round 5 call az: packed encode look-back back-off (s_sleep 0 / 1 / 2 base / 4) and the length sort off, A/B.
set -o pipefail
OUT=${1:-gpurun_out/r05az}
mkdir -p "$OUT"
timeout -k 10 600 python3 tools/abmulti.py --kernel packed --reps 3 --configs config2,northstar,config3 \
  --libs base=minhq_amd/libmhq_huff.so,sl0=build/v/lib_sl0.so,sl1=build/v/lib_sl1.so,sl4=build/v/lib_sl4.so,nosort=build/v/lib_nosort.so > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab.txt"
