#!/bin/bash
# Packed encode look-back variants (build/r06y): b0 = 64-bit shuffle sums,
# d1 = DPP sums, d1w4 = DPP + 4 windows, d1s1 = DPP + s_sleep 1; b0b/d1b are
# copies of b0/d1 (the noise between identical builds).  bash tools/r06/ab3.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
for v in d1 d1w4; do
  MHQ_LIB_PATH=build/r06y/lib_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_encode_packed.py \
    -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/tests_$v.txt" 2>&1 || { tail -30 "$OUT/tests_$v.txt"; exit 1; }
  echo "$v: $(tail -1 "$OUT/tests_$v.txt")"
done
L=b0=build/r06y/lib_b0.so,d1=build/r06y/lib_d1.so,d1w4=build/r06y/lib_d1w4.so,d1s1=build/r06y/lib_d1s1.so,b0b=build/r06y/lib_b0b.so,d1b=build/r06y/lib_d1b.so
timeout -k 10 500 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar,config3 --libs $L \
  --reps 7 > "$OUT/ab_lb.txt" 2>&1 || { tail -20 "$OUT/ab_lb.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_lb.txt"
