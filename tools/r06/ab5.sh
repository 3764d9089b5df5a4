#!/bin/bash
# Packed encode: staged ranges whose codes overflow the output staging in halves too (new, the in-tree
# library) against per-literal global sizing and encoding (old); the packed
# tests on the new library first.  bash tools/r06/ab4.sh OUT
set -o pipefail
OUT=${1:?}; mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_encode_packed.py -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/tests_packed.txt" 2>&1 || { tail -30 "$OUT/tests_packed.txt"; exit 1; }
tail -1 "$OUT/tests_packed.txt"
L=old=build/r06q/lib_old.so,new=build/r06q/lib_new.so,oldb=build/r06q/lib_oldb.so,newb=build/r06q/lib_newb.so
timeout -k 10 500 python3 -u tools/abmulti.py --kernel packed --configs config2,northstar,config2print,clustered:32:60 \
  --libs $L --reps 5 > "$OUT/ab_outhalves.txt" 2>&1 || { tail -20 "$OUT/ab_halves.txt"; exit 1; }
grep -v amdgpu.ids "$OUT/ab_outhalves.txt"
